// Does a tile-major workgroup order (consecutive workgroups = consecutive
// 1024-candle tiles of one symbol row, each tile independent with a 128-candle
// halo re-read) stream the enrich traffic mix (5 fp64 inputs, 14 outputs)
// faster than the row walk (one workgroup walks a whole row)? Same occupancy
// limiter as the enrich kernel (dynamic LDS). No arithmetic.
// Build: hipcc -O3 --offload-arch=gfx950 tools/tile_ceiling.hip -o tools/tile_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int NIN = 5, NOUT = 14, K = 4, NT = 256, TILE = NT * K, HALO = 128;

struct Args {
  const double* in[NIN];
  double* out[NOUT];
  long S, T, ld;
};

// one workgroup per (symbol, tile); tile index fastest
__global__ __launch_bounds__(NT) void tile_major(Args a, int ntiles, int halo_inputs) {
  extern __shared__ double lim[];
  if (a.S < 0) lim[threadIdx.x] = 0.0;
  const long sym = blockIdx.x / ntiles;
  const long tb = (long)(blockIdx.x % ntiles) * TILE;
  const long base = sym * a.ld;
  double hsum = 0.0;
  // halo: the 128 candles before the tile for the first `halo_inputs` inputs
  if (threadIdx.x < HALO && tb > 0)
    for (int f = 0; f < halo_inputs; ++f) hsum += a.in[f][base + tb - HALO + threadIdx.x];
  const long t = tb + threadIdx.x * K;
  if (t >= a.T) return;
  dbl2 cu[NIN][2];
  for (int f = 0; f < NIN; ++f) {
    const dbl2* p = reinterpret_cast<const dbl2*>(a.in[f] + base + t);
    cu[f][0] = p[0];
    cu[f][1] = p[1];
  }
  dbl2 acc0 = {hsum, 0}, acc1 = {0, 0};
  for (int f = 0; f < NIN; ++f) {
    acc0 += cu[f][0];
    acc1 += cu[f][1];
  }
  for (int o = 0; o < NOUT; ++o) {
    dbl2* q = reinterpret_cast<dbl2*>(a.out[o] + base + t);
    q[0] = acc0 + (double)o;
    q[1] = acc1;
  }
}

// the enrich kernel's order: one workgroup walks a whole row
__global__ __launch_bounds__(NT) void row_walk(Args a) {
  extern __shared__ double lim[];
  if (a.S < 0) lim[threadIdx.x] = 0.0;
  const long base = (long)blockIdx.x * a.ld;
  for (long t = threadIdx.x * K; t < a.T; t += TILE) {
    dbl2 cu[NIN][2];
    for (int f = 0; f < NIN; ++f) {
      const dbl2* p = reinterpret_cast<const dbl2*>(a.in[f] + base + t);
      cu[f][0] = p[0];
      cu[f][1] = p[1];
    }
    dbl2 acc0 = {0, 0}, acc1 = {0, 0};
    for (int f = 0; f < NIN; ++f) {
      acc0 += cu[f][0];
      acc1 += cu[f][1];
    }
    for (int o = 0; o < NOUT; ++o) {
      dbl2* q = reinterpret_cast<dbl2*>(a.out[o] + base + t);
      q[0] = acc0 + (double)o;
      q[1] = acc1;
    }
  }
}

int main() {
  const long S = 12500, T = 10000, ld = T;
  const int reps = 10;
  const size_t arr = (size_t)S * ld * sizeof(double);
  char* buf;
  CK(hipMalloc(&buf, arr * (NIN + NOUT)));
  CK(hipMemset(buf, 0, arr * (NIN + NOUT)));
  Args a;
  for (int f = 0; f < NIN; ++f) a.in[f] = (const double*)(buf + arr * f);
  for (int o = 0; o < NOUT; ++o) a.out[o] = (double*)(buf + arr * (NIN + o));
  a.S = S;
  a.T = T;
  a.ld = ld;
  const int ntiles = (int)((T + TILE - 1) / TILE);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V { const char* name; int mode; int lds; int halo; };
  const V vs[] = {{"row_3wg", 0, 52000, 0},  {"tile_3wg", 1, 52000, 0}, {"tile_3wg_halo2", 1, 52000, 2},
                  {"tile_4wg_halo2", 1, 39000, 2}, {"row_4wg", 0, 39000, 0}, {"tile_6wg_halo2", 1, 26000, 2},
                  {"row_3wg_b", 0, 52000, 0}, {"tile_3wg_halo2_b", 1, 52000, 2}};
  for (const V& v : vs) {
    for (int r = 0; r < reps + 2; ++r) {
      if (r == 2) CK(hipEventRecord(e0));
      if (v.mode) tile_major<<<(unsigned)(S * ntiles), NT, v.lds>>>(a, ntiles, v.halo);
      else row_walk<<<(unsigned)S, NT, v.lds>>>(a);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double gb = (double)S * T * 8.0 * (NIN + NOUT) / 1e9;
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", v.name, ms, gb / ms * 1e3);
  }
  CK(hipFree(buf));
  return 0;
}
