// What limits the one-workgroup-per-symbol streaming structure of the enrich
// kernel? Variants of a no-arithmetic kernel with the enrich traffic mix
// (5 fp64 inputs read, 14 written, [S][ld] rows, 1024-candle tiles per WG):
// allocation stagger between arrays, padded row pitch, swizzled symbol order,
// workgroup size, register prefetch of the next tile.
// Build: hipcc -O3 --offload-arch=gfx950 tools/row_ceiling.hip -o tools/row_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int NIN = 5, NOUT = 14, K = 4;

struct Args {
  const double* in[NIN];
  double* out[NOUT];
  long S, T, ld;
  int swz;
};

template <int NT, bool PREFETCH>
__global__ __launch_bounds__(NT) void row_tiles(Args a) {
  extern __shared__ double occupancy_limiter[];   // dynamic LDS only limits WGs/CU
  if (a.S < 0) occupancy_limiter[threadIdx.x] = 0.0;
  long sym = blockIdx.x;
  if (a.swz) sym = (sym * 7919) % a.S;   // scatter concurrently running rows
  const long base = sym * a.ld;
  constexpr int TILE = NT * K;
  dbl2 nx[NIN][2];
  long tb = threadIdx.x * K;
  if (PREFETCH && tb < a.T)
    for (int f = 0; f < NIN; ++f) {
      const dbl2* p = reinterpret_cast<const dbl2*>(a.in[f] + base + tb);
      nx[f][0] = p[0];
      nx[f][1] = p[1];
    }
  for (; tb < a.T; tb += TILE) {
    dbl2 cu[NIN][2];
    for (int f = 0; f < NIN; ++f) {
      if (PREFETCH) {
        cu[f][0] = nx[f][0];
        cu[f][1] = nx[f][1];
      } else {
        const dbl2* p = reinterpret_cast<const dbl2*>(a.in[f] + base + tb);
        cu[f][0] = p[0];
        cu[f][1] = p[1];
      }
    }
    if (PREFETCH && tb + TILE < a.T)
      for (int f = 0; f < NIN; ++f) {
        const dbl2* p = reinterpret_cast<const dbl2*>(a.in[f] + base + tb + TILE);
        nx[f][0] = p[0];
        nx[f][1] = p[1];
      }
    dbl2 acc0 = {0, 0}, acc1 = {0, 0};
    for (int f = 0; f < NIN; ++f) {
      acc0 += cu[f][0];
      acc1 += cu[f][1];
    }
    for (int o = 0; o < NOUT; ++o) {
      dbl2* q = reinterpret_cast<dbl2*>(a.out[o] + base + tb);
      q[0] = acc0 + (double)o;
      q[1] = acc1;
    }
  }
}

// register prefetch two tiles ahead: the loop is unrolled by two so the two
// buffers alternate roles without register moves (a move would wait for the
// load in flight)
__device__ __forceinline__ void load_tile2(const Args& a, long base, long tb, dbl2 (&r)[NIN][2]) {
  if (tb < a.T)
    for (int f = 0; f < NIN; ++f) {
      const dbl2* p = reinterpret_cast<const dbl2*>(a.in[f] + base + tb);
      r[f][0] = p[0];
      r[f][1] = p[1];
    }
}
__device__ __forceinline__ void emit_tile(const Args& a, long base, long tb, const dbl2 (&cu)[NIN][2]) {
  dbl2 acc0 = {0, 0}, acc1 = {0, 0};
  for (int f = 0; f < NIN; ++f) {
    acc0 += cu[f][0];
    acc1 += cu[f][1];
  }
  for (int o = 0; o < NOUT; ++o) {
    dbl2* q = reinterpret_cast<dbl2*>(a.out[o] + base + tb);
    q[0] = acc0 + (double)o;
    q[1] = acc1;
  }
}
__global__ __launch_bounds__(256) void row_tiles_pf2(Args a) {
  extern __shared__ double occupancy_limiter[];
  if (a.S < 0) occupancy_limiter[threadIdx.x] = 0.0;
  const long base = (long)blockIdx.x * a.ld;
  constexpr int TILE = 256 * K;
  dbl2 A[NIN][2], B[NIN][2];
  long tb = threadIdx.x * K;
  load_tile2(a, base, tb, A);
  load_tile2(a, base, tb + TILE, B);
  for (; tb < a.T; tb += 2 * TILE) {
    emit_tile(a, base, tb, A);
    load_tile2(a, base, tb + 2 * TILE, A);
    if (tb + TILE < a.T) {
      emit_tile(a, base, tb + TILE, B);
      load_tile2(a, base, tb + 3 * TILE, B);
    }
  }
}

int main(int argc, char** argv) {
  const long S = 12500, T = 10000;
  const int reps = 10;
  struct V { const char* name; long pad; long stagger; int swz; int nt; int pf; int lds; };
  const V vs[] = {
      {"pf1_3wg", 0, 0, 0, 256, 1, 52000},  {"pf2_2wg", 0, 0, 0, 256, 2, 78000},
      {"pf2_3wg", 0, 0, 0, 256, 2, 52000},  {"pf1_2wg", 0, 0, 0, 256, 1, 78000},
      {"pf1_3wg_b", 0, 0, 0, 256, 1, 52000}, {"pf2_2wg_b", 0, 0, 0, 256, 2, 78000},
      {"pf2_3wg_b", 0, 0, 0, 256, 2, 52000}, {"pf1_4wg", 0, 0, 0, 256, 1, 39000},
      {"pf1_5wg", 0, 0, 0, 256, 1, 31000},  {"pf1_6wg", 0, 0, 0, 256, 1, 26000},
      {"pf1_8wg", 0, 0, 0, 256, 1, 19000},  {"pf2_4wg", 0, 0, 0, 256, 2, 39000},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const V& v : vs) {
    const long ld = T + v.pad;
    const size_t arr = (size_t)S * ld * sizeof(double);
    const size_t slot = arr + v.stagger;   // one allocation, arrays staggered
    char* buf;
    CK(hipMalloc(&buf, slot * (NIN + NOUT) + 4096));
    CK(hipMemset(buf, 0, slot * (NIN + NOUT)));
    Args a;
    for (int f = 0; f < NIN; ++f) a.in[f] = (const double*)(buf + slot * f);
    for (int o = 0; o < NOUT; ++o) a.out[o] = (double*)(buf + slot * (NIN + o));
    a.S = S;
    a.T = T;
    a.ld = ld;
    a.swz = v.swz;
    for (int r = 0; r < reps + 2; ++r) {
      if (r == 2) CK(hipEventRecord(e0));
      if (v.pf == 2) row_tiles_pf2<<<S, 256, v.lds>>>(a);
      else if (v.pf) row_tiles<256, true><<<S, 256, v.lds>>>(a);
      else row_tiles<256, false><<<S, 256, v.lds>>>(a);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double gb = (double)S * T * 8.0 * (NIN + NOUT) / 1e9;
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", v.name, ms, gb / ms * 1e3);
    CK(hipFree(buf));
  }
  return 0;
}
