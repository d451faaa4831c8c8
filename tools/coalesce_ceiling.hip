// Does the per-instruction coverage of the enrich kernel's accesses matter?
// The kernel gives each lane 4 consecutive candles (32 B per field) and moves
// them with two 16-byte instructions: each instruction covers every other
// 16 bytes of the wave's 2 KiB (half of each 128-byte line it touches).
// "split" instead gives lane L candles {2L, 2L+1} and {128 + 2L, 129 + 2L} of
// the wave's 256, so each instruction covers one contiguous KiB. Same traffic
// mix as the kernel (5 fp64 rows read, 14 written per symbol, 1024-candle
// tiles per 256-thread workgroup, next tile prefetched in registers),
// occupancy pinned with dynamic LDS.
// Build: hipcc -O3 --offload-arch=gfx950 tools/coalesce_ceiling.hip -o tools/coalesce_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int NIN = 5, NOUT = 14, NT = 256, TILE = 1024;

struct Args {
  const double* in[NIN];
  double* out[NOUT];
  long S, T, ld;
};

// offsets (in candles, within the tile) of a lane's two 16-byte pieces
template <bool SPLIT>
__device__ __forceinline__ void offs(int tid, int& a, int& b) {
  if (SPLIT) {
    const int w = tid >> 6, l = tid & 63;
    a = w * 256 + 2 * l;
    b = a + 128;
  } else {
    a = 4 * tid;
    b = a + 2;
  }
}

template <bool SPLIT, bool NTS>
__global__ __launch_bounds__(NT) void walk(Args a) {
  extern __shared__ double occupancy_limiter[];
  if (a.S < 0) occupancy_limiter[threadIdx.x] = 0.0;
  const long base = (long)blockIdx.x * a.ld;
  int oa, ob;
  offs<SPLIT>(threadIdx.x, oa, ob);
  dbl2 nx[NIN][2];
  for (int f = 0; f < NIN; ++f) {
    nx[f][0] = *reinterpret_cast<const dbl2*>(a.in[f] + base + oa);
    nx[f][1] = *reinterpret_cast<const dbl2*>(a.in[f] + base + ob);
  }
  for (long t0 = 0; t0 < a.T; t0 += TILE) {
    dbl2 cu[NIN][2];
    for (int f = 0; f < NIN; ++f) {
      cu[f][0] = nx[f][0];
      cu[f][1] = nx[f][1];
    }
    if (t0 + TILE < a.T)
      for (int f = 0; f < NIN; ++f) {
        nx[f][0] = *reinterpret_cast<const dbl2*>(a.in[f] + base + t0 + TILE + oa);
        nx[f][1] = *reinterpret_cast<const dbl2*>(a.in[f] + base + t0 + TILE + ob);
      }
    dbl2 s0 = {0, 0}, s1 = {0, 0};
    for (int f = 0; f < NIN; ++f) {
      s0 += cu[f][0];
      s1 += cu[f][1];
    }
    for (int o = 0; o < NOUT; ++o) {
      dbl2* q0 = reinterpret_cast<dbl2*>(a.out[o] + base + t0 + oa);
      dbl2* q1 = reinterpret_cast<dbl2*>(a.out[o] + base + t0 + ob);
      const dbl2 v0 = s0 + (double)o, v1 = s1;
      if (NTS) {
        __builtin_nontemporal_store(v0, q0);
        __builtin_nontemporal_store(v1, q1);
      } else {
        *q0 = v0;
        *q1 = v1;
      }
    }
  }
}

int main(int argc, char** argv) {
  const long S = argc > 1 ? atol(argv[1]) : 12500, T = 10240;   // whole tiles: the probe has no tail path
  const int reps = 10;
  struct V { const char* name; int split; int nts; int lds; };
  const V vs[] = {
      {"half_3wg", 0, 0, 52000}, {"split_3wg", 1, 0, 52000}, {"half_nt_3wg", 0, 1, 52000},
      {"split_nt_3wg", 1, 1, 52000}, {"half_nt_4wg", 0, 1, 39000}, {"split_nt_4wg", 1, 1, 39000},
      {"half_nt_3wg_b", 0, 1, 52000}, {"split_nt_3wg_b", 1, 1, 52000},
  };
  const size_t arr = (size_t)S * T * sizeof(double);
  char* buf;
  CK(hipMalloc(&buf, arr * (NIN + NOUT)));
  CK(hipMemset(buf, 0, arr * (NIN + NOUT)));
  Args a;
  for (int f = 0; f < NIN; ++f) a.in[f] = (const double*)(buf + arr * f);
  for (int o = 0; o < NOUT; ++o) a.out[o] = (double*)(buf + arr * (NIN + o));
  a.S = S;
  a.T = T;
  a.ld = T;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const V& v : vs) {
    for (int r = 0; r < reps + 2; ++r) {
      if (r == 2) CK(hipEventRecord(e0));
      if (v.split && v.nts) walk<true, true><<<S, NT, v.lds>>>(a);
      else if (v.split) walk<true, false><<<S, NT, v.lds>>>(a);
      else if (v.nts) walk<false, true><<<S, NT, v.lds>>>(a);
      else walk<false, false><<<S, NT, v.lds>>>(a);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double gb = (double)S * T * 8.0 * (NIN + NOUT) / 1e9;
    printf("{\"variant\": \"%s\", \"S\": %ld, \"ms\": %.4f, \"GBps\": %.1f}\n", v.name, S, ms, gb / ms * 1e3);
  }
  CK(hipFree(buf));
  return 0;
}
