// Streaming ceiling for the enrich kernel's HBM traffic mix on this GPU:
// 5 fp64 inputs read once + 14 fp64 outputs written once per candle
// ([S][T] row-major, same layout and workgroup->symbol mapping as
// enrich_kernel), with no arithmetic. The achieved GB/s is the practical
// roofline the enrich kernel's fraction should be read against.
// Build: hipcc -O3 --offload-arch=gfx950 tools/stream_ceiling.hip -o tools/stream_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int NIN = 5, NOUT = 14, K = 4, NT = 256, TILE = NT * K;

struct Args {
  const double* in[NIN];
  double* out[NOUT];
  long S, T;
};

// one workgroup per row, walk the row in 1024-candle tiles (enrich's shape)
template <bool NTS>
__global__ __launch_bounds__(NT) void row_tiles(Args a, int nin, int nout) {
  const long base = (long)blockIdx.x * a.T;
  for (long tb = threadIdx.x * K; tb < a.T; tb += TILE) {
    double acc[K] = {0, 0, 0, 0};
#pragma unroll
    for (int f = 0; f < NIN; ++f) {
      if (f >= nin) break;
      const dbl2* p = reinterpret_cast<const dbl2*>(a.in[f] + base + tb);
      dbl2 x0 = p[0], x1 = p[1];
      acc[0] += x0.x; acc[1] += x0.y; acc[2] += x1.x; acc[3] += x1.y;
    }
    for (int o = 0; o < nout; ++o) {
      dbl2* q = reinterpret_cast<dbl2*>(a.out[o] + base + tb);
      if (NTS) {
        __builtin_nontemporal_store(dbl2{acc[0] + o, acc[1]}, q);
        __builtin_nontemporal_store(dbl2{acc[2], acc[3] + o}, q + 1);
      } else {
        q[0] = dbl2{acc[0] + o, acc[1]};
        q[1] = dbl2{acc[2], acc[3] + o};
      }
    }
    if (nout == 0 && acc[0] == 12345.0) a.out[0][base + tb] = acc[1] + acc[2] + acc[3];
  }
}

// flat grid-stride stream over all elements (no row structure)
template <bool NTS>
__global__ __launch_bounds__(NT) void flat(Args a, long n, int nin, int nout) {
  for (long i = ((long)blockIdx.x * NT + threadIdx.x) * 2; i < n; i += (long)gridDim.x * NT * 2) {
    dbl2 acc = {0, 0};
#pragma unroll
    for (int f = 0; f < NIN; ++f) { if (f >= nin) break; acc += *reinterpret_cast<const dbl2*>(a.in[f] + i); }
    for (int o = 0; o < nout; ++o) {
      if (NTS) __builtin_nontemporal_store(acc, reinterpret_cast<dbl2*>(a.out[o] + i));
      else *reinterpret_cast<dbl2*>(a.out[o] + i) = acc;
    }
    if (nout == 0 && acc.x == 12345.0) a.out[0][i] = acc.y;
  }
}

int main(int argc, char** argv) {
  long S = argc > 1 ? atol(argv[1]) : 12500, T = argc > 2 ? atol(argv[2]) : 10000;
  Args a;
  a.S = S; a.T = T;
  const size_t bytes = (size_t)S * T * sizeof(double);
  for (int f = 0; f < NIN; ++f) { double* p; CK(hipMalloc(&p, bytes)); CK(hipMemset(p, 0, bytes)); a.in[f] = p; }
  for (int o = 0; o < NOUT; ++o) CK(hipMalloc(&a.out[o], bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int reps = 10;
  struct V { int kind, nin, nout, nts, wgpcu; };
  const V vs[] = {{0, 5, 14, 1, 0}, {0, 5, 14, 0, 0}, {0, 5, 0, 1, 0},
                  {1, 5, 14, 1, 8}, {1, 5, 14, 0, 8}, {1, 5, 14, 1, 32}, {1, 5, 0, 1, 16},
                  {1, 0, 14, 1, 16}, {1, 0, 14, 0, 16}, {1, 1, 1, 1, 16}, {1, 1, 1, 0, 16},
                  {1, 0, 1, 1, 16}, {1, 1, 0, 1, 16}, {1, 5, 5, 1, 16}};
  for (const V& v : vs) {
    for (int r = 0; r < reps + 2; ++r) {
      if (r == 2) CK(hipEventRecord(e0));
      if (v.kind == 0) {
        if (v.nts) row_tiles<true><<<S, NT>>>(a, v.nin, v.nout);
        else row_tiles<false><<<S, NT>>>(a, v.nin, v.nout);
      } else {
        if (v.nts) flat<true><<<ncu * v.wgpcu, NT>>>(a, S * T, v.nin, v.nout);
        else flat<false><<<ncu * v.wgpcu, NT>>>(a, S * T, v.nin, v.nout);
      }
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double gb = (double)S * T * 8.0 * (v.nin + v.nout) / 1e9;
    printf("{\"kernel\": \"%s\", \"reads\": %d, \"writes\": %d, \"nt\": %d, \"wg_per_cu\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
           v.kind == 0 ? "row_tiles" : "flat", v.nin, v.nout, v.nts, v.wgpcu, ms, gb / ms * 1e3);
  }
  return 0;
}
