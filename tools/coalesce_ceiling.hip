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

// one 16-byte piece per lane and field (2 candles), tiles of 2 * NT2 candles:
// the coalesced pattern at a smaller tile (K = 2) or a larger workgroup
template <int NT2>
__global__ __launch_bounds__(NT2) void walk2(Args a) {
  extern __shared__ double occupancy_limiter[];
  if (a.S < 0) occupancy_limiter[threadIdx.x] = 0.0;
  constexpr int TL = 2 * NT2;
  const long base = (long)blockIdx.x * a.ld;
  const int oa = 2 * threadIdx.x;
  dbl2 nx[NIN];
  for (int f = 0; f < NIN; ++f) nx[f] = *reinterpret_cast<const dbl2*>(a.in[f] + base + oa);
  for (long t0 = 0; t0 < a.T; t0 += TL) {
    dbl2 cu[NIN];
    for (int f = 0; f < NIN; ++f) cu[f] = nx[f];
    if (t0 + TL < a.T)
      for (int f = 0; f < NIN; ++f) nx[f] = *reinterpret_cast<const dbl2*>(a.in[f] + base + t0 + TL + oa);
    dbl2 s0 = {0, 0};
    for (int f = 0; f < NIN; ++f) s0 += cu[f];
    for (int o = 0; o < NOUT; ++o)
      __builtin_nontemporal_store(s0 + (double)o, reinterpret_cast<dbl2*>(a.out[o] + base + t0 + oa));
  }
}

// mixed patterns: loads (LSPLIT) and the first NHALF output rows in one
// layout, the remaining output rows split
template <bool LSPLIT, int NHALF>
__global__ __launch_bounds__(NT) void walk_mix(Args a) {
  extern __shared__ double occupancy_limiter[];
  if (a.S < 0) occupancy_limiter[threadIdx.x] = 0.0;
  const long base = (long)blockIdx.x * a.ld;
  int la, lb, ha, hb, sa, sb;
  offs<LSPLIT>(threadIdx.x, la, lb);
  offs<false>(threadIdx.x, ha, hb);
  offs<true>(threadIdx.x, sa, sb);
  dbl2 nx[NIN][2];
  for (int f = 0; f < NIN; ++f) {
    nx[f][0] = *reinterpret_cast<const dbl2*>(a.in[f] + base + la);
    nx[f][1] = *reinterpret_cast<const dbl2*>(a.in[f] + base + lb);
  }
  for (long t0 = 0; t0 < a.T; t0 += TILE) {
    dbl2 cu[NIN][2];
    for (int f = 0; f < NIN; ++f) {
      cu[f][0] = nx[f][0];
      cu[f][1] = nx[f][1];
    }
    if (t0 + TILE < a.T)
      for (int f = 0; f < NIN; ++f) {
        nx[f][0] = *reinterpret_cast<const dbl2*>(a.in[f] + base + t0 + TILE + la);
        nx[f][1] = *reinterpret_cast<const dbl2*>(a.in[f] + base + t0 + TILE + lb);
      }
    dbl2 s0 = {0, 0}, s1 = {0, 0};
    for (int f = 0; f < NIN; ++f) {
      s0 += cu[f][0];
      s1 += cu[f][1];
    }
    for (int o = 0; o < NOUT; ++o) {
      const int oa = o < NHALF ? ha : sa, ob = o < NHALF ? hb : sb;
      __builtin_nontemporal_store(s0 + (double)o, reinterpret_cast<dbl2*>(a.out[o] + base + t0 + oa));
      __builtin_nontemporal_store(s1, reinterpret_cast<dbl2*>(a.out[o] + base + t0 + ob));
    }
  }
}

// the kernel's layout (lane = 4 consecutive candles) with the outputs
// redistributed before the stores: v_permlane32_swap pairs lane a's candles
// {4a, 4a+1} (lanes < 32) with lane a's {4a+2, 4a+3} moved to lane a + 32, so
// one 16-byte store instruction covers candles [0, 128) of the wave's slice
// in a lane-permuted order (PERM), or additionally a ds_bpermute puts them in
// lane order (BPERM: lane L = 2a + b pulls lane a + 32 b).
__device__ __forceinline__ void swap32(dbl2& A, dbl2& B) {
  union U { dbl2 d; unsigned u[4]; } a, b;
  a.d = A;
  b.d = B;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    auto r = __builtin_amdgcn_permlane32_swap(a.u[i], b.u[i], false, false);
    a.u[i] = r[0];
    b.u[i] = r[1];
  }
  A = a.d;
  B = b.d;
}
__device__ __forceinline__ dbl2 pull(dbl2 X, int addr) {
  union U { dbl2 d; int u[4]; } x;
  x.d = X;
#pragma unroll
  for (int i = 0; i < 4; ++i) x.u[i] = __builtin_amdgcn_ds_bpermute(addr, x.u[i]);
  return x.d;
}
template <bool BPERM>
__global__ __launch_bounds__(NT) void walk_swap(Args a) {
  extern __shared__ double occupancy_limiter[];
  if (a.S < 0) occupancy_limiter[threadIdx.x] = 0.0;
  const long base = (long)blockIdx.x * a.ld;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  int la, lb;
  offs<false>(tid, la, lb);
  // store offsets: PERM: lane a < 32 -> 4a, lane 32 + a -> 4a + 2; BPERM: 2 l
  const int sa = w * 256 + (BPERM ? 2 * l : (l < 32 ? 4 * l : 4 * (l - 32) + 2));
  const int addr = 4 * ((l >> 1) + 32 * (l & 1));
  dbl2 nx[NIN][2];
  for (int f = 0; f < NIN; ++f) {
    nx[f][0] = *reinterpret_cast<const dbl2*>(a.in[f] + base + la);
    nx[f][1] = *reinterpret_cast<const dbl2*>(a.in[f] + base + lb);
  }
  for (long t0 = 0; t0 < a.T; t0 += TILE) {
    dbl2 cu[NIN][2];
    for (int f = 0; f < NIN; ++f) {
      cu[f][0] = nx[f][0];
      cu[f][1] = nx[f][1];
    }
    if (t0 + TILE < a.T)
      for (int f = 0; f < NIN; ++f) {
        nx[f][0] = *reinterpret_cast<const dbl2*>(a.in[f] + base + t0 + TILE + la);
        nx[f][1] = *reinterpret_cast<const dbl2*>(a.in[f] + base + t0 + TILE + lb);
      }
    dbl2 s0 = {0, 0}, s1 = {0, 0};
    for (int f = 0; f < NIN; ++f) {
      s0 += cu[f][0];
      s1 += cu[f][1];
    }
    for (int o = 0; o < NOUT; ++o) {
      dbl2 A = s0 + (double)o, B = s1;
      swap32(A, B);
      if (BPERM) {
        A = pull(A, addr);
        B = pull(B, addr);
      }
      __builtin_nontemporal_store(A, reinterpret_cast<dbl2*>(a.out[o] + base + t0 + sa));
      __builtin_nontemporal_store(B, reinterpret_cast<dbl2*>(a.out[o] + base + t0 + sa + 128));
    }
  }
}

int main(int argc, char** argv) {
  const long S = argc > 1 ? atol(argv[1]) : 12500, T = 10240;   // whole tiles: the probe has no tail path
  const int reps = 10;
  struct V { const char* name; int split; int nts; int lds; };   // split 2/3: walk2<256>/<512>
  const bool quick = argc > 2;   // only the kernel-relevant variants
  const V vq[] = {{"half_nt_3wg", 0, 1, 52000}, {"split_nt_3wg", 1, 1, 52000}, {"swap_perm_3wg", 7, 1, 52000},
                  {"swap_bperm_3wg", 8, 1, 52000}, {"half_nt_3wg_b", 0, 1, 52000}, {"swap_perm_3wg_b", 7, 1, 52000}};
  const V vs[] = {
      {"half_3wg", 0, 0, 52000}, {"split_3wg", 1, 0, 52000}, {"half_nt_3wg", 0, 1, 52000},
      {"split_nt_3wg", 1, 1, 52000}, {"half_nt_4wg", 0, 1, 39000}, {"split_nt_4wg", 1, 1, 39000},
      {"half_nt_3wg_b", 0, 1, 52000}, {"split_nt_3wg_b", 1, 1, 52000},
      {"k2t512_nt_3wg", 2, 1, 52000}, {"k2t512_nt_4wg", 2, 1, 39000}, {"k2t512_nt_5wg", 2, 1, 31000},
      {"k2t512_nt_6wg", 2, 1, 26000}, {"k2nt512_t1024_nt_2wg", 3, 1, 78000}, {"k2nt512_t1024_nt_3wg", 3, 1, 52000},
      {"mix_lhalf_s4half", 4, 1, 52000}, {"mix_lhalf_s0half", 5, 1, 52000}, {"mix_lsplit_s4half", 6, 1, 52000},
      {"split_nt_3wg_c", 1, 1, 52000}, {"half_nt_3wg_c", 0, 1, 52000},
      {"swap_perm_3wg", 7, 1, 52000}, {"swap_bperm_3wg", 8, 1, 52000},
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
  const int nv = quick ? (int)(sizeof(vq) / sizeof(vq[0])) : (int)(sizeof(vs) / sizeof(vs[0]));
  for (int iv = 0; iv < nv; ++iv) {
    const V& v = quick ? vq[iv] : vs[iv];
    for (int r = 0; r < reps + 2; ++r) {
      if (r == 2) CK(hipEventRecord(e0));
      if (v.split == 7) walk_swap<false><<<S, NT, v.lds>>>(a);
      else if (v.split == 8) walk_swap<true><<<S, NT, v.lds>>>(a);
      else if (v.split == 4) walk_mix<false, 4><<<S, NT, v.lds>>>(a);
      else if (v.split == 5) walk_mix<false, 0><<<S, NT, v.lds>>>(a);
      else if (v.split == 6) walk_mix<true, 4><<<S, NT, v.lds>>>(a);
      else if (v.split == 2) walk2<256><<<S, 256, v.lds>>>(a);
      else if (v.split == 3) walk2<512><<<S, 512, v.lds>>>(a);
      else if (v.split && v.nts) walk<true, true><<<S, NT, v.lds>>>(a);
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
