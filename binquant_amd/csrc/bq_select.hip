// Whole-series order statistics and the sequential label cooldown of the
// strategy pipelines.
//
//   bq_row_quantile: per row, numpy.quantile(x[~isnan(x)], q) with numpy's
//     default 'linear' method (numpy/lib/_function_base_impl.py _quantile,
//     numpy 2.2): virtual index (n-1)*q, previous = floor, next = previous+1
//     clamped to n-1, gamma = index - previous, and numpy's two-sided _lerp
//     (a + (b-a)*g for g < 0.5, b - (b-a)*(1-g) otherwise). NaN when the row
//     has no observation. Restates FailedSpikeFade.auto_calibrate
//     (strategies/failed_spike_fade.py:229-257, np.quantile of dropna'd
//     volume_ratio / price_change_abs) and Series.quantile
//     (relative_strength_reversal_range.py:98).
//
//     Mapping: one 256-thread workgroup per row, radix select over the
//     order-preserving 64-bit image of the doubles: 8 passes of an 8-bit digit
//     histogram in LDS narrow the k-th key (the digit picked by a block scan
//     of the bins) — stopping as soon as one key carries the selected prefix
//     (then fetched directly) — one more pass finds its successor. Rows up to 10,240
//     values keep their keys in registers (one HBM read); longer rows stream
//     each pass (L2-resident after the first); no sort, no scratch in HBM.
//
//   bq_cooldown: FailedSpikeFade.apply_cooldown
//     (strategies/failed_spike_fade.py:495-520): walking forward, a label
//     within `bars` of the last KEPT label is cleared and flagged suppressed.
//     The dependence is sequential (the kept set depends on earlier
//     suppressions), so lane = symbol, one pass over its row.
#include "bq_device.h"
#include "binquant_amd.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

namespace bq {

constexpr int SQ_NT = 256;

__device__ __forceinline__ uint64_t order_key(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ double key_value(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)u);
}

// block-wide sum of an int (all threads get the result)
__device__ __forceinline__ int block_sum(int v, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int w = 0; w < SQ_NT / 64; ++w) s += red[w];
  return s;
}

__device__ __forceinline__ uint64_t block_min_u64(uint64_t v, uint64_t* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t p = __shfl_xor(v, o);
    v = p < v ? p : v;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  uint64_t m = red[0];
#pragma unroll
  for (int w = 1; w < SQ_NT / 64; ++w) m = red[w] < m ? red[w] : m;
  return m;
}

// KR > 0: the row's keys stay in registers (KR per thread, T <= 256 * KR), so
// the row is read from HBM once; KR == 0 streams the row on every pass. The
// digit whose bin holds rank k is found by a block-wide scan of the 256 bins
// (one bin per thread), not by a serial walk.
template <int KR>
__global__ __launch_bounds__(SQ_NT) void row_quantile_kernel(const double* __restrict__ x, int T, int64_t ld_in,
                                                             double q, double* __restrict__ out) {
  __shared__ unsigned hist[256];
  __shared__ int red_i[SQ_NT / 64];
  __shared__ uint64_t red_u[SQ_NT / 64];
  __shared__ unsigned wsum[SQ_NT / 64];
  __shared__ uint64_t s_prefix, s_key;
  __shared__ int s_k, s_h;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* __restrict__ r = x + (int64_t)blockIdx.x * ld_in;

  // key 0 never encodes a number (order_key sets bit 63 for positives and
  // only an all-ones NaN would map a negative to 0): it marks NaN / padding
  uint64_t kr[KR > 0 ? KR : 1];
  int cnt = 0;
  if (KR > 0) {
#pragma unroll
    for (int i = 0; i < (KR > 0 ? KR : 1); ++i) {
      const int t = tid + i * SQ_NT;
      const double v = t < T ? r[t] : qnan();
      kr[i] = v == v ? order_key(v) : 0ull;
      cnt += v == v;
    }
  } else {
    for (int t = tid; t < T; t += SQ_NT) cnt += r[t] == r[t];
  }
  const int n = block_sum(cnt, red_i);
  if (n == 0) {
    if (tid == 0) out[blockIdx.x] = qnan();
    return;
  }
  const double vi = (double)(n - 1) * q;
  const double fl = floor(vi);
  const int prev = (int)fl;
  const int next = prev + 1 < n ? prev + 1 : n - 1;
  const double gamma = vi - fl;

  // radix select of the prev-th smallest key
  uint64_t prefix = 0, mask = 0;
  int k = prev;
  for (int sh = 56; sh >= 0; sh -= 8) {
    hist[tid] = 0;   // SQ_NT == 256 bins
    __syncthreads();
    if (KR > 0) {
#pragma unroll
      for (int i = 0; i < (KR > 0 ? KR : 1); ++i) {
        const uint64_t key = kr[i];
        if (key && (key & mask) == prefix) atomicAdd(&hist[(key >> sh) & 255u], 1u);
      }
    } else {
      for (int t = tid; t < T; t += SQ_NT) {
        const double v = r[t];
        if (v == v) {
          const uint64_t key = order_key(v);
          if ((key & mask) == prefix) atomicAdd(&hist[(key >> sh) & 255u], 1u);
        }
      }
    }
    __syncthreads();
    // exclusive prefix of the bins; the bin with excl <= k < excl + h holds rank k
    const unsigned h = hist[tid];
    unsigned incl = h;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    unsigned excl = incl - h;
#pragma unroll
    for (int w = 0; w < SQ_NT / 64; ++w) excl += w < wave ? wsum[w] : 0u;
    if (h > 0 && (int)excl <= k && k < (int)(excl + h)) {
      s_prefix = prefix | ((uint64_t)tid << sh);
      s_k = k - (int)excl;
      s_h = (int)h;
    }
    __syncthreads();
    prefix = s_prefix;
    k = s_k;
    mask |= 255ull << sh;
    if (s_h == 1 && sh > 0) {
      // one key carries this prefix: it is the k-th; fetch it instead of
      // narrowing the remaining digits (a row of ~2 000 distinct doubles is
      // usually down to one key after 2-3 of the 8 passes)
      if (KR > 0) {
#pragma unroll
        for (int i = 0; i < (KR > 0 ? KR : 1); ++i) {
          const uint64_t key = kr[i];
          if (key && (key & mask) == prefix) s_key = key;
        }
      } else {
        for (int t = tid; t < T; t += SQ_NT) {
          const double v = r[t];
          if (v == v && (order_key(v) & mask) == prefix) s_key = order_key(v);
        }
      }
      __syncthreads();
      prefix = s_key;
      break;
    }
  }
  const double a = key_value(prefix);
  double b = a;
  if (next != prev) {
    int le = 0;
    uint64_t above = ~0ull;
    if (KR > 0) {
#pragma unroll
      for (int i = 0; i < (KR > 0 ? KR : 1); ++i) {
        const uint64_t key = kr[i];
        if (key) {
          le += key <= prefix;
          if (key > prefix && key < above) above = key;
        }
      }
    } else {
      for (int t = tid; t < T; t += SQ_NT) {
        const double v = r[t];
        if (v == v) {
          const uint64_t key = order_key(v);
          le += key <= prefix;
          if (key > prefix && key < above) above = key;
        }
      }
    }
    const int nle = block_sum(le, red_i);
    const uint64_t mn = block_min_u64(above, red_u);
    b = nle > next ? a : key_value(mn);
  }
  if (tid == 0) {
    const double d = b - a;
    out[blockIdx.x] = gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
  }
}

// Rows of up to 64 * RQ_KW values: one WAVE per row (4 rows per workgroup),
// the same radix select with the row's keys in the wave's registers (RQ_KW
// per lane) and the 256-bin histogram in LDS — no workgroup barrier: the
// block kernel's passes were ~4 barriers each over 4 waves of one row.
// The top digits of real rows fall in a handful of bins (sign + exponent: a
// row of ratios around 1.0 puts every key in 2 bins), and same-address LDS
// atomics of one instruction serialise (r6k PMC: 80 % of the kernel's LDS
// cycles were bank-conflict cycles), so each wave keeps RQ_NCOPY copies of
// the bins, lane l adding into copy l % RQ_NCOPY; the copies sit RQ_CSTRIDE
// dwords apart (8 banks of skew), and the owner lane of a bin sums them.
// NaN maps to the all-ones key: above every number (order_key never yields
// it), so it is never the k-th (k < n) and needs no test in the passes.
constexpr int RQ_KW = 32;
constexpr int RQ_WPB = 4;
constexpr int RQ_NCOPY = 8;
constexpr int RQ_CSTRIDE = 256 + 8;

// inclusive wave scan of an unsigned (DPP rows + row carries)
__device__ __forceinline__ unsigned wave_scan_add_u32(unsigned v, int lane) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const unsigned y = __shfl_up(v, d, WAVE);
    if (lane >= d) v += y;
  }
  return v;
}

__global__ __launch_bounds__(RQ_WPB * WAVE) void row_quantile_wave_kernel(const double* __restrict__ x, int64_t S,
                                                                            int T, int64_t ld_in, double q,
                                                                            double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned hist_all[RQ_WPB][RQ_NCOPY * RQ_CSTRIDE];
  const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
  const int64_t row = (int64_t)blockIdx.x * RQ_WPB + wv;
  if (row >= S) return;   // whole wave; no workgroup barrier below
  unsigned* hist = hist_all[wv];
  unsigned* mine = hist + (lane & (RQ_NCOPY - 1)) * RQ_CSTRIDE;
  const double* __restrict__ r = x + row * ld_in;
  // lane-contiguous pairs of values: 16-byte loads
  uint64_t kr[RQ_KW];
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < RQ_KW; ++i) {
    const int t = (i >> 1) * (2 * WAVE) + 2 * lane + (i & 1);
    const double v = t < T ? r[t] : qnan();
    kr[i] = v == v ? order_key(v) : ~0ull;
    cnt += v == v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  const int n = cnt;
  if (n == 0) {
    if (lane == 0) out[row] = qnan();
    return;
  }
  const double vi = (double)(n - 1) * q;
  const double fl = floor(vi);
  const int prev = (int)fl;
  const int next = prev + 1 < n ? prev + 1 : n - 1;
  const double gamma = vi - fl;
  uint64_t prefix = 0, mask = 0;
  int k = prev;
  for (int sh = 56; sh >= 0; sh -= 8) {
#pragma unroll
    for (int c = 0; c < RQ_NCOPY; ++c)
      *reinterpret_cast<uint4*>(hist + c * RQ_CSTRIDE + 4 * lane) = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < RQ_KW; ++i) {
      const uint64_t key = kr[i];
      if ((key & mask) == prefix) atomicAdd(&mine[(unsigned)(key >> sh) & 255u], 1u);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // lane l owns bins 4l .. 4l + 3: its 4 counts over the copies, then the
    // wave's exclusive prefix
    unsigned h[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int c = 0; c < RQ_NCOPY; ++c) {
      const uint4 w = *reinterpret_cast<const uint4*>(hist + c * RQ_CSTRIDE + 4 * lane);
      h[0] += w.x;
      h[1] += w.y;
      h[2] += w.z;
      h[3] += w.w;
    }
    const unsigned tot = h[0] + h[1] + h[2] + h[3];
    const unsigned incl = wave_scan_add_u32(tot, lane);
    unsigned excl = incl - tot;
    int found = -1, fk = 0, fh = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (found < 0 && h[b] > 0 && (int)excl <= k && k < (int)(excl + h[b])) {
        found = 4 * lane + b;
        fk = k - (int)excl;
        fh = (int)h[b];
      }
      excl += h[b];
    }
    // exactly one lane found the bin: broadcast it
    const uint64_t bal = __ballot(found >= 0);
    const int src = __builtin_ctzll(bal);
    const int bin = __shfl(found, src, WAVE);
    k = __shfl(fk, src, WAVE);
    const int hb = __shfl(fh, src, WAVE);
    prefix |= (uint64_t)bin << sh;
    mask |= 255ull << sh;
    if (hb == 1 && sh > 0) {   // one key carries the prefix: fetch it
      uint64_t got = 0;
#pragma unroll
      for (int i = 0; i < RQ_KW; ++i) {
        const uint64_t key = kr[i];
        if ((key & mask) == prefix) got = key;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t p = __shfl_xor(got, o);
        got = p > got ? p : got;
      }
      prefix = got;
      break;
    }
    // the next pass clears the bins other lanes are still reading
    __builtin_amdgcn_wave_barrier();
  }
  const double a = key_value(prefix);
  double b = a;
  if (next != prev) {
    // NaN keys (all ones) are above a and never the minimum above it while a
    // number is; with none above, le == n > next
    int le = 0;
    uint64_t above = ~0ull;
#pragma unroll
    for (int i = 0; i < RQ_KW; ++i) {
      const uint64_t key = kr[i];
      le += key <= prefix;
      if (key > prefix && key < above) above = key;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      le += __shfl_xor(le, o);
      const uint64_t p = __shfl_xor(above, o);
      above = p < above ? p : above;
    }
    b = le > next ? a : key_value(above);
  }
  if (lane == 0) {
    const double d = b - a;
    out[row] = gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
  }
}

// One wave per symbol row: 64 candles per step are read as one coalesced
// 64-byte load, the labels of the step become one ballot mask, and the greedy
// (keep a label iff it is more than `bars` after the last kept one) walks only
// the set bits of the mask with wave-uniform scalar arithmetic — labels are
// sparse, so a row costs ~T/64 steps instead of T dependent byte loads.
__global__ __launch_bounds__(256) void cooldown_kernel(const uint8_t* __restrict__ label, int64_t S, int T,
                                                       int64_t ld_in, int bars, uint8_t* __restrict__ kept,
                                                       uint8_t* __restrict__ suppressed, int64_t ld_out) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int64_t s = (int64_t)blockIdx.x * (256 / WAVE) + threadIdx.x / WAVE;
  if (s >= S) return;   // whole wave
  const uint8_t* __restrict__ l = label + s * ld_in;
  uint8_t* __restrict__ k = kept + s * ld_out;
  uint8_t* __restrict__ u = suppressed + s * ld_out;
  int last = -0x40000000;   // "None": never within reach
  for (int t0 = 0; t0 < T; t0 += WAVE) {
    const int t = t0 + lane;
    const bool on = t < T && l[t] != 0;
    uint64_t m = __ballot(on);
    uint64_t keep = 0;
    while (m) {
      const int i = __builtin_ctzll(m);
      m &= m - 1;
      if (t0 + i - last > bars) {
        keep |= 1ull << i;
        last = t0 + i;
      }
    }
    if (t < T) {
      const bool kb = (keep >> lane) & 1ull;
      k[t] = (uint8_t)kb;
      u[t] = (uint8_t)(on && !kb);
    }
  }
}

}  // namespace bq

namespace {
// BQ_ROW_QUANTILE_WAVE=0: the workgroup-per-row kernel for every row length
bool row_quantile_wave() {
  static const bool on = [] {
    const char* e = getenv("BQ_ROW_QUANTILE_WAVE");
    return !(e && e[0] == '0');
  }();
  return on;
}
}  // namespace

extern "C" {

int bq_row_quantile(const double* x, int64_t S, int64_t T, int64_t ld_in, double q, double* out, void* stream) {
  using namespace bq;
  if (!x || !out || S < 0 || T < 0 || ld_in < T || !(q >= 0.0 && q <= 1.0) || T > 0x7fffffff || S > 0x7fffffff)
    return BQ_EINVAL;
  if (S == 0) return BQ_OK;
  const dim3 g((unsigned)S), blk(SQ_NT);
  hipStream_t st = (hipStream_t)stream;
  if (T <= RQ_KW * WAVE && row_quantile_wave())
    hipLaunchKernelGGL(row_quantile_wave_kernel, dim3((unsigned)((S + RQ_WPB - 1) / RQ_WPB)), dim3(RQ_WPB * WAVE), 0,
                       st, x, S, (int)T, ld_in, q, out);
  else if (T <= 8 * SQ_NT) hipLaunchKernelGGL(row_quantile_kernel<8>, g, blk, 0, st, x, (int)T, ld_in, q, out);
  else if (T <= 16 * SQ_NT) hipLaunchKernelGGL(row_quantile_kernel<16>, g, blk, 0, st, x, (int)T, ld_in, q, out);
  else if (T <= 40 * SQ_NT) hipLaunchKernelGGL(row_quantile_kernel<40>, g, blk, 0, st, x, (int)T, ld_in, q, out);
  else hipLaunchKernelGGL(row_quantile_kernel<0>, g, blk, 0, st, x, (int)T, ld_in, q, out);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_cooldown(const uint8_t* label, int64_t S, int64_t T, int64_t ld_in, int32_t bars, uint8_t* kept,
                uint8_t* suppressed, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!label || !kept || !suppressed || S < 0 || T < 0 || ld_in < T || ld_out < T || bars < 0 ||
      T > 0x7fffffff)
    return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  hipLaunchKernelGGL(cooldown_kernel, dim3((unsigned)((S + 3) / 4)), dim3(256), 0, (hipStream_t)stream, label, S,
                     (int)T, ld_in, (int)bars, kept, suppressed, ld_out);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
