// Fused failed-spike stages (gfx950): FailedSpikeFade.detect
// (strategies/failed_spike_fade.py:260-544) on an [S][T] panel in two passes
// per row around the whole-series calibration:
//
//   bq_spike_base   compute_base_features (:260-322) and the early-feature
//                   operands (:324-357): the candle geometry, pct changes of
//                   the pad-filled close, the rolling means / sums / integer
//                   counts (base window, 2 / 3 / 5-bar sums, 10-bar body
//                   stats, the streak counts) formed in the kernel, the
//                   z-scores / ratios / momentum against the rolling std
//                   columns (inputs: the bit-exact Welford replays of
//                   bq_rolling_batch), the streak flags;
//   bq_spike_flags  after auto_calibrate (:229-257: per-row thresholds from
//                   bq_row_quantile) — the volume-cluster, price-break (the
//                   dynamic threshold: maximum(base, rolling quantile),
//                   ffilled), cumulative and acceleration flags and the
//                   preliminary labels (:360-488).
//
// Staged, the pipeline ran ~10 element-wise / window launches that wrote and
// re-read every intermediate (~2.4x its algorithmic bytes). Every expression
// is the staged programs' (the reference's operation order); the rolling
// means / sums are direct window sums in time order with pandas' rules
// (min_periods = window, the same-value and sign rules), equal to the staged
// panel-mode sums to rounding; integer counts and every flag downstream of
// them are exact.
//
// Mapping (as bq_pump): one 256-thread workgroup per row, tiles of 1024
// candles (4 per lane), an LDS ring with a 32-candle halo for the series the
// windows read.
#include "bq_device.h"
#include "binquant_amd.h"

#include <stdint.h>
#include <string.h>

namespace bq {

constexpr int SP_NT = 256;
constexpr int SP_NW = SP_NT / WAVE;
constexpr int SP_K = 4;
constexpr int SP_TT = SP_NT * SP_K;   // 1024
constexpr int SP_H = 32;
constexpr int SP_R = SP_H + SP_TT;
constexpr int SP_Q = SP_R / SP_K;
__device__ __forceinline__ int sp_slot(int p) { return (p & (SP_K - 1)) * SP_Q + (p >> 2); }
constexpr double SP_EPS = 1e-6;

typedef double sp_dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void sp_load(const double* __restrict__ row, int tb, int T, bool vec, double (&x)[SP_K]) {
  if (vec && tb + SP_K <= T) {
    const sp_dbl2* p = reinterpret_cast<const sp_dbl2*>(row + tb);
    const sp_dbl2 a = p[0], b = p[1];
    x[0] = a.x;
    x[1] = a.y;
    x[2] = b.x;
    x[3] = b.y;
  } else {
#pragma unroll
    for (int k = 0; k < SP_K; ++k) x[k] = tb + k < T ? row[tb + k] : qnan();
  }
}

__device__ __forceinline__ void sp_put_bytes(uint8_t* __restrict__ row, int tb, int T, bool vec4, const bool (&b)[SP_K]) {
  if (vec4 && tb + SP_K <= T) {
    const uint32_t w = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    *reinterpret_cast<uint32_t*>(row + tb) = w;
  } else {
#pragma unroll
    for (int k = 0; k < SP_K; ++k)
      if (tb + k < T) row[tb + k] = b[k] ? 1 : 0;
  }
}

// Every window of the two passes has min_periods = w: a window holding a
// missing value (NaN / +-inf: pandas' window ops) is NaN whatever else it
// holds. So the aggregates add raw values and count the observed ones only to
// detect that, and pandas' rules apply to complete windows only, where they
// reduce to sums: calc_mean's sign rule to the sign-bit count (its neg_ct,
// signbit as pandas counts it) and the same-value rule to sum |v - ref| about
// a value of the window (zero iff every value equals it; the result is then
// the newest value, times the count for a sum). No min / max, no selects per
// value; a complete window's sum is the same sum in the same order as before.
struct SpAgg {
  double s, sa;
  int n, neg;
  __device__ __forceinline__ void init() {
    s = sa = 0.0;
    n = neg = 0;
  }
  __device__ __forceinline__ void add(double v, double ref) {
    n += win_ok(v);
    neg += (int)((unsigned long long)__double_as_longlong(v) >> 63);
    s += v;
    sa += fabs(v - ref);
  }
  // this (older) followed by b (newer)
  __device__ __forceinline__ SpAgg then(const SpAgg& b) const {
    SpAgg r;
    r.s = s + b.s;
    r.sa = sa + b.sa;
    r.n = n + b.n;
    r.neg = neg + b.neg;
    return r;
  }
};

// last: the window's newest value
template <bool MEAN>
__device__ __forceinline__ double sp_finish(const SpAgg& a, int t, int w, double last) {
  if (t < w - 1 || a.n < w) return qnan();
  const bool same = a.sa == 0.0;
  if (!MEAN) return same ? last * (double)a.n : a.s;
  double r = a.s / (double)a.n;
  if (same) r = last;
  else if (a.neg == 0 && r < 0.0) r = 0.0;
  else if (a.neg == a.n && r > 0.0) r = 0.0;
  return r;
}

// x.rolling(w).sum() / .mean() at candle t over values f(j), j = -w+1 .. 0
// (time order)
template <bool MEAN, typename F>
__device__ __forceinline__ double sp_window(int t, int w, F f) {
  if (t < w - 1) return qnan();
  const double last = f(0);
  SpAgg a;
  a.init();
  for (int j = -w + 1; j <= 0; ++j) a.add(f(j), last);
  return sp_finish<MEAN>(a, t, w, last);
}

// The same statistic at a lane's SP_K consecutive candles tb .. tb + 3 (ring
// positions pb .. pb + 3): their windows share the W - 3 positions
// pb + 4 - W .. pb, aggregated once; each candle adds its own older (lead) and
// newer (trail) extras — W + 3 values read instead of 4 W. The sum is
// (lead + core) + trail instead of strictly time-ordered (rounding). The
// reference of the same-value test: the value at pb, inside every one of the
// lane's windows.
// F(p): the value at ring position p (windows shorter than SP_K: one
// aggregate per candle)
template <bool MEAN, typename F>
__device__ __forceinline__ void sp_window4(int tb, int pb, int w, F f, double (&r)[SP_K]) {
  if (w < SP_K) {
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      const double last = f(pb + k);
      SpAgg a;
      a.init();
      for (int p = pb + k - w + 1; p <= pb + k; ++p) a.add(f(p), last);
      r[k] = sp_finish<MEAN>(a, tb + k, w, last);
    }
    return;
  }
  const double ref = f(pb);
  SpAgg core;
  core.init();
  for (int p = pb + SP_K - w; p <= pb; ++p) core.add(f(p), ref);
  SpAgg trail;
  trail.init();
  SpAgg lead[SP_K];
  lead[SP_K - 1].init();
#pragma unroll
  for (int k = SP_K - 2; k >= 0; --k) {   // lead_k = value at pb + k + 1 - w, then lead_{k+1}
    SpAgg one;
    one.init();
    one.add(f(pb + k + 1 - w), ref);
    lead[k] = one.then(lead[k + 1]);
  }
#pragma unroll
  for (int k = 0; k < SP_K; ++k) {
    const double last = f(pb + k);
    if (k > 0) trail.add(last, ref);
    r[k] = sp_finish<MEAN>(lead[k].then(core).then(trail), tb + k, w, last);
  }
}

// an integer count over the window (values 0 / 1, never missing): the sum
template <typename F>
__device__ __forceinline__ double sp_count(int t, int w, F f) {
  if (t < w - 1) return qnan();
  int c = 0;
  for (int j = -w + 1; j <= 0; ++j) c += f(j);
  return (double)c;
}

// x.rolling(w).std() (ddof 1, min_periods = w) at a lane's SP_K consecutive
// candles from the ring values f(p): sums of d = x - r about a reference r
// inside every one of the lane's windows (the value at the lane's first
// candle), shared like sp_window4 (one core over the W - 3 common positions,
// lead / trail extras per candle): var = (S2 - S1^2 / n) / (n - 1). With r in
// the window, |mean - r| is at most the window's range, so the cancellation
// costs O(n eps) relative — the window's variance to rounding, where pandas'
// online add / remove recurrence over the whole row (roll_var) drifts when the
// std is small against the values (~1e-8 relative at std / mean ~ 2e-5): the
// panel result is then the one closer to the exactly computed value
// (tests/test_spike_std_gpu.py). pandas' rules: a missing value in the window
// -> NaN (min_periods = w); n <= 1 -> NaN; every value equal (sum |d| == 0)
// -> 0.
struct SpVar {
  double s1, s2, sa;
  int n;
  __device__ __forceinline__ void init() {
    s1 = s2 = sa = 0.0;
    n = 0;
  }
  __device__ __forceinline__ void add(double v, double r) {
    n += win_ok(v);
    const double d = v - r;
    s1 += d;
    s2 = fma(d, d, s2);
    sa += fabs(d);
  }
  __device__ __forceinline__ SpVar then(const SpVar& b) const {
    SpVar x;
    x.s1 = s1 + b.s1;
    x.s2 = s2 + b.s2;
    x.sa = sa + b.sa;
    x.n = n + b.n;
    return x;
  }
};

__device__ __forceinline__ double sp_var_finish(double s1, double s2, double sa, int n, int t, int w) {
  if (t < w - 1 || w <= 1 || n < w) return qnan();
  if (sa == 0.0) return 0.0;
  const double var = (s2 - s1 * (s1 / (double)n)) / (double)(n - 1);
  return sqrt(var > 0.0 ? var : 0.0);
}

template <typename F>
__device__ __forceinline__ void sp_std4(int tb, int pb, int w, F f, double (&r)[SP_K]) {
  if (w < SP_K) {   // windows shorter than the lane: each about its own newest value
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      SpVar a;
      a.init();
      const double rk = f(pb + k);
      for (int p = pb + k - w + 1; p <= pb + k; ++p) a.add(f(p), rk);
      r[k] = sp_var_finish(a.s1, a.s2, a.sa, a.n, tb + k, w);
    }
    return;
  }
  const double ref = f(pb);
  SpVar core;
  core.init();
  for (int p = pb + SP_K - w; p <= pb; ++p) core.add(f(p), ref);
  SpVar lead[SP_K], trail;
  trail.init();
  lead[SP_K - 1].init();
#pragma unroll
  for (int k = SP_K - 2; k >= 0; --k) {
    SpVar one;
    one.init();
    one.add(f(pb + k + 1 - w), ref);
    lead[k] = one.then(lead[k + 1]);
  }
#pragma unroll
  for (int k = 0; k < SP_K; ++k) {
    if (k > 0) trail.add(f(pb + k), ref);
    const SpVar x = lead[k].then(core).then(trail);
    r[k] = sp_var_finish(x.s1, x.s2, x.sa, x.n, tb + k, w);
  }
}

// sp_window4<true> and sp_std4 over the same window in ONE walk of the ring
// (the count and sum |d| serve both). Same values as the two separate calls.
struct SpAggV {
  SpAgg a;
  double s1, s2;
  __device__ __forceinline__ void init() {
    a.init();
    s1 = s2 = 0.0;
  }
  __device__ __forceinline__ void add(double v, double r) {
    a.add(v, r);
    const double d = v - r;
    s1 += d;
    s2 = fma(d, d, s2);
  }
  __device__ __forceinline__ SpAggV then(const SpAggV& b) const {
    SpAggV x;
    x.a = a.then(b.a);
    x.s1 = s1 + b.s1;
    x.s2 = s2 + b.s2;
    return x;
  }
};

template <typename F>
__device__ __forceinline__ void sp_mean_std4(int tb, int pb, int w, F f, double (&ma)[SP_K], double (&sd)[SP_K]) {
  if (w < SP_K) {   // short windows: the separate forms (per-candle references)
    sp_window4<true>(tb, pb, w, f, ma);
    sp_std4(tb, pb, w, f, sd);
    return;
  }
  const double ref = f(pb);
  SpAggV core;
  core.init();
  for (int p = pb + SP_K - w; p <= pb; ++p) core.add(f(p), ref);
  SpAggV lead[SP_K], trail;
  trail.init();
  lead[SP_K - 1].init();
#pragma unroll
  for (int k = SP_K - 2; k >= 0; --k) {
    SpAggV one;
    one.init();
    one.add(f(pb + k + 1 - w), ref);
    lead[k] = one.then(lead[k + 1]);
  }
#pragma unroll
  for (int k = 0; k < SP_K; ++k) {
    const double last = f(pb + k);
    if (k > 0) trail.add(last, ref);
    const SpAggV x = lead[k].then(core).then(trail);
    ma[k] = sp_finish<true>(x.a, tb + k, w, last);
    sd[k] = sp_var_finish(x.s1, x.s2, x.a.sa, x.a.n, tb + k, w);
  }
}

// ---- pass 1: base features ------------------------------------------------------------
enum { SB_O = 0, SB_H, SB_L, SB_C, SB_V, SB_Q, SB_CF, SB_PSTD, SB_VSTD, SB_S8, SB_S20, SB_BSD, SB_NIN };

struct SpikeBaseArgs {
  const double* in[SB_NIN];
  double* out[BQ_NUM_SPIKE_BASE_F];
  uint8_t* flag[BQ_NUM_SPIKE_BASE_B];
  double* sd[BQ_NUM_SPIKE_STD];   // TP: the std columns the kernel forms (NULL = not written)
  int64_t S, ld_in, ld_out;
  int T, w, n, pad;
};

// 3 workgroups per CU (168 VGPRs, 12 B of spill) instead of 2 at 178 VGPRs:
// a19 4.10 -> 3.99 ms (A/B, same box)
// TP: the five std columns formed here (sp_std over the rings, written to
// A.sd) instead of read from the replay's columns (A.in[SB_PSTD ..])
#ifndef BQ_SP_TP_WGS
#define BQ_SP_TP_WGS 3   // workgroups per CU of the TP instantiation
#endif
// WC > 0: the base window (and streak length SN) as compile-time constants
// (the strategy's defaults): the window walks unroll and their ring slots
// become lane-base + immediate offsets instead of per-element index math
template <bool TP, int WC = 0, int SN = 0>
__global__ __launch_bounds__(SP_NT, TP ? BQ_SP_TP_WGS : 3) void spike_base_kernel(const SpikeBaseArgs A, int vin, int vout,
                                                                                int vb) {
  // rings: close, ffilled close, volume, quote volume, body size pct, pct
  // change (formed once per candle, read by every window), candle colour
  __shared__ double sC[SP_R], sF[SP_R], sV[SP_R], sQ[SP_R], sB[SP_R], sP[SP_R];
  __shared__ signed char sG[SP_R];   // +1 close > open, -1 close < open, 0 otherwise
  const int tid = threadIdx.x;
  const int64_t sym = blockIdx.x;
  const int T = A.T, W = WC > 0 ? WC : A.w, N = SN > 0 ? SN : A.n;
  const int64_t irow = sym * A.ld_in, orow = sym * A.ld_out;
  if (tid < SP_H) {
    sC[sp_slot(tid)] = sF[sp_slot(tid)] = sV[sp_slot(tid)] = sQ[sp_slot(tid)] = qnan();
    sB[sp_slot(tid)] = sP[sp_slot(tid)] = qnan();
    sG[sp_slot(tid)] = 0;
  }
  for (int t0 = 0; t0 < T; t0 += SP_TT) {
    const int tb = t0 + SP_K * tid, pb = SP_H + SP_K * tid;
    double o[SP_K], h[SP_K], l[SP_K], c[SP_K], v[SP_K], q[SP_K], cf[SP_K];
    sp_load(A.in[SB_O] + irow, tb, T, vin, o);
    sp_load(A.in[SB_H] + irow, tb, T, vin, h);
    sp_load(A.in[SB_L] + irow, tb, T, vin, l);
    sp_load(A.in[SB_C] + irow, tb, T, vin, c);
    sp_load(A.in[SB_V] + irow, tb, T, vin, v);
    sp_load(A.in[SB_Q] + irow, tb, T, vin, q);
    sp_load(A.in[SB_CF] + irow, tb, T, vin, cf);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      sC[sp_slot(pb + k)] = c[k];
      sF[sp_slot(pb + k)] = cf[k];
      sV[sp_slot(pb + k)] = v[k];
      sQ[sp_slot(pb + k)] = q[k];
      sB[sp_slot(pb + k)] = fabs(c[k] - o[k]) / (o[k] + SP_EPS);
      sG[sp_slot(pb + k)] = c[k] > o[k] ? 1 : (c[k] < o[k] ? -1 : 0);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SP_K; ++k) sP[sp_slot(pb + k)] = cf[k] / sF[sp_slot(pb + k - 1)] - 1.0;
    __syncthreads();
    const bool whole = t0 + SP_TT <= T, vo = vout != 0, v4 = vb != 0;
    auto put = [&](int col, const double (&r)[SP_K]) {
      if (A.out[col]) store_lines<SP_K>(A.out[col] + orow, tb, T, vo, r, whole);
    };
    auto putb = [&](int col, const bool (&b)[SP_K]) {
      if (A.flag[col]) sp_put_bytes(A.flag[col] + orow, tb, T, v4, b);
    };
    // ring readers (p = ring position of the candle)
    auto pc_at = [&](int p) { return sP[sp_slot(p)]; };   // pct_change of the ffilled close
    auto bsp_at = [&](int p) { return sB[sp_slot(p)]; };
    double r[SP_K], pc[SP_K], body[SP_K], bsp[SP_K];
    bool b[SP_K];
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      pc[k] = pc_at(pb + k);
      body[k] = fabs(c[k] - o[k]);
      bsp[k] = bsp_at(pb + k);
    }
    put(BQ_SPIKE_PRICE_CHANGE, pc);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = fabs(pc[k]);
    put(BQ_SPIKE_PRICE_CHANGE_ABS, r);
    put(BQ_SPIKE_BODY_SIZE, body);
    put(BQ_SPIKE_BODY_SIZE_PCT, bsp);
    double uw[SP_K], lw[SP_K];
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      uw[k] = h[k] - fmax(c[k], o[k]);
      lw[k] = fmin(c[k], o[k]) - l[k];
    }
    put(BQ_SPIKE_UPPER_WICK, uw);
    put(BQ_SPIKE_LOWER_WICK, lw);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = uw[k] / (body[k] + SP_EPS);
    put(BQ_SPIKE_UPPER_WICK_RATIO, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = lw[k] / (body[k] + SP_EPS);
    put(BQ_SPIKE_LOWER_WICK_RATIO, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = h[k] - l[k];
    put(BQ_SPIKE_TOTAL_RANGE, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = (h[k] - l[k]) / (o[k] + SP_EPS);
    put(BQ_SPIKE_RANGE_PCT, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) b[k] = c[k] > o[k];
    putb(BQ_SPIKE_IS_BULLISH, b);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = (c[k] - o[k]) / (o[k] + SP_EPS);
    put(BQ_SPIKE_CLOSE_OPEN_RATIO, r);
    // price: mean over the base window, z-score against the replayed std
    double ma[SP_K], sd[SP_K];
    // the std columns (TP): formed from the rings, written once
    auto std4 = [&](int wc, int slot_col, auto fr, double (&x)[SP_K]) {
      sp_std4(tb, pb, wc, fr, x);
      if (A.sd[slot_col]) store_lines<SP_K>(A.sd[slot_col] + orow, tb, T, vo, x, whole);
    };
    auto c_at = [&](int p) { return sC[sp_slot(p)]; };
    auto v_at = [&](int p) { return sV[sp_slot(p)]; };
    auto put_sd = [&](int col, const double (&x)[SP_K]) {
      if (A.sd[col]) store_lines<SP_K>(A.sd[col] + orow, tb, T, vo, x, whole);
    };
    if constexpr (TP) {
      sp_mean_std4(tb, pb, W, c_at, ma, sd);
      put_sd(BQ_SPIKE_STD_PRICE, sd);
    } else {
      sp_window4<true>(tb, pb, W, c_at, ma);
      sp_load(A.in[SB_PSTD] + irow, tb, T, vin, sd);
    }
    put(BQ_SPIKE_PRICE_MA, ma);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = (c[k] - ma[k]) / (sd[k] + SP_EPS);
    put(BQ_SPIKE_PRICE_ZSCORE, r);
    // volume
    if constexpr (TP) {
      sp_mean_std4(tb, pb, W, v_at, ma, sd);
      put_sd(BQ_SPIKE_STD_VOLUME, sd);
    } else {
      sp_window4<true>(tb, pb, W, v_at, ma);
    }
    put(BQ_SPIKE_VOLUME_MA, ma);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = v[k] / (ma[k] + SP_EPS);
    put(BQ_SPIKE_VOLUME_RATIO, r);
    if constexpr (!TP) sp_load(A.in[SB_VSTD] + irow, tb, T, vin, sd);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = (v[k] - ma[k]) / (sd[k] + SP_EPS);
    put(BQ_SPIKE_VOLUME_ZSCORE, r);
    // quote volume
    sp_window4<true>(tb, pb, W, [&](int p) { return sQ[sp_slot(p)]; }, ma);
    put(BQ_SPIKE_QUOTE_VOLUME_MA, ma);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = q[k] / (ma[k] + SP_EPS);
    put(BQ_SPIKE_QUOTE_VOLUME_RATIO, r);
    // momentum of the ffilled close
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = cf[k] / sF[sp_slot(pb + k - 3)] - 1.0;
    put(BQ_SPIKE_MOMENTUM_3, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = cf[k] / sF[sp_slot(pb + k - 5)] - 1.0;
    put(BQ_SPIKE_MOMENTUM_5, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = (h[k] - c[k]) / (h[k] + SP_EPS);
    put(BQ_SPIKE_CLOSE_TO_HIGH, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = (c[k] - l[k] + SP_EPS) / (c[k] + SP_EPS);
    put(BQ_SPIKE_CLOSE_TO_LOW, r);
    // the 8 / 20-bar std ratio and the compression flag
    {
      double s8[SP_K], s20[SP_K];
      if constexpr (TP) {
        std4(8, BQ_SPIKE_STD_8, c_at, s8);
        std4(20, BQ_SPIKE_STD_20, c_at, s20);
      } else {
        sp_load(A.in[SB_S8] + irow, tb, T, vin, s8);
        sp_load(A.in[SB_S20] + irow, tb, T, vin, s20);
      }
#pragma unroll
      for (int k = 0; k < SP_K; ++k) {
        r[k] = s8[k] / (s20[k] + SP_EPS);
        b[k] = s8[k] < s20[k] * 0.6;
      }
      put(BQ_SPIKE_STD_RATIO_8_20, r);
      putb(BQ_SPIKE_VOL_COMPRESSION_FLAG, b);
    }
    // pct-change sums, positive count, absolute sum
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = sp_window<false>(tb + k, 2, [&](int j) { return pc_at(pb + k + j); });
    put(BQ_SPIKE_PC_2C, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = sp_window<false>(tb + k, 3, [&](int j) { return pc_at(pb + k + j); });
    put(BQ_SPIKE_PC_3C, r);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = sp_count(tb + k, 5, [&](int j) { return pc_at(pb + k + j) > 0.0 ? 1 : 0; });
    put(BQ_SPIKE_PC_POS_COUNT_5, r);
    sp_window4<false>(tb, pb, 5, [&](int p) { return fabs(pc_at(p)); }, r);
    put(BQ_SPIKE_PC_ABS_SUM_5, r);
    // body size: 10-bar mean, z-score against the replayed std
    if constexpr (TP) {
      sp_mean_std4(tb, pb, 10, bsp_at, ma, sd);
      put_sd(BQ_SPIKE_STD_BODY_PCT_10, sd);
    } else {
      sp_window4<true>(tb, pb, 10, bsp_at, ma);
    }
    put(BQ_SPIKE_BODY_SIZE_PCT_MA_10, ma);
    if constexpr (!TP) sp_load(A.in[SB_BSD] + irow, tb, T, vin, sd);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) r[k] = (bsp[k] - ma[k]) / (sd[k] + SP_EPS);
    put(BQ_SPIKE_BODY_SIZE_PCT_Z, r);
    // detect_streaks: green / red counts over the streak length
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      const double g = sp_count(tb + k, N, [&](int j) { return sG[sp_slot(pb + k + j)] > 0 ? 1 : 0; });
      b[k] = g >= (double)N;
    }
    putb(BQ_SPIKE_UPWARD, b);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      const double g = sp_count(tb + k, N, [&](int j) { return sG[sp_slot(pb + k + j)] < 0 ? 1 : 0; });
      b[k] = g >= (double)N;
    }
    putb(BQ_SPIKE_DOWNWARD, b);

    if (t0 + SP_TT >= T) break;
    __syncthreads();
    if (pb >= SP_TT) {
#pragma unroll
      for (int k = 0; k < SP_K; ++k) {
        const int a = sp_slot(pb + k), d = sp_slot(pb + k - SP_TT);
        sC[d] = sC[a];
        sF[d] = sF[a];
        sV[d] = sV[a];
        sQ[d] = sQ[a];
        sB[d] = sB[a];
        sP[d] = sP[a];
        sG[d] = sG[a];
      }
    }
    __syncthreads();
  }
}

// ---- pass 2: flags and labels ---------------------------------------------------------
enum { SF_O = 0, SF_C, SF_CF, SF_VR, SF_DYN, SF_NIN };

struct SpikeFlagArgs {
  const double* in[SF_NIN];           // open, close, ffilled close, volume_ratio, rolling quantile of |pc|
  const double *vcmr, *pbbt;          // [S] calibrated volume-cluster ratio / price-break base
  double* out[BQ_NUM_SPIKE_FLAG_F];
  uint8_t* flag[BQ_NUM_SPIKE_FLAG_B];
  int64_t S, ld_in, ld_out;
  int T, cluster_w, cluster_min, cw, accel_w, mode, both, bullish;
  double cum_thr, accel_vd, accel_pc, body_min;
};

// 4 workgroups per CU (120 VGPRs, no spill): a19 -0.06 ms (A/B, same box)
__global__ __launch_bounds__(SP_NT, 4) void spike_flags_kernel(const SpikeFlagArgs A, int vin, int vout, int vb) {
  __shared__ double sF[SP_R], sP[SP_R], sVR[SP_R], sTP[SP_R];
  // the cluster conditions per candle, one byte each in time order (bit 0:
  // VR >= VC, bit 1: VR >= 0.8 VC; 0 before the row and for a missing ratio),
  // so a lane's 36-candle condition masks are 9 dword reads, not 36 compares
  __shared__ uint32_t sCB[SP_R / 4];
  __shared__ int sW[SP_NW];
  __shared__ int sCar;
  __shared__ double sTV;   // threshold carried across tiles (the ffill)
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t sym = blockIdx.x;
  const int T = A.T;
  const int64_t irow = sym * A.ld_in, orow = sym * A.ld_out;
  const double VC = A.vcmr[sym], PB = A.pbbt[sym];
  if (tid < SP_H) sF[sp_slot(tid)] = sP[sp_slot(tid)] = sVR[sp_slot(tid)] = sTP[sp_slot(tid)] = qnan();
  if (tid < SP_H / 4) sCB[tid] = 0u;
  const double vc8 = VC * 0.8;
  if (tid == 0) {
    sCar = -1;
    sTV = qnan();
  }
  for (int t0 = 0; t0 < T; t0 += SP_TT) {
    const int tb = t0 + SP_K * tid, pb = SP_H + SP_K * tid;
    double o[SP_K], c[SP_K], cf[SP_K], vr[SP_K], dy[SP_K];
    sp_load(A.in[SF_O] + irow, tb, T, vin, o);
    sp_load(A.in[SF_C] + irow, tb, T, vin, c);
    sp_load(A.in[SF_CF] + irow, tb, T, vin, cf);
    sp_load(A.in[SF_VR] + irow, tb, T, vin, vr);
    sp_load(A.in[SF_DYN] + irow, tb, T, vin, dy);
    // the volume ratio one candle past the tile (shift(base, -1) of the last candle)
    const double vr_next = tb + SP_K < T ? A.in[SF_VR][irow + tb + SP_K] : qnan();
    int lv[SP_K];
    int last = -1;
    uint32_t cb = 0u;
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      const int t = tb + k;
      cb |= ((vr[k] >= VC ? 1u : 0u) | (vr[k] >= vc8 ? 2u : 0u)) << (8 * k);
      // where(isnan(D), D, maximum(PB, D)): NaN stays, else the larger
      const double d = dy[k];
      const double tp = d != d ? d : (PB != PB ? qnan() : (PB > d ? PB : d));
      if (tp == tp && t < T) last = t;
      lv[k] = last;
      sF[sp_slot(pb + k)] = cf[k];
      sVR[sp_slot(pb + k)] = vr[k];
      sTP[sp_slot(pb + k)] = tp;
    }
    sCB[pb / 4] = cb;
    {
      const int inc = wave_scan_max_dpp(lv[SP_K - 1] + 1, lane);
      if (lane == WAVE - 1) sW[w] = inc - 1;
      const int ex = dpp_i32<DPP_WAVE_SHR1>(inc) - 1;
      __syncthreads();
      int cc = max(sCar, ex);
      for (int u = 0; u < w; ++u) cc = max(cc, sW[u]);
#pragma unroll
      for (int k = 0; k < SP_K; ++k) {
        lv[k] = max(lv[k], cc);
        sP[sp_slot(pb + k)] = cf[k] / sF[sp_slot(pb + k - 1)] - 1.0;   // the ring is complete (barrier above)
      }
      __syncthreads();
    }
    const bool whole = t0 + SP_TT <= T, vo = vout != 0, v4 = vb != 0;
    auto put = [&](int col, const double (&r)[SP_K]) {
      if (A.out[col]) store_lines<SP_K>(A.out[col] + orow, tb, T, vo, r, whole);
    };
    auto putb = [&](int col, const bool (&b)[SP_K]) {
      if (A.flag[col]) sp_put_bytes(A.flag[col] + orow, tb, T, v4, b);
    };
    auto pc_at = [&](int p) { return sP[sp_slot(p)]; };
    double r[SP_K], thr[SP_K];
    bool b[SP_K], vcf[SP_K], pbf[SP_K], cumf[SP_K], cums[SP_K], accl[SP_K], accs[SP_K];
    const int AW = A.accel_w;
    // condition bits of candles tb - 31 .. tb + 4 (bit u <-> candle tb - 31 + u;
    // before the row and missing ratios: 0): VR >= VC and VR >= 0.8 VC
    uint64_t m1 = 0, m8 = 0;
    {
      // candles pb - 32 .. pb + 3 from 9 dwords of bytes: the low bit of each
      // byte gathered into a nibble by one multiply (the 4 partial products'
      // bits never meet), bit j <-> candle pb - 32 + j
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const uint32_t wd = sCB[(pb - SP_H) / 4 + i];
        const uint32_t n1 = (((wd & 0x01010101u) * 0x204081u) >> 21) & 0xFu;
        const uint32_t n8 = ((((wd >> 1) & 0x01010101u) * 0x204081u) >> 21) & 0xFu;
        m1 |= (uint64_t)n1 << (4 * i);
        m8 |= (uint64_t)n8 << (4 * i);
      }
      m1 = (m1 >> 1) | ((uint64_t)(vr_next >= VC) << 35);
      m8 = (m8 >> 1) | ((uint64_t)(vr_next >= vc8) << 35);
    }
    // bits of the window of w candles ending at candle tb + e (e <= 4)
    auto win_bits = [&](uint64_t m, int e, int w) { return (m >> (31 + e - w + 1)) & ((1ull << w) - 1ull); };
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      const int t = tb + k, p = pb + k;
      // diff(VR, 3) and its first difference (t - 3 < 0: NaN)
      const double d3 = vr[k] - (t >= 3 ? sVR[sp_slot(p - 3)] : qnan());
      const double d3p = (t >= 1 ? sVR[sp_slot(p - 1)] : qnan()) - (t >= 4 ? sVR[sp_slot(p - 4)] : qnan());
      r[k] = d3;
      thr[k] = d3 - (t >= 1 ? d3p : qnan());
    }
    put(BQ_SPIKE_VOL_RATIO_SLOPE_3, r);
    put(BQ_SPIKE_VOL_RATIO_ACCEL, thr);
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      const int t = tb + k, p = pb + k;
      // volume_cluster_flag: count of (VR >= VC) over the cluster window
      // (min_periods 1), base = count >= min & cond; "last": base & ~base[t+1]
      auto base_at = [&](int j) {   // candle t + j, j in -1 .. 1
        if (t + j >= T || t + j < 0) return false;
        const int cnt = __popcll(win_bits(m1, k + j, A.cluster_w));
        return cnt >= A.cluster_min && ((m1 >> (31 + k + j)) & 1ull);
      };
      const bool b0 = base_at(0);
      vcf[k] = A.mode == 0 ? (b0 && !base_at(1)) : (A.mode == 1 ? (b0 && !base_at(-1)) : b0);
      // price break against the ffilled dynamic threshold
      const int i = lv[k];
      const double th = i < 0 ? qnan() : (i >= t0 - SP_H ? sTP[sp_slot(i - t0 + SP_H)] : sTV);
      thr[k] = th;
      const double pc = pc_at(p), pca = fabs(pc);
      pbf[k] = pca >= th;
      // cumulative break: 3-bar sums of the positive / negative moves while
      // the 8/10-scaled cluster condition held in the window (NaN max -> True)
      const double cp = sp_window<false>(t, A.cw, [&](int j) {
        const double x = pc_at(p + j);
        return x < 0.0 ? 0.0 : x;
      });
      const double cn = sp_window<false>(t, A.cw, [&](int j) {
        const double x = pc_at(p + j);
        return fabs(x > 0.0 ? 0.0 : x);
      });
      // max(VR >= VC * 0.8) over the window, min_periods = window
      const double vm = t < A.cw - 1 ? qnan() : (win_bits(m8, k, A.cw) != 0 ? 1.0 : 0.0);
      const bool vol_cond = vm != vm || vm != 0.0;
      cumf[k] = (cp >= A.cum_thr) && vol_cond;
      cums[k] = (cn >= A.cum_thr) && vol_cond;
      // acceleration
      const double vd = vr[k] - (t >= AW ? sVR[sp_slot(p - AW)] : qnan());
      const bool acc = (vd >= A.accel_vd) && (pca >= A.accel_pc);
      accl[k] = acc && (pc > 0.0);
      accs[k] = acc && (pc < 0.0);
    }
    putb(BQ_SPIKE_VOLUME_CLUSTER_FLAG, vcf);
    putb(BQ_SPIKE_PRICE_BREAK_FLAG, pbf);
    put(BQ_SPIKE_PRICE_BREAK_THRESHOLD, thr);
    putb(BQ_SPIKE_CUM_BREAK_FLAG, cumf);
    putb(BQ_SPIKE_CUM_BREAK_SHORT_FLAG, cums);
    putb(BQ_SPIKE_ACCEL_FLAG, accl);
    putb(BQ_SPIKE_ACCEL_SHORT_FLAG, accs);
    const double th_last = thr[SP_K - 1];   // the ffilled threshold at the lane's last candle
    bool lp[SP_K], ls[SP_K];
#pragma unroll
    for (int k = 0; k < SP_K; ++k) {
      const double bsp = fabs(c[k] - o[k]) / (o[k] + SP_EPS);
      const bool combo = A.both ? (vcf[k] && pbf[k]) : (vcf[k] || pbf[k]);
      bool a = combo || cumf[k] || accl[k];
      if (A.bullish) a = a && (c[k] > o[k]);
      if (A.body_min > 0.0) a = a && (bsp >= A.body_min);
      lp[k] = a;
      bool s = (combo || cums[k] || accs[k]) && (c[k] < o[k]);
      if (A.body_min > 0.0) s = s && (bsp >= A.body_min);
      ls[k] = s;
      r[k] = qnan();
      b[k] = false;
    }
    putb(BQ_SPIKE_LABEL_PRE, lp);
    putb(BQ_SPIKE_LABEL_SHORT_PRE, ls);
    put(BQ_SPIKE_EARLY_PROBA, r);
    putb(BQ_SPIKE_EARLY_AUG_FLAG, b);

    if (t0 + SP_TT >= T) break;
    __syncthreads();
    if (pb >= SP_TT) {
#pragma unroll
      for (int k = 0; k < SP_K; ++k) {
        const int a = sp_slot(pb + k), d = sp_slot(pb + k - SP_TT);
        sF[d] = sF[a];
        sP[d] = sP[a];
        sVR[d] = sVR[a];
        sTP[d] = sTP[a];
      }
      sCB[(pb - SP_TT) / 4] = sCB[pb / 4];
    }
    if (tid == SP_NT - 1) {
      sCar = lv[SP_K - 1];
      sTV = th_last;
    }
    __syncthreads();
  }
}

}  // namespace bq

namespace {
bool sp_aligned(const void* p, unsigned a) { return (((uintptr_t)p) & (a - 1)) == 0; }
}

static int spike_base_launch(const double* const* in, int nin, int64_t S, int64_t T, int64_t ld_in,
                             int32_t base_window, int32_t streak_length, double* const* out_f, uint8_t* const* out_b,
                             double* const* out_sd, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!in || !out_f || !out_b || S < 0 || T < 0 || ld_in < T || ld_out < T || T > 0x7fffffff - SP_TT ||
      S > 0x7fffffff || base_window < 1 || base_window > SP_H - 2 || streak_length < 1 || streak_length > SP_H - 2)
    return BQ_EINVAL;
  SpikeBaseArgs A;
  memset(&A, 0, sizeof(A));
  for (int f = 0; f < nin; ++f) {
    if (!in[f]) return BQ_EINVAL;
    A.in[f] = in[f];
  }
  const bool tp = out_sd != nullptr;
  if (tp)
    for (int c = 0; c < BQ_NUM_SPIKE_STD; ++c) A.sd[c] = out_sd[c];
  for (int c = 0; c < BQ_NUM_SPIKE_BASE_F; ++c) A.out[c] = out_f[c];
  for (int c = 0; c < BQ_NUM_SPIKE_BASE_B; ++c) A.flag[c] = out_b[c];
  if (S == 0 || T == 0) return BQ_OK;
  A.S = S;
  A.T = (int)T;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.w = base_window;
  A.n = streak_length;
  int vin = (ld_in % 2) == 0, vout = (ld_out % 2) == 0, vb = (ld_out % 4) == 0;
  for (int f = 0; f < nin; ++f) vin &= sp_aligned(in[f], 16);
  for (int c = 0; c < BQ_NUM_SPIKE_BASE_F; ++c)
    if (out_f[c]) vout &= sp_aligned(out_f[c], 16);
  for (int c = 0; c < BQ_NUM_SPIKE_STD; ++c)
    if (A.sd[c]) vout &= sp_aligned(A.sd[c], 16);
  for (int c = 0; c < BQ_NUM_SPIKE_BASE_B; ++c)
    if (out_b[c]) vb &= sp_aligned(out_b[c], 4);
  if (tp && base_window == 12 && streak_length == 3)   // SpikeParams' defaults
    hipLaunchKernelGGL((spike_base_kernel<true, 12, 3>), dim3((unsigned)S), dim3(SP_NT), 0, (hipStream_t)stream, A, vin,
                       vout, vb);
  else if (tp)
    hipLaunchKernelGGL(spike_base_kernel<true>, dim3((unsigned)S), dim3(SP_NT), 0, (hipStream_t)stream, A, vin, vout,
                       vb);
  else
    hipLaunchKernelGGL(spike_base_kernel<false>, dim3((unsigned)S), dim3(SP_NT), 0, (hipStream_t)stream, A, vin, vout,
                       vb);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

extern "C" int bq_spike_base(const double* const* in, int64_t S, int64_t T, int64_t ld_in, int32_t base_window,
                             int32_t streak_length, double* const* out_f, uint8_t* const* out_b, int64_t ld_out,
                             void* stream) {
  return spike_base_launch(in, bq::SB_NIN, S, T, ld_in, base_window, streak_length, out_f, out_b, nullptr, ld_out,
                           stream);
}

extern "C" int bq_spike_base_std(const double* const* in, int64_t S, int64_t T, int64_t ld_in, int32_t base_window,
                                 int32_t streak_length, double* const* out_f, uint8_t* const* out_b,
                                 double* const* out_sd, int64_t ld_out, void* stream) {
  if (!out_sd) return BQ_EINVAL;
  return spike_base_launch(in, bq::SB_PSTD, S, T, ld_in, base_window, streak_length, out_f, out_b, out_sd, ld_out,
                           stream);
}

extern "C" int bq_spike_flags(const double* const* in, const double* vcmr, const double* pbbt, int64_t S, int64_t T,
                              int64_t ld_in, const bq_spike_params* p, double* const* out_f, uint8_t* const* out_b,
                              int64_t ld_out, void* stream) {
  using namespace bq;
  if (!in || !vcmr || !pbbt || !p || !out_f || !out_b || S < 0 || T < 0 || ld_in < T || ld_out < T ||
      T > 0x7fffffff - SP_TT || S > 0x7fffffff)
    return BQ_EINVAL;
  if (p->volume_cluster_window < 1 || p->volume_cluster_window > SP_H - 2 || p->cumulative_price_window < 2 ||
      p->cumulative_price_window > SP_H - 2 || p->accel_volume_deriv_window < 0 ||
      p->accel_volume_deriv_window > SP_H - 2 || p->label_mode < 0 || p->label_mode > 2)
    return BQ_EINVAL;
  SpikeFlagArgs A;
  memset(&A, 0, sizeof(A));
  for (int f = 0; f < SF_NIN; ++f) {
    if (!in[f]) return BQ_EINVAL;
    A.in[f] = in[f];
  }
  A.vcmr = vcmr;
  A.pbbt = pbbt;
  for (int c = 0; c < BQ_NUM_SPIKE_FLAG_F; ++c) A.out[c] = out_f[c];
  for (int c = 0; c < BQ_NUM_SPIKE_FLAG_B; ++c) A.flag[c] = out_b[c];
  if (S == 0 || T == 0) return BQ_OK;
  A.S = S;
  A.T = (int)T;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.cluster_w = p->volume_cluster_window;
  A.cluster_min = p->volume_cluster_min_count;
  A.cw = p->cumulative_price_window;
  A.accel_w = p->accel_volume_deriv_window;
  A.mode = p->label_mode;
  A.both = p->require_both_patterns;
  A.bullish = p->require_bullish_spike;
  A.cum_thr = p->cumulative_price_threshold;
  A.accel_vd = p->accel_volume_deriv_min;
  A.accel_pc = p->accel_price_change_min;
  A.body_min = p->body_size_pct_min;
  int vin = (ld_in % 2) == 0, vout = (ld_out % 2) == 0, vb = (ld_out % 4) == 0;
  for (int f = 0; f < SF_NIN; ++f) vin &= sp_aligned(in[f], 16);
  for (int c = 0; c < BQ_NUM_SPIKE_FLAG_F; ++c)
    if (out_f[c]) vout &= sp_aligned(out_f[c], 16);
  for (int c = 0; c < BQ_NUM_SPIKE_FLAG_B; ++c)
    if (out_b[c]) vb &= sp_aligned(out_b[c], 4);
  hipLaunchKernelGGL(spike_flags_kernel, dim3((unsigned)S), dim3(SP_NT), 0, (hipStream_t)stream, A, vin, vout, vb);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
