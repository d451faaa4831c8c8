// Fused activity-burst stages (gfx950): ActivityBurstPump.compute_indicators
// (strategies/activity_burst_pump.py:51-158) on an [S][T] panel in two
// streaming passes around the score's rolling quantile:
//
//   bq_burst_features  every column of :58-133 from open / high / low / close /
//                      volume (/ quote volume) and the two baseline medians
//                      (bq_rolling_batch): the safe baselines, the ratios,
//                      price_jump, range / body / close-to-high fractions,
//                      recent_up_closes ((close > close.shift(1)).rolling(3)
//                      .sum(), formed here), the six flags, the score — and a
//                      byte per candle with the AND of the six flags;
//   bq_burst_qualify   raw = flags & (score >= threshold.fillna(0)), then
//                      raw & ~raw.shift(1).rolling(3, min_periods=1).max()
//                      .fillna(False)                                (:140-156).
//
// Staged, the pipeline ran five element-wise / window launches that wrote and
// re-read the safe baselines, the fractions, the flags and the raw signal.
// Every expression is the reference's, in its operation order (the IEEE
// operations of the staged JIT programs), so each column equals the staged
// pipeline bit for bit. One thread = 4 consecutive candles of a row (16-byte
// loads, whole-line stores, 4-byte flag stores); the few look-back values
// (close t-1 .. t-3, raw t-3 .. t-1) are re-read from L1 / L2.
#include "bq_device.h"
#include "binquant_amd.h"

#include <stdint.h>
#include <string.h>

namespace bq {

constexpr int BU_NT = 256;
constexpr int BU_K = 4;
constexpr int BU_TT = BU_NT * BU_K;

enum { BU_O = 0, BU_H, BU_L, BU_C, BU_V, BU_Q, BU_MEDV, BU_MEDQ, BU_NIN };

struct BurstArgs {
  const double* in[BU_NIN];          // Q / MEDQ NULL without quote volume
  double* out[BQ_NUM_BURST_F];       // float columns (NULL: skip)
  uint8_t* flag[BQ_NUM_BURST_B];     // bool columns (NULL: skip)
  uint8_t* all;                      // AND of the six flags (for bq_burst_qualify)
  int64_t S, ld_in, ld_out;
  int T, has_q, min_up;
  double mb, vol_mult, qv_mult, price_thr, min_range, min_body, max_cth;
};

typedef double bu_dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void bu_load(const double* __restrict__ row, int tb, int T, bool vec, double (&x)[BU_K]) {
  if (vec && tb + BU_K <= T) {
    const bu_dbl2* p = reinterpret_cast<const bu_dbl2*>(row + tb);
    const bu_dbl2 a = p[0], b = p[1];
    x[0] = a.x;
    x[1] = a.y;
    x[2] = b.x;
    x[3] = b.y;
  } else {
#pragma unroll
    for (int k = 0; k < BU_K; ++k) x[k] = tb + k < T ? row[tb + k] : qnan();
  }
}

// 4 flags of consecutive candles: one 4-byte store when the row offset allows
__device__ __forceinline__ void bu_put_bytes(uint8_t* __restrict__ row, int tb, int T, bool vec4, const bool (&b)[BU_K]) {
  if (vec4 && tb + BU_K <= T) {
    const uint32_t w = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    *reinterpret_cast<uint32_t*>(row + tb) = w;
  } else {
#pragma unroll
    for (int k = 0; k < BU_K; ++k)
      if (tb + k < T) row[tb + k] = b[k] ? 1 : 0;
  }
}

__device__ __forceinline__ double clip_lo(double x, double lo) { return x < lo ? lo : x; }   // NaN stays

__global__ __launch_bounds__(BU_NT) void burst_features_kernel(const BurstArgs A, int vin, int vout, int vb) {
  const int T = A.T, nch = (T + BU_TT - 1) / BU_TT;
  const int64_t sym = blockIdx.x / nch;
  const int ch = (int)(blockIdx.x % nch), tb = ch * BU_TT + BU_K * threadIdx.x;
  const int64_t irow = sym * A.ld_in, orow = sym * A.ld_out;
  const bool hq = A.has_q != 0;
  double o[BU_K], h[BU_K], l[BU_K], c[BU_K], v[BU_K], q[BU_K], mv[BU_K], mq[BU_K];
  bu_load(A.in[BU_O] + irow, tb, T, vin, o);
  bu_load(A.in[BU_H] + irow, tb, T, vin, h);
  bu_load(A.in[BU_L] + irow, tb, T, vin, l);
  bu_load(A.in[BU_C] + irow, tb, T, vin, c);
  bu_load(A.in[BU_V] + irow, tb, T, vin, v);
  bu_load(A.in[BU_MEDV] + irow, tb, T, vin, mv);
  if (hq) {
    bu_load(A.in[BU_Q] + irow, tb, T, vin, q);
    bu_load(A.in[BU_MEDQ] + irow, tb, T, vin, mq);
  }
  // close t-3 .. t-1 of the first candle (NaN before the row)
  double cp[BU_K + 3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int t = tb - 3 + j;
    cp[j] = t >= 0 && t < T ? A.in[BU_C][irow + t] : qnan();
  }
#pragma unroll
  for (int k = 0; k < BU_K; ++k) cp[3 + k] = c[k];
  const double mb = A.mb;
  const bool whole = (ch + 1) * BU_TT <= T, vo = vout != 0, v4 = vb != 0;
  auto put = [&](int col, const double (&r)[BU_K]) {
    if (A.out[col]) store_lines<BU_K>(A.out[col] + orow, tb, T, vo, r, whole);
  };
  auto putb = [&](int col, const bool (&b)[BU_K]) {
    if (A.flag[col]) bu_put_bytes(A.flag[col] + orow, tb, T, v4, b);
  };
  double bvs[BU_K], vr[BU_K], bqs[BU_K], qvr[BU_K], pj[BU_K], rf[BU_K], bf[BU_K], cth[BU_K], ruc[BU_K], sc[BU_K];
  bool bull[BU_K], vsp[BU_K], qsp[BU_K], pjf[BU_K], ref[BU_K], bqf[BU_K], tqf[BU_K], all[BU_K];
#pragma unroll
  for (int k = 0; k < BU_K; ++k) {
    const int t = tb + k;
    bvs[k] = clip_lo(mv[k], mb);
    vr[k] = v[k] / bvs[k];
    bqs[k] = hq ? clip_lo(mq[k], mb) : bvs[k];
    qvr[k] = hq ? q[k] / bqs[k] : 1.0;
    const double pc = cp[2 + k];
    const double prev_close = clip_lo(pc, mb);
    const double range = clip_lo(h[k] - l[k], mb);
    const double body = fabs(c[k] - o[k]);
    pj[k] = (c[k] - pc) / prev_close;
    rf[k] = range / clip_lo(c[k], mb);
    bf[k] = body / range;
    cth[k] = (h[k] - c[k]) / range;
    bull[k] = c[k] > o[k];
    // (close > close.shift(1)).rolling(3).sum(): the up moves at t-2, t-1, t
    const int n_up = (cp[1 + k] > cp[k]) + (cp[2 + k] > cp[1 + k]) + (cp[3 + k] > cp[2 + k]);
    ruc[k] = t >= 2 ? (double)n_up : qnan();
    vsp[k] = v[k] > (A.vol_mult * bvs[k]);
    qsp[k] = hq ? q[k] > (A.qv_mult * bqs[k]) : true;
    pjf[k] = pj[k] > A.price_thr;
    ref[k] = rf[k] > A.min_range;
    bqf[k] = bull[k] & (bf[k] > A.min_body) & (cth[k] < A.max_cth);
    tqf[k] = ruc[k] >= (double)A.min_up;
    const double pjc = clip_lo(pj[k], 0.0);
    sc[k] = hq ? vr[k] * qvr[k] * pjc * (1 + bf[k]) : vr[k] * pjc;
    all[k] = vsp[k] & qsp[k] & pjf[k] & ref[k] & bqf[k] & tqf[k];
  }
  put(BQ_BURST_BASELINE_VOLUME_SAFE, bvs);
  put(BQ_BURST_VOLUME_RATIO, vr);
  put(BQ_BURST_BASELINE_QUOTE_VOLUME_SAFE, bqs);
  put(BQ_BURST_QUOTE_VOLUME_RATIO, qvr);
  put(BQ_BURST_PRICE_JUMP, pj);
  put(BQ_BURST_RANGE_FRAC, rf);
  put(BQ_BURST_BODY_FRAC, bf);
  put(BQ_BURST_CLOSE_TO_HIGH, cth);
  put(BQ_BURST_RECENT_UP_CLOSES, ruc);
  put(BQ_BURST_SCORE, sc);
  putb(BQ_BURST_IS_BULLISH, bull);
  putb(BQ_BURST_VOL_SPIKE, vsp);
  putb(BQ_BURST_QUOTE_VOL_SPIKE, qsp);
  putb(BQ_BURST_PRICE_JUMP_FLAG, pjf);
  putb(BQ_BURST_RANGE_EXPANSION_FLAG, ref);
  putb(BQ_BURST_BODY_QUALITY_FLAG, bqf);
  putb(BQ_BURST_TREND_QUALITY_FLAG, tqf);
  if (A.all) bu_put_bytes(A.all + orow, tb, T, v4, all);
}

struct QualifyArgs {
  const double *score, *thr;
  const uint8_t* all;
  uint8_t* out;
  int64_t ld_in, ld_b;   // row strides: score / threshold, bytes
  int T, cooldown;
};

// raw[t] = all[t] & (score[t] >= fillna(thr[t], 0)); qualified = raw & no raw
// in [t - cooldown, t - 1]
__global__ __launch_bounds__(BU_NT) void burst_qualify_kernel(const QualifyArgs A, int vb) {
  constexpr int MAXCD = 8;
  const int T = A.T, nch = (T + BU_TT - 1) / BU_TT, CD = A.cooldown;
  const int64_t sym = blockIdx.x / nch;
  const int tb = (int)(blockIdx.x % nch) * BU_TT + BU_K * threadIdx.x;
  const double* __restrict__ s = A.score + sym * A.ld_in;
  const double* __restrict__ th = A.thr + sym * A.ld_in;
  const uint8_t* __restrict__ al = A.all + sym * A.ld_b;
  auto raw = [&](int t) -> bool {
    if (t < 0 || t >= T) return false;
    const double tv = th[t];
    return al[t] != 0 && s[t] >= (tv != tv ? 0.0 : tv);
  };
  bool r[MAXCD + BU_K];
#pragma unroll
  for (int j = 0; j < MAXCD + BU_K; ++j) r[j] = j >= MAXCD - CD ? raw(tb - MAXCD + j) : false;
  bool q[BU_K];
#pragma unroll
  for (int k = 0; k < BU_K; ++k) {
    bool recent = false;
#pragma unroll
    for (int j = 0; j < MAXCD; ++j) recent |= j >= MAXCD - CD && r[k + j];
    q[k] = r[MAXCD + k] & !recent;
  }
  bu_put_bytes(A.out + sym * A.ld_b, tb, T, vb != 0, q);
}

}  // namespace bq

extern "C" int bq_burst_features(const double* const* in, int64_t S, int64_t T, int64_t ld_in,
                                 const bq_burst_params* p, double* const* out_f, uint8_t* const* out_b,
                                 uint8_t* all_flags, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!in || !p || !out_f || !out_b || S < 0 || T < 0 || ld_in < T || ld_out < T || T > 0x7fffffff - BU_TT ||
      S * ((T + BU_TT - 1) / BU_TT) > 0x7fffffff)
    return BQ_EINVAL;
  BurstArgs A;
  memset(&A, 0, sizeof(A));
  const bool hq = in[BU_Q] != nullptr;
  if (hq != (in[BU_MEDQ] != nullptr)) return BQ_EINVAL;
  for (int f = 0; f < BU_NIN; ++f) {
    if (!in[f] && f != BU_Q && f != BU_MEDQ) return BQ_EINVAL;
    A.in[f] = in[f];
  }
  for (int c = 0; c < BQ_NUM_BURST_F; ++c) A.out[c] = out_f[c];
  for (int c = 0; c < BQ_NUM_BURST_B; ++c) A.flag[c] = out_b[c];
  A.all = all_flags;
  if (S == 0 || T == 0) return BQ_OK;
  A.S = S;
  A.T = (int)T;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.has_q = hq;
  A.min_up = p->min_recent_up_closes;
  A.mb = p->min_baseline_volume;
  A.vol_mult = p->volume_multiplier;
  A.qv_mult = p->quote_volume_multiplier;
  A.price_thr = p->price_threshold;
  A.min_range = p->min_range_frac;
  A.min_body = p->min_body_frac;
  A.max_cth = p->max_close_to_high;
  auto aligned = [](const void* q, unsigned a) { return (((uintptr_t)q) & (a - 1)) == 0; };
  int vin = (ld_in % 2) == 0, vout = (ld_out % 2) == 0, vb = (ld_out % 4) == 0;
  for (int f = 0; f < BU_NIN; ++f)
    if (in[f]) vin &= aligned(in[f], 16);
  for (int c = 0; c < BQ_NUM_BURST_F; ++c)
    if (out_f[c]) vout &= aligned(out_f[c], 16);
  for (int c = 0; c < BQ_NUM_BURST_B; ++c)
    if (out_b[c]) vb &= aligned(out_b[c], 4);
  if (all_flags) vb &= aligned(all_flags, 4);
  const dim3 grid((unsigned)(S * ((T + BU_TT - 1) / BU_TT)));
  hipLaunchKernelGGL(burst_features_kernel, grid, dim3(BU_NT), 0, (hipStream_t)stream, A, vin, vout, vb);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

extern "C" int bq_burst_qualify(const double* score, const double* threshold, const uint8_t* all_flags, int64_t S,
                                int64_t T, int64_t ld_in, int64_t ld_b, int32_t cooldown_bars, uint8_t* qualified,
                                void* stream) {
  using namespace bq;
  if (!score || !threshold || !all_flags || !qualified || S < 0 || T < 0 || ld_in < T || ld_b < T ||
      T > 0x7fffffff - BU_TT || S * ((T + BU_TT - 1) / BU_TT) > 0x7fffffff || cooldown_bars < 0 || cooldown_bars > 8)
    return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  QualifyArgs A;
  A.score = score;
  A.thr = threshold;
  A.all = all_flags;
  A.out = qualified;
  A.ld_in = ld_in;
  A.ld_b = ld_b;
  A.T = (int)T;
  A.cooldown = cooldown_bars;
  const int vb = (ld_b % 4) == 0 && (((uintptr_t)qualified) & 3u) == 0;
  const dim3 grid((unsigned)(S * ((T + BU_TT - 1) / BU_TT)));
  hipLaunchKernelGGL(burst_qualify_kernel, grid, dim3(BU_NT), 0, (hipStream_t)stream, A, vb);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
