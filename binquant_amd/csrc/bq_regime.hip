// Regime annotation, candidate scoring and portfolio selection on the device
// (SURVEY §8f rows 2 and 3): element-wise over symbols / candidates, plus a
// segmented arg-max per cohort.
//
//   bq_micro_regime   RegimeTransitionDetector._annotate_symbol_regime
//                     (market_regime/regime_transitions.py:162-232) and
//                     _symbol_transition_event (:251-277), per symbol.
//   bq_context_score  RuleBasedMarketContextModel.evaluate
//                     (market_regime/context_scoring.py:13-114) and
//                     SignalContextScorer.adjust_score
//                     (market_regime/signal_context_scorer.py:15-28), per
//                     candidate, against one LiveMarketContext.
//   bq_cohort_select  the winner of LiquidationSweepPortfolioSelector /
//                     GradualGainerPortfolioSelector._dispatch_winner
//                     (strategies/liquidation_sweep_pump.py:38-87,
//                     strategies/gradual_gainer_retest.py:33-70): per cohort
//                     the accepted candidate with the largest
//                     (rank_score, symbol), a re-submitted symbol keeping its
//                     latest best score.
// Every formula keeps the reference's operation order (the file is built with
// -ffp-contract=off), so results equal the Python floats bit for bit.
#include "bq_device.h"
#include "binquant_amd.h"

namespace bq {

__device__ __forceinline__ double clampd(double x, double lo = -1.0, double hi = 1.0) {
  // shared/utils.py:12-13: max(low, min(high, value))
  const double m = x < hi ? x : hi;   // Python min(high, x): x if x < high else high
  return m > lo ? m : lo;              // Python max(low, m): m if m > low else low
}
// shared/utils.py:16-17 max(0.0, value): value if value > 0.0 else 0.0 (-0.0 -> 0.0)
__device__ __forceinline__ double nneg(double x) { return x > 0.0 ? x : 0.0; }
__device__ __forceinline__ double pmin(double a, double b) { return b < a ? b : a; }   // Python min(a, b)

// ---- per-symbol micro regime ------------------------------------------------------
__global__ __launch_bounds__(256) void micro_regime_kernel(int64_t n, const double* __restrict__ trend,
                                                           const uint8_t* __restrict__ above20,
                                                           const uint8_t* __restrict__ above50,
                                                           const double* __restrict__ rs,
                                                           const double* __restrict__ bbw,
                                                           const double* __restrict__ atr,
                                                           const double* __restrict__ ret,
                                                           const int8_t* __restrict__ prev_regime,
                                                           const double* __restrict__ prev_strength,
                                                           int8_t* __restrict__ regime, double* __restrict__ strength,
                                                           int8_t* __restrict__ transition,
                                                           double* __restrict__ transition_strength) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double ts = trend[i], r = rs[i], bw = bbw[i], ap = atr[i];
  const double a20 = above20[i] ? 1.0 : 0.0, a50 = above50[i] ? 1.0 : 0.0;
  const double up = clampd(0.45 * nneg(ts * 30.0) + 0.2 * a20 + 0.15 * a50 + 0.2 * nneg(r * 20.0), 0.0, 1.0);
  const double down = clampd(0.45 * nneg(-ts * 30.0) + 0.2 * (1.0 - a20) + 0.15 * (1.0 - a50) + 0.2 * nneg(-r * 20.0),
                             0.0, 1.0);
  const double rng = clampd(0.38 * (1.0 - pmin(fabs(ts) * 30.0, 1.0)) + 0.34 * (1.0 - pmin(bw / 0.08, 1.0)) +
                                0.28 * (1.0 - pmin(ap / 0.04, 1.0)),
                            0.0, 1.0);
  const double vol = clampd(0.55 * pmin(ap / 0.05, 1.0) + 0.45 * pmin(bw / 0.12, 1.0), 0.0, 1.0);
  // Python max(a, b, c, d): the first of the largest
  double st = up;
  if (down > st) st = down;
  if (rng > st) st = rng;
  if (vol > st) st = vol;
  int8_t reg = BQ_MICRO_TRANSITIONAL;
  if (vol >= 0.72 && fabs(ret[i]) >= 0.015) reg = BQ_MICRO_VOLATILE;
  else if (up >= 0.52 && up >= down + 0.1) reg = BQ_MICRO_TREND_UP;
  else if (down >= 0.52 && down >= up + 0.1) reg = BQ_MICRO_TREND_DOWN;
  else if (rng >= 0.5) reg = BQ_MICRO_RANGE;
  const int8_t pr = prev_regime ? prev_regime[i] : (int8_t)-1;
  int8_t tr = -1;
  double tst = 0.0;
  if (pr >= 0 && pr != reg) {
    if (reg == BQ_MICRO_VOLATILE) tr = BQ_MT_VOLATILITY_EXPANSION;
    else if ((pr == BQ_MICRO_RANGE || pr == BQ_MICRO_TRANSITIONAL) && reg == BQ_MICRO_TREND_UP) tr = BQ_MT_BREAKOUT_UP;
    else if ((pr == BQ_MICRO_RANGE || pr == BQ_MICRO_TRANSITIONAL) && reg == BQ_MICRO_TREND_DOWN) tr = BQ_MT_BREAKDOWN;
    else if (pr == BQ_MICRO_TREND_DOWN && reg == BQ_MICRO_TREND_UP) tr = BQ_MT_RECOVERY;
    else if (pr == BQ_MICRO_TREND_UP && reg == BQ_MICRO_RANGE) tr = BQ_MT_MEAN_REVERSION;
    else if (reg == BQ_MICRO_TREND_UP) tr = BQ_MT_ENTERED_TREND_UP;
    else if (reg == BQ_MICRO_TREND_DOWN) tr = BQ_MT_ENTERED_TREND_DOWN;
    else if (reg == BQ_MICRO_RANGE) tr = BQ_MT_ENTERED_RANGE;
    else tr = BQ_MT_ENTERED_TRANSITIONAL;
    const double ps = prev_strength ? prev_strength[i] : 0.0;
    tst = clampd(st + fabs(st - ps) - 0.25, 0.0, 1.0);
  }
  regime[i] = reg;
  strength[i] = st;
  if (transition) transition[i] = tr;
  if (transition_strength) transition_strength[i] = tst;
}

// ---- candidate scoring against one context ------------------------------------------
__global__ __launch_bounds__(256) void context_score_kernel(int64_t n, const int8_t* __restrict__ direction,
                                                            const double* __restrict__ rs,
                                                            const double* __restrict__ trend,
                                                            const double* __restrict__ local_score,
                                                            const bq_context_scalars C, const bq_scorer_weights W,
                                                            double* __restrict__ out, int64_t ld_out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double* o = out + i;
  const double ls = local_score ? local_score[i] : 0.0;
  if (!C.present || !(C.confidence > 0.0)) {   // _empty_score: everything 0
    for (int k = 0; k < BQ_NUM_SCORE_FIELDS; ++k) o[k * ld_out] = 0.0;
    o[BQ_SC_ADJUSTED * ld_out] = ls + 0.0 * W.context_weight * (0.0 + (W.support_weight * 0.0) - (W.risk_weight * 0.0));
    return;
  }
  const int dir = direction[i];
  const double r = rs[i], t = trend[i];
  double breadth, btc_al, cross, over, dstress;
  if (dir == BQ_DIR_SHORT) {
    breadth = C.short_tailwind;
    btc_al = clampd(-C.btc_regime_score);
    cross = clampd(0.6 * (-r) + 0.4 * (-t));
    over = clampd(0.6 * nneg(-r) + 0.4 * nneg(-t), 0.0, 1.0);
    dstress = C.market_stress_score * 0.35;
  } else {
    breadth = C.long_tailwind;
    btc_al = clampd(C.btc_regime_score);
    cross = clampd(0.6 * r + 0.4 * t);
    over = clampd(0.6 * nneg(r) + 0.4 * nneg(t), 0.0, 1.0);
    dstress = -C.market_stress_score;
  }
  double sup = clampd(0.35 * breadth + 0.25 * btc_al + 0.25 * cross + 0.15 * dstress);
  double fol = clampd(0.45 * breadth + 0.3 * btc_al + 0.25 * cross);
  const double adv = clampd(0.55 * C.market_stress_score + 0.25 * nneg(-sup) + 0.2 * (1.0 - over), 0.0, 1.0);
  if (dir == BQ_DIR_LONG && breadth < 0.0 && over > 0.0) {
    sup = clampd(sup + 0.2 * over);
    fol = clampd(fol + 0.15 * over);
  }
  if (dir == BQ_DIR_SHORT && breadth < 0.0 && over > 0.0) sup = clampd(sup + 0.1 * over);
  o[BQ_SC_CONFIDENCE * ld_out] = C.confidence;
  o[BQ_SC_BREADTH * ld_out] = breadth;
  o[BQ_SC_BTC_ALIGNMENT * ld_out] = btc_al;
  o[BQ_SC_CROSS_ASSET * ld_out] = cross;
  o[BQ_SC_FOLLOWTHROUGH * ld_out] = fol;
  o[BQ_SC_ADVERSE * ld_out] = adv;
  o[BQ_SC_OVERRIDE * ld_out] = over;
  o[BQ_SC_SUPPORTIVENESS * ld_out] = sup;
  // SignalContextScorer.adjust_score
  o[BQ_SC_ADJUSTED * ld_out] =
      ls + C.confidence * W.context_weight * (fol + (W.support_weight * sup) - (W.risk_weight * adv));
}

// ---- cohort winners ---------------------------------------------------------------------
// order-preserving u64 key of a double (-0.0 folded onto +0.0: Python
// compares them equal, the symbol then decides)
__device__ __forceinline__ unsigned long long okey(double x) {
  if (x == 0.0) x = 0.0;
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}

__global__ __launch_bounds__(256) void cohort_score_kernel(int64_t n, const int32_t* __restrict__ cohort,
                                                           const uint8_t* __restrict__ accepted,
                                                           const double* __restrict__ score,
                                                           unsigned long long* __restrict__ best) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n || (accepted && !accepted[i])) return;
  atomicMax(best + cohort[i], okey(score[i]));
}

__global__ __launch_bounds__(256) void cohort_tie_kernel(int64_t n, const int32_t* __restrict__ cohort,
                                                         const uint8_t* __restrict__ accepted,
                                                         const double* __restrict__ score,
                                                         const int32_t* __restrict__ symbol_rank,
                                                         const unsigned long long* __restrict__ best,
                                                         unsigned long long* __restrict__ tie) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n || (accepted && !accepted[i])) return;
  const int c = cohort[i];
  if (okey(score[i]) != best[c]) return;
  // low word i + 1: a zero word means "no accepted candidate"; the largest
  // index wins a (score, symbol) tie (the later submission replaced it)
  atomicMax(tie + c, ((unsigned long long)(uint32_t)symbol_rank[i] << 32) | (unsigned long long)(uint32_t)(i + 1));
}

__global__ __launch_bounds__(256) void cohort_winner_kernel(int32_t n_cohorts, const unsigned long long* __restrict__ tie,
                                                            int64_t* __restrict__ winner) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n_cohorts) return;
  winner[c] = tie[c] ? (int64_t)(tie[c] & 0xffffffffull) - 1 : -1;
}

}  // namespace bq

extern "C" {

int bq_micro_regime(int64_t n, const double* trend, const uint8_t* above_ema20, const uint8_t* above_ema50,
                    const double* rs, const double* bb_width, const double* atr_pct, const double* return_pct,
                    const int8_t* prev_regime, const double* prev_strength, int8_t* regime, double* strength,
                    int8_t* transition, double* transition_strength, void* stream) {
  using namespace bq;
  if (n < 0 || !trend || !above_ema20 || !above_ema50 || !rs || !bb_width || !atr_pct || !return_pct || !regime ||
      !strength)
    return BQ_EINVAL;
  if (n == 0) return BQ_OK;
  hipLaunchKernelGGL(micro_regime_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                     trend, above_ema20, above_ema50, rs, bb_width, atr_pct, return_pct, prev_regime, prev_strength,
                     regime, strength, transition, transition_strength);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_context_score(int64_t n, const int8_t* direction, const double* rs, const double* trend,
                     const double* local_score, const bq_context_scalars* ctx, const bq_scorer_weights* weights,
                     double* out, int64_t ld_out, void* stream) {
  using namespace bq;
  if (n < 0 || !direction || !rs || !trend || !ctx || !weights || !out || ld_out < n) return BQ_EINVAL;
  if (n == 0) return BQ_OK;
  hipLaunchKernelGGL(context_score_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                     direction, rs, trend, local_score, *ctx, *weights, out, ld_out);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_cohort_select(int64_t n, const int32_t* cohort, const uint8_t* accepted, const double* score,
                     const int32_t* symbol_rank, int32_t n_cohorts, unsigned long long* scratch, int64_t* winner,
                     void* stream) {
  using namespace bq;
  if (n < 0 || n > 0x7fffffff || n_cohorts < 0 || (n > 0 && (!cohort || !score || !symbol_rank)) || !winner ||
      (n_cohorts > 0 && !scratch))
    return BQ_EINVAL;
  if (n_cohorts == 0) return BQ_OK;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(scratch, 0, (size_t)n_cohorts * 2 * sizeof(unsigned long long), st) != hipSuccess) return BQ_EHIP;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  if (n > 0) {
    hipLaunchKernelGGL(cohort_score_kernel, dim3(blocks), dim3(256), 0, st, n, cohort, accepted, score, scratch);
    hipLaunchKernelGGL(cohort_tie_kernel, dim3(blocks), dim3(256), 0, st, n, cohort, accepted, score, symbol_rank,
                       scratch, scratch + n_cohorts);
  }
  hipLaunchKernelGGL(cohort_winner_kernel, dim3((unsigned)((n_cohorts + 255) / 256)), dim3(256), 0, st, n_cohorts,
                     scratch + n_cohorts, winner);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
