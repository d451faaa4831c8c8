// Sequential per-symbol state machines on a [S][T] panel (lane = symbol).
//
//   bq_supertrend: pybinbot Indicators.set_supertrend(df, multiplier=3.0) as
//   called by Coinrule.supertrend_swing_reversal
//   (strategies/coinrule/coinrule.py:140-160, "period adjusted to 10"), which
//   reads bool(df["supertrend"].iloc[-1]). pybinbot is absent, so
//   the recurrence is the restatement in oracle/indicators_ref.py:supertrend:
//     hl2 = (high + low) / 2; upper = hl2 + m * ATR; lower = hl2 - m * ATR
//     trend[0] = up; for t >= 1:
//       close[t] > upper[t-1] -> up;  close[t] < lower[t-1] -> down;
//       otherwise keep the trend, and hold the band on the trend's side
//       (up: lower[t] = max(lower[t], lower[t-1]); down: upper[t] =
//       min(upper[t], upper[t-1])).
//   ATR (TR.rolling(period).mean(), the `atr` restatement) comes in as an
//   input column so the kernel only runs the comparisons; NaN bands in the
//   warm-up compare false, so the trend holds its initial `up` state.
//
// Mapping: one wave = 64 symbols; chunks of ST_CT candles are read coalesced
// and transposed through LDS (bq_device.h stage_*); the next chunk's loads are
// in flight while the current chunk's recurrence runs.
#include "bq_device.h"
#include "binquant_amd.h"

namespace bq {

constexpr int ST_CT = 16;   // candles per staged chunk

struct StArgs {
  const double *h, *l, *c, *atr;
  uint8_t* up;
  double *upper, *lower;
  int64_t S, ld_in, ld_out;
  int T;
  double mult;
};

__global__ __launch_bounds__(WAVE) void supertrend_kernel(const StArgs A) {
  __shared__ double sX[4][ST_CT * STG_PITCH];   // h, l, c, atr; then upper, lower, trend
  const int lane = threadIdx.x;
  const int64_t sym0 = (int64_t)blockIdx.x * WAVE;
  const int T = A.T;
  double rh[ST_CT], rl[ST_CT], rc[ST_CT], ra[ST_CT];
  stage_load<ST_CT>(A.h, A.ld_in, sym0, A.S, 0, T, lane, rh);
  stage_load<ST_CT>(A.l, A.ld_in, sym0, A.S, 0, T, lane, rl);
  stage_load<ST_CT>(A.c, A.ld_in, sym0, A.S, 0, T, lane, rc);
  stage_load<ST_CT>(A.atr, A.ld_in, sym0, A.S, 0, T, lane, ra);
  bool up = true;
  double up_p = qnan(), lo_p = qnan();
  for (int t0 = 0; t0 < T; t0 += ST_CT) {
    stage_put<ST_CT>(sX[0], lane, rh);
    stage_put<ST_CT>(sX[1], lane, rl);
    stage_put<ST_CT>(sX[2], lane, rc);
    stage_put<ST_CT>(sX[3], lane, ra);
    __syncthreads();
    // prefetch the next chunk (unconditional: past T the clamped loads give
    // NaN that is never used; no branch keeps the loop's waits counted)
    stage_load<ST_CT>(A.h, A.ld_in, sym0, A.S, t0 + ST_CT, T, lane, rh);
    stage_load<ST_CT>(A.l, A.ld_in, sym0, A.S, t0 + ST_CT, T, lane, rl);
    stage_load<ST_CT>(A.c, A.ld_in, sym0, A.S, t0 + ST_CT, T, lane, rc);
    stage_load<ST_CT>(A.atr, A.ld_in, sym0, A.S, t0 + ST_CT, T, lane, ra);
    const int n = min(ST_CT, T - t0);
    for (int j = 0; j < n; ++j) {
      const int i = j * STG_PITCH + lane;
      const double hl2 = (sX[0][i] + sX[1][i]) / 2.0;
      const double c = sX[2][i], m_atr = A.mult * sX[3][i];
      double bu = hl2 + m_atr, bl = hl2 - m_atr;
      if (t0 + j > 0) {
        if (c > up_p) up = true;
        else if (c < lo_p) up = false;
        else {
          if (up && bl < lo_p) bl = lo_p;
          if (!up && bu > up_p) bu = up_p;
        }
      }
      up_p = bu;
      lo_p = bl;
      sX[0][i] = bu;
      sX[1][i] = bl;
      sX[2][i] = up ? 1.0 : 0.0;
    }
    __syncthreads();
    stage_store<ST_CT>(sX[0], A.upper, A.ld_out, sym0, A.S, t0, T, lane);   // null: dropped
    stage_store<ST_CT>(sX[1], A.lower, A.ld_out, sym0, A.S, t0, T, lane);
    stage_store<ST_CT>(sX[2], A.up, A.ld_out, sym0, A.S, t0, T, lane);
    __syncthreads();
  }
}

}  // namespace bq

extern "C" int bq_supertrend(const double* const* hlca, int64_t S, int64_t T, int64_t ld_in, double multiplier,
                             uint8_t* up, double* upper, double* lower, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!hlca || !up || S < 0 || T < 0 || ld_in < T || ld_out < T || T > 0x7fffffff || !(multiplier == multiplier))
    return BQ_EINVAL;
  if (ld_out > BQ_MAX_ROLL_LD) return BQ_EINVAL;   // 32-bit buffer offsets over a wave's 64 rows
  for (int i = 0; i < 4; ++i)
    if (!hlca[i]) return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  StArgs A;
  A.h = hlca[0];
  A.l = hlca[1];
  A.c = hlca[2];
  A.atr = hlca[3];
  A.up = up;
  A.upper = upper;
  A.lower = lower;
  A.S = S;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.mult = multiplier;
  const unsigned blocks = (unsigned)((S + WAVE - 1) / WAVE);
  hipLaunchKernelGGL(supertrend_kernel, dim3(blocks), dim3(WAVE), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
