// Rolling-window statistics with pandas semantics, for the strategy feature
// pipelines:
//
//   bq_rolling: x.shift(shift).rolling(window, min_periods).{quantile(q),
//               median(), mean(), sum()} — NaNs are skipped and counted out
//               of nobs, the result is NaN while nobs < min_periods.
//     quantile: pandas roll_quantile, linear interpolation
//               (vlow + (vhigh - vlow) * (q*(nobs-1) - idx)); q = 0 / 1 give
//               rolling min / max;
//     median:   pandas roll_median_c (mean of the two middle values for even
//               nobs);
//     mean:     sum / nobs with pandas' same-value rule;
//     sum:      Kahan-compensated like pandas add_sum / remove_sum, same-value
//               rule (value * nobs), 0 for an empty window when min_periods = 0;
//     var/std:  ddof 1, pandas' compensated Welford update, same-value rule -> 0.
//     Used by ActivityBurstPump.compute_indicators
//     (strategies/activity_burst_pump.py:58-63 median(19), :134-139
//     quantile(0.92, 80), :147-152 max(3)), LiquidationSweepPump.compute_pump_score
//     (strategies/liquidation_sweep_pump.py:218-245: mean(20), max/min(6),
//     quantile(0.80, 48)), FailedSpikeFade (quantile(0.85, 60)).
//
//   bq_ewm: x.ewm(alpha, adjust=False, min_periods).mean() with
//           ignore_na=False NaN gaps (the BTC left-merge of
//           liquidation_sweep_pump.py:255-267 and the Wilder ATR/RSI of
//           :215-217 and mean_reversion_fade.py:88-109).
//
// Mapping (bq_rolling): order statistics are not prefix-able, so each lane
// owns a run of SEG consecutive outputs of one symbol and keeps its window
// SORTED in LDS (lane-interleaved: element j of lane l at j*64 + l, so a wave's
// accesses hit 64 distinct banks). Per step it binary-searches the leaving and
// the entering value and shifts only the span between them. The window is
// rebuilt from the w values before each run (warm-up), so runs are
// independent: S * ceil(T / SEG) lanes in flight.
//
// Mapping (bq_ewm): lane = symbol, one sequential pass with pandas' exact
// update (bit-for-bit the pandas recursion).
#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

constexpr int RW_LANES = 64;           // one wave per workgroup
constexpr int RW_MAXW = BQ_MAX_ROLLING_WINDOW;
constexpr int RW_SEG = 256;            // outputs per lane

struct RollArgs {
  const double* x;
  double* out;
  int64_t S, ld_in, ld_out;
  int T, win, minp, shift, mode, nseg;
  double q;
};

// lane-interleaved sorted window
struct Win {
  double* base;   // LDS base of this wave's windows
  int lane, n;
  __device__ __forceinline__ double& at(int j) const { return base[j * RW_LANES + lane]; }
  // first index with at(i) >= v  (lower bound)
  __device__ __forceinline__ int lower(double v) const {
    int lo = 0, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (at(mid) < v) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  }
  __device__ __forceinline__ void insert(double v) {
    const int p = lower(v);
    for (int j = n; j > p; --j) at(j) = at(j - 1);
    at(p) = v;
    ++n;
  }
  __device__ __forceinline__ void erase(double v) {   // v is present
    const int p = lower(v);
    for (int j = p; j < n - 1; ++j) at(j) = at(j + 1);
    --n;
  }
  // erase `old` and insert `nw` with one shift of the span between them
  __device__ __forceinline__ void replace(double old, double nw) {
    const int po = lower(old);
    if (nw >= old) {
      // move elements (po, pn) one slot down, new value at pn-1
      int p = po;
      while (p + 1 < n && at(p + 1) < nw) {
        at(p) = at(p + 1);
        ++p;
      }
      at(p) = nw;
    } else {
      int p = po;
      while (p > 0 && at(p - 1) > nw) {
        at(p) = at(p - 1);
        --p;
      }
      at(p) = nw;
    }
  }
};

__global__ __launch_bounds__(RW_LANES) void rolling_kernel(const RollArgs A) {
  __shared__ double sw[RW_MAXW * RW_LANES];
  const int lane = threadIdx.x;
  const int64_t item = (int64_t)blockIdx.x * RW_LANES + lane;
  if (item >= A.S * A.nseg) return;   // whole lane idle; no barriers below
  const int64_t sym = item / A.nseg;
  const int seg = (int)(item % A.nseg);
  const int T = A.T, w = A.win, sh = A.shift;
  const double* __restrict__ x = A.x + sym * A.ld_in;
  double* __restrict__ out = A.out + sym * A.ld_out;
  const int t_begin = seg * RW_SEG;
  const int t_end = min(T, t_begin + RW_SEG);
  // value entering the window of output t: x[t - shift] (NaN outside [0, T))
  auto val = [&](int t) -> double {
    const int i = t - sh;
    return (i >= 0 && i < T) ? x[i] : qnan();
  };
  Win W{sw, lane, 0};
  // Moment modes follow pandas' window aggregations update for update
  // (pandas/_libs/window/aggregations.pyx, 2.3.3): add_sum/remove_sum and
  // add_mean/remove_mean keep a Kahan sum with SEPARATE add and remove
  // compensations; add_var/remove_var a compensated Welford mean + ssqdm.
  // Each step removes the leaving value, then adds the entering one.
  const bool welford = A.mode >= BQ_ROLL_VAR;
  double sum = 0.0, c_add = 0.0, c_rem = 0.0, last = qnan();
  double mean = 0.0, ssq = 0.0;
  int neg = 0, run = 0;   // signbit count (mean clamps); same-value run
  auto add = [&](double v) {
    ++W.n;
    if (welford) {
      const double prev_mean = mean - c_add;
      const double y = v - c_add;
      const double t = y - mean;
      c_add = (t + mean) - y;
      mean = mean + t / (double)W.n;
      ssq = ssq + (v - prev_mean) * (v - mean);
    } else {
      const double y = v - c_add;
      const double t = sum + y;
      c_add = (t - sum) - y;
      sum = t;
      neg += signbit(v) ? 1 : 0;
    }
    run = v == last ? run + 1 : 1;   // pandas counts equal values as they are added
    last = v;
  };
  auto remove = [&](double v) {
    --W.n;
    if (welford) {
      if (W.n) {
        const double prev_mean = mean - c_rem;
        const double y = v - c_rem;
        const double t = y - mean;
        c_rem = (t + mean) - y;
        mean = mean - t / (double)W.n;
        ssq = ssq - (v - prev_mean) * (v - mean);
      } else {
        mean = 0.0;
        ssq = 0.0;
      }
    } else {
      const double y = -v - c_rem;
      const double t = sum + y;
      c_rem = (t - sum) - y;
      sum = t;
      neg -= signbit(v) ? 1 : 0;
    }
  };
  // warm-up: window of output t_begin - 1, i.e. values of t in [t_begin - w, t_begin)
  for (int t = t_begin - w; t < t_begin; ++t) {
    const double v = val(t);
    if (v == v) {
      if (A.mode <= 1) {
        W.insert(v);
        run = v == last ? run + 1 : 1;
        last = v;
      } else {
        add(v);
      }
    }
  }
  for (int t = t_begin; t < t_end; ++t) {
    const double vn = val(t), vo = val(t - w);
    const bool in = vn == vn, outv = vo == vo;
    if (A.mode <= 1) {
      if (in && outv) W.replace(vo, vn);
      else if (in) W.insert(vn);
      else if (outv) W.erase(vo);
    } else {
      if (outv) remove(vo);
      if (in) add(vn);
    }
    const int n = W.n;
    double r;
    if (n == 0 && A.minp == 0 && A.mode == BQ_ROLL_SUM) r = 0.0;
    else if (n < A.minp || n == 0) r = qnan();
    else if (A.mode == BQ_ROLL_QUANTILE) {
      if (n == 1) r = W.at(0);
      else {
        const double idxf = A.q * (double)(n - 1);
        const int idx = (int)idxf;
        if ((double)idx == idxf) r = W.at(idx);
        else {
          const double lo = W.at(idx), hi = W.at(idx + 1);
          r = lo + (hi - lo) * (idxf - (double)idx);
        }
      }
    } else if (A.mode == BQ_ROLL_MEDIAN) {
      r = (n & 1) ? W.at(n >> 1) : (W.at((n >> 1) - 1) + W.at(n >> 1)) / 2.0;
    } else if (A.mode == BQ_ROLL_MEAN) {
      r = run >= n ? last : sum / (double)n;   // same-value rule
      if (neg == 0 && r < 0.0) r = 0.0;        // pandas calc_mean sign clamps
      else if (neg == n && r > 0.0) r = 0.0;
    } else if (A.mode == BQ_ROLL_SUM) {
      r = run >= n ? last * (double)n : sum;   // same-value rule
    } else {   // var / std (pandas calc_var), ddof 1 or 0
      const int ddof = (A.mode == BQ_ROLL_VAR || A.mode == BQ_ROLL_STD) ? 1 : 0;
      double var;
      if (n <= ddof) var = qnan();
      else if (n == 1 || run >= n) var = 0.0;
      else {
        var = ssq / (double)(n - ddof);
        var = var < 0.0 ? 0.0 : var;
      }
      r = (A.mode == BQ_ROLL_VAR || A.mode == BQ_ROLL_VAR0) ? var : sqrt(var);
    }
    out[t] = r;
  }
}

// ---- ewm(alpha, adjust=False, ignore_na=False, min_periods) ---------------------
__global__ __launch_bounds__(256) void ewm_kernel(const double* __restrict__ x, double* __restrict__ out, int64_t S,
                                                  int T, int64_t ld_in, int64_t ld_out, double alpha, int minp) {
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= S) return;
  const double* r = x + s * ld_in;
  double* o = out + s * ld_out;
  const double om = 1.0 - alpha;
  double weighted = r[0];
  int nobs = weighted == weighted;
  double old_wt = 1.0;
  o[0] = nobs >= minp ? weighted : qnan();
  for (int i = 1; i < T; ++i) {
    const double cur = r[i];
    const bool obs = cur == cur;
    nobs += obs;
    if (weighted == weighted) {
      old_wt *= om;
      if (obs) {
        if (weighted != cur) {
          weighted = old_wt * weighted + alpha * cur;
          weighted /= old_wt + alpha;
        }
        old_wt = 1.0;
      }
    } else if (obs) {
      weighted = cur;
    }
    o[i] = nobs >= minp ? weighted : qnan();
  }
}

}  // namespace bq

extern "C" {

int bq_rolling(const double* x, int64_t S, int64_t T, int64_t ld_in, int32_t window, int32_t min_periods,
               int32_t shift, int32_t mode, double q, double* out, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!x || !out || S < 0 || T < 0 || ld_in < T || ld_out < T || window < 1 || window > RW_MAXW ||
      min_periods < 0 || shift < 0 || mode < BQ_ROLL_QUANTILE || mode > BQ_ROLL_STD0 || !(q >= 0.0 && q <= 1.0) ||
      T > 0x7fffffff)
    return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  RollArgs A;
  A.x = x;
  A.out = out;
  A.S = S;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.win = window;
  A.minp = min_periods;
  A.shift = shift;
  A.mode = mode;
  A.q = q;
  A.nseg = (int)((T + RW_SEG - 1) / RW_SEG);
  const int64_t items = S * (int64_t)A.nseg;
  const unsigned blocks = (unsigned)((items + RW_LANES - 1) / RW_LANES);
  hipLaunchKernelGGL(rolling_kernel, dim3(blocks), dim3(RW_LANES), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_ewm(const double* x, int64_t S, int64_t T, int64_t ld_in, double alpha, int32_t min_periods, double* out,
           int64_t ld_out, void* stream) {
  using namespace bq;
  if (!x || !out || S < 0 || T < 0 || ld_in < T || ld_out < T || !(alpha > 0.0 && alpha <= 1.0) ||
      min_periods < 0 || T > 0x7fffffff)
    return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  const unsigned blocks = (unsigned)((S + 255) / 256);
  hipLaunchKernelGGL(ewm_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, out, S, (int)T, ld_in, ld_out,
                     alpha, (int)min_periods);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
