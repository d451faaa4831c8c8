// Rolling beta / correlation of each symbol's log returns against the
// benchmark's (BTC), at every timestamp of an index-aligned [S][T] panel.
//
// Restates ContextEvaluator.dynamic_btc_beta_corr
// (producers/context_evaluator.py:154-194): returns = log(c / c.shift(1)) for
// the symbol and for BTC, inner-joined on the index and dropna'd (so the
// series start at candle 1), then with pandas' rolling(window) kernels
// (pandas/core/window/rolling.py cov/corr, pandas 2.3.3):
//   mean_xy, mean_x, mean_y = roll_mean(...)            (same-value rule)
//   cov  = (mean_xy - mean_x * mean_y) * (n / (n - 1))
//   beta = cov / var_y            (var_y == 0 -> NaN: var.replace(0, nan))
//   corr = cov / (var_x * var_y) ** 0.5                 (roll_var, ddof 1)
// NaN where the window is incomplete (t < window).
//
// One wave per symbol walks the row in tiles of 256 candles (4 per lane), with
// no cross-wave step: waves of different symbols never wait for each other,
// so one's latency hides behind another's arithmetic (the 256-thread block
// walker this replaces spent most of its time in barriers). Per candle the
// window sums come from tile-local prefix sums (wave DPP scans) in an LDS ring
// of 512 candles: a window sum is one difference, O(1) per candle whatever the
// window. At the end of a tile the lanes holding its last 128 prefixes write
// them back re-based to the next tile's frame (minus the tile total), so the
// prefixes never grow past one tile (no cancellation on long rows) and a read
// needs no frame test. The squares are summed about row-constant references
// (the row's first return) so the variances do not cancel; the means follow
// pandas' roll_mean including its same-value rule (runs of equal values,
// tracked with wave max-scans and a per-tile carry), so constant-return
// windows (a halted symbol: returns exactly 0) give pandas' exact 0
// covariance / NaN correlation. The previous candle of lane 0 and the run /
// total carries come from the previous tile through readlane; the next tile's
// prices are in flight while the current one computes.
#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

constexpr int BC_NT = 256;   // beta_btc_stats_kernel block
constexpr int BC_NW = BC_NT / WAVE;
constexpr int BC_K = 4;      // candles per lane
constexpr int BC_TT = BC_NT * BC_K;
constexpr int BC_H = 128;
constexpr int BC_R = BC_H + BC_TT;
constexpr int BC_Q = BC_R / BC_K;
static_assert(BC_R % BC_K == 0 && BC_H >= BQ_MAX_WINDOW + 2, "ring shape");
// ring position -> slot, lane-interleaved (in the natural layout the lanes'
// candles are K apart: multi-way bank conflicts on every access)
__device__ __forceinline__ int bslot(int p) { return (p % BC_K) * BC_Q + p / BC_K; }

struct BetaArgs {
  const double* close;   // PAIRS: symbol returns
  const double* btc;     // PAIRS: benchmark returns, same row stride
  double* beta;
  double* corr;
  const double* ystat;   // MODE 3: [3][T] benchmark window mean, variance (ddof 1), 1 / variance
  int64_t ld_in, ld_out;
  int T, win;
  double inv_w, inv_w1, bias;   // 1/w, 1/(w-1), w/(w-1)
  int vin, vbtc, vout;   // 16-byte aligned rows: close / btc loads, beta / corr stores
};

// 1 / sqrt(v) for v >= 0 (+inf at 0) with two Newton steps
__device__ __forceinline__ double rsq_nr(double v) {
  const double r0 = __builtin_amdgcn_rsq(v);
  const double h = 0.5 * v;
  double r = r0 * fma(-h * r0, r0, 1.5);
  r = r * fma(-h * r, r, 1.5);
  return v > 0.0 ? r : r0;   // select, not a branch
}

// inclusive wave prefix sum of a double (DPP row scans + readlane row carries)
__device__ __forceinline__ double wave_scan_f64(double x, int lane) {
  x += dpp_f64<DPP_ROW_SHR1>(x);
  x += dpp_f64<DPP_ROW_SHR2>(x);
  x += dpp_f64<DPP_ROW_SHR4>(x);
  x += dpp_f64<DPP_ROW_SHR8>(x);
  const double r0 = readlane_f64(x, 15), r1 = readlane_f64(x, 31), r2 = readlane_f64(x, 47);
  const int row = lane >> 4;
  const double c = row == 0 ? 0.0 : (row == 1 ? r0 : (row == 2 ? r0 + r1 : (r0 + r1) + r2));
  return x + c;
}

// A lane's 4 consecutive candles: two 16-byte accesses where the row allows
// (each instruction then fills half of every line it touches instead of a
// quarter; nontemporal loads measured slower here, nontemporal stores faster).
typedef double bq_v2d __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void ld4(const double* __restrict__ r, int t, int T, bool vec, double (&v)[4]) {
  if (vec && t + 4 <= T) {
    const bq_v2d* p = reinterpret_cast<const bq_v2d*>(r + t);
    const bq_v2d a = p[0], b = p[1];
    v[0] = a.x;
    v[1] = a.y;
    v[2] = b.x;
    v[3] = b.y;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = t + k < T ? r[t + k] : qnan();
  }
}

// write-once outputs: whole-line nontemporal stores (bq_device.h store_lines);
// the wave's lanes all call it (one wave per symbol)
__device__ __forceinline__ void st4(double* r, int t, int T, bool vec, const double (&v)[4]) {
  store_lines<4>(r, t, T, vec, v);
}

constexpr int BW_TT = WAVE * BC_K;   // candles per tile
constexpr int BW_R = 512;            // ring: a tile plus a halo of up to 256 candles
constexpr int BW_Q = BW_R / BC_K;
static_assert(BW_R >= BW_TT + BC_H && (BW_R & (BW_R - 1)) == 0 && BC_K == 4, "wave ring shape");
// candle index (negative: before the row) -> ring slot, lane-interleaved
__device__ __forceinline__ int wslot(int t) {
  const unsigned p = (unsigned)t & (BW_R - 1);
  return (int)((p & (BC_K - 1)) * BW_Q + (p >> 2));
}
#ifndef BQ_BW_WAVES
#define BQ_BW_WAVES 3   // waves per SIMD the MODE 3 register budget is cut for
#endif

// MODE 0: close / btc prices, returns formed here (first return NaN, first
// full window at t = w). MODE 2: close prices + the benchmark's returns as one
// row shared by every symbol (formed once per launch, not once per wave).
// MODE 1: rows of dropna'd return pairs (bq_join_returns), first full window
// at t = w - 1.
// MODE 3: as MODE 2, and the benchmark's window mean / variance / inverse
// variance at every t are read from A.ystat (beta_btc_stats_kernel, once per
// launch): the wave scans three series (x, x*y, (x - rx)^2) instead of five.
template <int MODE>
__global__ __launch_bounds__(WAVE, MODE == 3 ? BQ_BW_WAVES : 2) void beta_wave_kernel(const BetaArgs A) {
  constexpr bool PAIRS = MODE == 1, BRET = MODE >= 2, YST = MODE == 3;
  constexpr int NS = YST ? 3 : 5;   // x, x*y, (x - rx)^2 [, y, (y - ry)^2]
  __shared__ double sP[NS][BW_R];
  const int lane = threadIdx.x;
  const int64_t sym = blockIdx.x;
  const double* __restrict__ rc = A.close + sym * A.ld_in;
  const double* __restrict__ rb = PAIRS ? A.btc + sym * A.ld_in : A.btc;
  const int T = A.T;
  const int win = __builtin_amdgcn_readfirstlane(A.win);
  // row references of the squared deviations: the first return
  const int t_first = PAIRS ? 0 : 1;
  double rx = 0.0, ry = 0.0;
  if (T > t_first) {
    rx = PAIRS ? rc[0] : log_return(rc[1], rc[0]);
    ry = PAIRS ? rb[0] : (BRET ? rb[1] : log_return(rb[1], rb[0]));
    if (rx != rx) rx = 0.0;
    if (ry != ry) ry = 0.0;
  }
  // empty prefixes before the row (the halo of the first tile)
#pragma unroll
  for (int h = 0; h < BC_H; h += WAVE)
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) sP[s2][wslot(h + lane - BC_H)] = 0.0;
  // carries of the previous tile (wave-uniform)
  double cprev = qnan(), bprev = qnan(), xprev = qnan(), yprev = qnan(), xyprev = qnan();
  int carx = -1, cary = -1, carxy = -1;
  const bool vin = A.vin, vbtc = A.vbtc, vout = A.vout;
  double cn[BC_K], bn[BC_K];
  ld4(rc, BC_K * lane, T, vin, cn);
  ld4(rb, BC_K * lane, T, vbtc, bn);
  const double wd = (double)win;
  for (int t0 = 0; t0 < T; t0 += BW_TT) {
    const int tb = t0 + BC_K * lane;
    // MODE 3: the benchmark's window stats of this tile (L2 hits: every symbol
    // reads the same rows), issued before the next tile's prefetch so that
    // waiting for them does not wait for it (loads retire in order)
    double ym[BC_K], yv[BC_K], yi[BC_K];
    if (YST) {
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        const bool ok = tb + k < T;
        ym[k] = ok ? A.ystat[tb + k] : 0.0;
        yv[k] = ok ? A.ystat[T + tb + k] : 0.0;
        yi[k] = ok ? A.ystat[2 * T + tb + k] : 0.0;
      }
    }
    double x[BC_K], y[BC_K];
    {
      double c[BC_K], b[BC_K];
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        c[k] = cn[k];
        b[k] = bn[k];
      }
      if (t0 + BW_TT < T) {   // next tile's inputs in flight during this one
        ld4(rc, tb + BW_TT, T, vin, cn);
        ld4(rb, tb + BW_TT, T, vbtc, bn);
      }
      double pc = dpp_f64<DPP_WAVE_SHR1>(c[BC_K - 1]), pbt = dpp_f64<DPP_WAVE_SHR1>(b[BC_K - 1]);
      if (lane == 0) {
        pc = cprev;
        pbt = bprev;
      }
      cprev = readlane_f64(c[BC_K - 1], WAVE - 1);
      if (!BRET) bprev = readlane_f64(b[BC_K - 1], WAVE - 1);
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        if (PAIRS) {
          x[k] = c[k];
          y[k] = b[k];
        } else {
          x[k] = log_return(c[k], pc);   // NaN at candle 0 (dropna)
          y[k] = BRET ? b[k] : log_return(b[k], pbt);
        }
        pc = c[k];
        pbt = b[k];
      }
    }
    // per-candle terms (a candle without both returns adds nothing), their
    // tile-local inclusive prefixes, and the last index where x / y / x*y
    // changed (the same-value rule)
    double q[NS][BC_K];
    int lcx[BC_K], lcy[BC_K], lcxy[BC_K];
    {
      double acc[NS];
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) acc[s2] = 0.0;
      double px = dpp_f64<DPP_WAVE_SHR1>(x[BC_K - 1]), py = dpp_f64<DPP_WAVE_SHR1>(y[BC_K - 1]);
      double pxy = dpp_f64<DPP_WAVE_SHR1>(x[BC_K - 1] * y[BC_K - 1]);
      if (lane == 0) {
        px = xprev;
        py = yprev;
        pxy = xyprev;
      }
      int lx = -1, ly = -1, lxy = -1;
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        const int t = tb + k;
        const bool ok = x[k] == x[k] && y[k] == y[k];
        const double xy = x[k] * y[k];
        if (ok) {
          const double u = x[k] - rx;
          acc[0] += x[k];
          acc[1] += xy;
          acc[2] = fma(u, u, acc[2]);
          if (!YST) {
            const double v = y[k] - ry;
            acc[3] += y[k];
            acc[4] = fma(v, v, acc[4]);
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) q[s2][k] = acc[s2];
        if (t == 0 || !(x[k] == px)) lx = t;
        if (!YST && (t == 0 || !(y[k] == py))) ly = t;   // MODE 3: the benchmark's own runs are in ystat
        if (t == 0 || !(xy == pxy)) lxy = t;
        lcx[k] = lx;
        lcy[k] = ly;
        lcxy[k] = lxy;
        px = x[k];
        py = y[k];
        pxy = xy;
      }
      xprev = readlane_f64(x[BC_K - 1], WAVE - 1);
      if (!YST) yprev = readlane_f64(y[BC_K - 1], WAVE - 1);
      xyprev = readlane_f64(x[BC_K - 1] * y[BC_K - 1], WAVE - 1);
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) {
        const double ex = wave_scan_f64(acc[s2], lane) - acc[s2];
#pragma unroll
        for (int k = 0; k < BC_K; ++k) q[s2][k] += ex;
      }
      const int ix = wave_scan_max_dpp(lx + 1, lane) - 1, iy = YST ? -1 : wave_scan_max_dpp(ly + 1, lane) - 1,
                ixy = wave_scan_max_dpp(lxy + 1, lane) - 1;
      const int cx = max(carx, dpp_i32<DPP_WAVE_SHR1>(ix + 1) - 1),
                cy = YST ? -1 : max(cary, dpp_i32<DPP_WAVE_SHR1>(iy + 1) - 1),
                cxy = max(carxy, dpp_i32<DPP_WAVE_SHR1>(ixy + 1) - 1);
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        lcx[k] = max(lcx[k], cx);
        lcy[k] = max(lcy[k], cy);
        lcxy[k] = max(lcxy[k], cxy);
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) sP[s2][wslot(tb + k)] = q[s2][k];
      }
    }
    __syncthreads();   // one wave: orders the ring writes before the reads
    double beta[BC_K], corr[BC_K];
#pragma unroll
    for (int k = 0; k < BC_K; ++k) {
      const int t = tb + k;
      // (computed for every lane, the incomplete windows masked at the end:
      // a ring read before the row start is a zeroed slot)
      // window sums: own prefix minus the prefix at t - win (this tile's frame)
      const int o = wslot(t - win);
      double S[NS];
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) S[s2] = q[s2][k] - sP[s2][o];
      // pandas: mean_xy, mean_x, mean_y = roll_mean (same-value rule)
      const bool cx = lcx[k] <= t - win + 1, cxy = lcxy[k] <= t - win + 1;
      const double mx = cx ? x[k] : S[0] * A.inv_w;
      const double mxy = cxy ? x[k] * y[k] : S[1] * A.inv_w;
      // variances about the row references: sum (x - rx)^2 - (sum (x - rx))^2 / w
      const double Su = S[0] - wd * rx;
      double vx = cx ? 0.0 : (S[2] - Su * Su * A.inv_w) * A.inv_w1;
      double my, vy, ivy;
      if (YST) {
        my = ym[k];
        vy = yv[k];
        ivy = yi[k];
      } else {
        const bool cy = lcy[k] <= t - win + 1;
        my = cy ? y[k] : S[3] * A.inv_w;
        const double Sv = S[3] - wd * ry;
        vy = cy ? 0.0 : (S[4] - Sv * Sv * A.inv_w) * A.inv_w1;
        vy = vy < 0.0 ? 0.0 : vy;
        ivy = vy == 0.0 ? qnan() : rcp_nr(vy);
      }
      const double cov = (mxy - mx * my) * A.bias;
      vx = vx < 0.0 ? 0.0 : vx;
      // reciprocal / reciprocal square root with Newton refinement (a few ulps,
      // well inside the 1e-9 bar) instead of IEEE divides: cov / vy, and
      // cov / sqrt(vx vy) (+-inf / NaN when vx vy == 0, as pandas' division)
      const bool full = t >= win - (PAIRS ? 1 : 0);
      beta[k] = full ? cov * ivy : qnan();
      corr[k] = full ? cov * rsq_nr(vx * vy) : qnan();
    }
    const int64_t orow = sym * A.ld_out;
    if (A.beta) st4(A.beta + orow, tb, T, vout, beta);
    if (A.corr) st4(A.corr + orow, tb, T, vout, corr);
    carx = __builtin_amdgcn_readlane(lcx[BC_K - 1], WAVE - 1);
    cary = __builtin_amdgcn_readlane(lcy[BC_K - 1], WAVE - 1);
    carxy = __builtin_amdgcn_readlane(lcxy[BC_K - 1], WAVE - 1);
    if (t0 + BW_TT >= T) break;
    // the halo of the next tile: this tile's last 128 prefixes in the next
    // tile's frame (held in registers by lanes 32..63)
    double tot[NS];
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) tot[s2] = readlane_f64(q[s2][BC_K - 1], WAVE - 1);
    __syncthreads();   // this tile's ring reads are done
    if (BC_K * lane >= BW_TT - BC_H) {
#pragma unroll
      for (int k = 0; k < BC_K; ++k)
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) sP[s2][wslot(tb + k)] = q[s2][k] - tot[s2];
    }
  }
}

// The benchmark's rolling(w) mean and variance (ddof 1) of its log returns
// at every t (NaN while t < w; pandas' same-value rule: a constant window has
// the value itself as mean and 0 variance): ystat[0][t], ystat[1][t], and
// 1 / variance (NaN where the variance is 0: beta's var.replace(0, nan))
// in ystat[2][t]. One
// 256-thread workgroup walks the row with the prefix scheme of the main
// kernel. y = returns row (y[0] NaN).
// bp != NULL: y is formed here from the benchmark's prices
// (log_return(bp[t], bp[t-1]), NaN at t = 0) and written to ystat[3][t] for
// the symbol walk, so a call needs no separate returns pass.
__global__ __launch_bounds__(BC_NT) void beta_btc_stats_kernel(const double* __restrict__ y,
                                                               const double* __restrict__ bp, int T, int win,
                                                               double inv_w, double inv_w1, double* ystat) {
  __shared__ double sP[2][BC_R];
  __shared__ double sWt[2][BC_NW];
  __shared__ int sWl[BC_NW];
  __shared__ int sCar;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const auto yv = [&](int t) -> double {
    if (t < 0 || t >= T) return qnan();
    if (bp) return t == 0 ? qnan() : log_return(bp[t], bp[t - 1]);
    return y[t];
  };
  double ry = T > 1 ? yv(1) : 0.0;
  if (ry != ry) ry = 0.0;
  if (tid < BC_H) sP[0][bslot(tid)] = sP[1][bslot(tid)] = 0.0;
  if (tid == 0) sCar = -1;
  for (int t0 = 0; t0 < T; t0 += BC_TT) {
    const int tb = t0 + BC_K * tid, pb = BC_H + BC_K * tid;
    double v[BC_K], q[2][BC_K], acc[2] = {0.0, 0.0};
    int lc[BC_K], l = -1;
    double pv = tb >= 1 && tb <= T ? yv(tb - 1) : qnan();
#pragma unroll
    for (int k = 0; k < BC_K; ++k) {
      const int t = tb + k;
      v[k] = yv(t);
      if (bp && t < T) ystat[3 * T + t] = v[k];
      if (v[k] == v[k]) {
        const double d = v[k] - ry;
        acc[0] += v[k];
        acc[1] = fma(d, d, acc[1]);
      }
      q[0][k] = acc[0];
      q[1][k] = acc[1];
      if (t == 0 || !(v[k] == pv)) l = t;
      lc[k] = l;
      pv = v[k];
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const double inc = wave_scan_f64(acc[s2], lane);
      if (lane == WAVE - 1) sWt[s2][w] = inc;
#pragma unroll
      for (int k = 0; k < BC_K; ++k) q[s2][k] += inc - acc[s2];
    }
    const int il = wave_scan_max_dpp(l + 1, lane) - 1;
    if (lane == WAVE - 1) sWl[w] = il;
    const int exl = dpp_i32<DPP_WAVE_SHR1>(il + 1) - 1;
    __syncthreads();
    int c = max(sCar, exl);
    double base[2] = {0.0, 0.0};
    for (int u = 0; u < w; ++u) {
      c = max(c, sWl[u]);
      base[0] += sWt[0][u];
      base[1] += sWt[1][u];
    }
#pragma unroll
    for (int k = 0; k < BC_K; ++k) {
      lc[k] = max(lc[k], c);
      q[0][k] += base[0];
      q[1][k] += base[1];
      sP[0][bslot(pb + k)] = q[0][k];
      sP[1][bslot(pb + k)] = q[1][k];
    }
    __syncthreads();
    const double wd = (double)win;
#pragma unroll
    for (int k = 0; k < BC_K; ++k) {
      const int t = tb + k, o = bslot(pb + k - win);
      if (t >= T) continue;
      double m = qnan(), var = qnan();
      if (t >= win) {
        const double Sy = q[0][k] - sP[0][o], Svv = q[1][k] - sP[1][o];
        if (lc[k] <= t - win + 1) {
          m = v[k];
          var = 0.0;
        } else {
          m = div_exact(Sy, wd, inv_w);
          const double Sv = Sy - wd * ry;
          var = (Svv - Sv * Sv * inv_w) * inv_w1;
          var = var < 0.0 ? 0.0 : var;
        }
      }
      ystat[t] = m;
      ystat[T + t] = var;
      ystat[2 * T + t] = var == 0.0 ? qnan() : 1.0 / var;
    }
    if (t0 + BC_TT >= T) break;
    double last[2] = {sP[0][bslot(BC_R - 1)], sP[1][bslot(BC_R - 1)]};
    __syncthreads();
    if (pb >= BC_TT) {
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        sP[0][bslot(pb + k - BC_TT)] = q[0][k] - last[0];
        sP[1][bslot(pb + k - BC_TT)] = q[1][k] - last[1];
      }
    }
    if (tid == BC_NT - 1) sCar = lc[BC_K - 1];
  }
}

}  // namespace bq

namespace {
int launch_beta(int mode, const double* close, const double* btc_close, int64_t S, int64_t T, int64_t ld_in,
                int32_t window, double* beta, double* corr, int64_t ld_out, void* stream,
                double* ystat = nullptr) {
  using namespace bq;
  if (!close || !btc_close || S < 0 || T < 0 || ld_in < T || ld_out < T || window < 2 ||
      window > BQ_MAX_WINDOW || T > 0x7fffffff || S > 0x7fffffff)
    return BQ_EINVAL;
  if (S == 0 || T == 0 || (!beta && !corr)) return BQ_OK;
  BetaArgs A;
  A.close = close;
  A.btc = btc_close;
  A.beta = beta;
  A.corr = corr;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.win = window;
  A.inv_w = 1.0 / (double)window;
  A.inv_w1 = 1.0 / (double)(window - 1);
  A.bias = (double)window / (double)(window - 1);
  A.ystat = ystat;
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  A.vin = a16(close) && (ld_in & 1) == 0;
  A.vbtc = (mode == 4 ? a16(ystat + 3 * T) : a16(btc_close)) && (mode != 1 || (ld_in & 1) == 0);
  A.vout = (!beta || a16(beta)) && (!corr || a16(corr)) && (ld_out & 1) == 0;
  if (mode == 3 || mode == 4) {   // 4: benchmark prices, its returns formed by the pre-pass into ystat[3]
    hipLaunchKernelGGL(beta_btc_stats_kernel, dim3(1), dim3(BC_NT), 0, (hipStream_t)stream,
                       mode == 3 ? btc_close : nullptr, mode == 4 ? btc_close : nullptr, A.T, window, A.inv_w,
                       A.inv_w1, ystat);
    if (mode == 4) A.btc = ystat + 3 * T;
    hipLaunchKernelGGL(beta_wave_kernel<3>, dim3((unsigned)S), dim3(WAVE), 0, (hipStream_t)stream, A);
  } else if (mode == 1) hipLaunchKernelGGL(beta_wave_kernel<1>, dim3((unsigned)S), dim3(WAVE), 0, (hipStream_t)stream, A);
  else if (mode == 2) hipLaunchKernelGGL(beta_wave_kernel<2>, dim3((unsigned)S), dim3(WAVE), 0, (hipStream_t)stream, A);
  else hipLaunchKernelGGL(beta_wave_kernel<0>, dim3((unsigned)S), dim3(WAVE), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
}  // namespace

extern "C" int bq_beta_corr(const double* close, const double* btc_close, int64_t S, int64_t T, int64_t ld_in,
                            int32_t window, double* beta, double* corr, int64_t ld_out, void* stream) {
  return launch_beta(0, close, btc_close, S, T, ld_in, window, beta, corr, ld_out, stream);
}

extern "C" int bq_beta_corr_bret(const double* close, const double* btc_returns, double* scratch, int64_t S,
                                 int64_t T, int64_t ld_in, int32_t window, double* beta, double* corr, int64_t ld_out,
                                 void* stream) {
  return launch_beta(scratch ? 3 : 2, close, btc_returns, S, T, ld_in, window, beta, corr, ld_out, stream, scratch);
}

extern "C" int bq_beta_corr_ws(const double* close, const double* btc_close, double* scratch, int64_t S, int64_t T,
                               int64_t ld_in, int32_t window, double* beta, double* corr, int64_t ld_out,
                               void* stream) {
  if (!scratch) return BQ_EINVAL;
  return launch_beta(4, close, btc_close, S, T, ld_in, window, beta, corr, ld_out, stream, scratch);
}

extern "C" int bq_beta_corr_pairs(const double* x, const double* y, int64_t S, int64_t T, int64_t ld_in,
                                  int32_t window, double* beta, double* corr, int64_t ld_out, void* stream) {
  return launch_beta(1, x, y, S, T, ld_in, window, beta, corr, ld_out, stream);
}
