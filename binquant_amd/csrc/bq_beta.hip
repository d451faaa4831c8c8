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
// One 256-thread workgroup per symbol walks the row in tiles of 1024 candles
// (4 per lane). Per candle the five window sums come from tile-local prefix
// sums (wave DPP scans + LDS across waves) kept in an LDS ring with a
// 128-candle halo re-based to end at 0: a window sum is one difference, O(1)
// per candle whatever the window (the per-lane window walk this replaces cost
// w + K steps per K candles). The squares are summed about row-constant
// references (the row's first return) so the variances do not cancel; the
// means follow pandas' roll_mean including its same-value rule (runs of
// equal values, tracked with block max-scans), so constant-return windows
// (a halted symbol: returns exactly 0) give pandas' exact 0 covariance / NaN
// correlation. The benchmark's return at candle t is the same for every row
// (index-aligned mode): it is recomputed per block (one log per candle).
#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

constexpr int BC_NT = 256;
constexpr int BC_NW = BC_NT / WAVE;
constexpr int BC_K = 4;
constexpr int BC_TT = BC_NT * BC_K;
constexpr int BC_H = 128;
constexpr int BC_R = BC_H + BC_TT;
constexpr int BC_Q = BC_R / BC_K;
constexpr int BC_NS = 5;
static_assert(BC_R % BC_K == 0 && BC_H >= BQ_MAX_WINDOW + 2, "ring shape");   // prefix series: x, y, x*y, (x - rx)^2, (y - ry)^2
// ring position -> slot, lane-interleaved (in the natural layout the lanes'
// candles are K apart: multi-way bank conflicts on every access)
__device__ __forceinline__ int bslot(int p) { return (p % BC_K) * BC_Q + p / BC_K; }

struct BetaArgs {
  const double* close;   // PAIRS: symbol returns
  const double* btc;     // PAIRS: benchmark returns, same row stride
  double* beta;
  double* corr;
  const double* ystat;   // MODE 3: [2][T] benchmark window mean, variance (ddof 1)
  int64_t ld_in, ld_out;
  int T, win;
  double inv_w, inv_w1, bias;   // 1/w, 1/(w-1), w/(w-1)
};

__device__ __forceinline__ double log_return(double c, double p) { return log(c / p); }

// 1 / v with the hardware reciprocal and two Newton steps (v > 0)
__device__ __forceinline__ double rcp_nr(double v) {
  double r = __builtin_amdgcn_rcp(v);
  r = fma(r, fma(-v, r, 1.0), r);
  return fma(r, fma(-v, r, 1.0), r);
}

// 1 / sqrt(v) for v >= 0 (+inf at 0) with two Newton steps
__device__ __forceinline__ double rsq_nr(double v) {
  double r = __builtin_amdgcn_rsq(v);
  if (!(v > 0.0)) return r;
  const double h = 0.5 * v;
  r = r * fma(-h * r, r, 1.5);
  return r * fma(-h * r, r, 1.5);
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

// MODE 0: close / btc prices, returns formed here (first return NaN, first
// full window at t = w). MODE 2: close prices + the benchmark's returns as one
// row shared by every symbol (formed once per launch, not once per block).
// MODE 1: rows of dropna'd return pairs (bq_join_returns), first full window
// at t = w - 1.
// MODE 3: as MODE 2, and the benchmark's window mean / variance at every t
// are read from A.ystat (beta_btc_stats_kernel, once per launch): the block
// scans three series (x, x*y, (x - rx)^2) instead of five.
template <int MODE>
__global__ __launch_bounds__(BC_NT, MODE == 3 ? 3 : 2) void beta_corr_kernel(const BetaArgs A) {
  constexpr bool PAIRS = MODE == 1, BRET = MODE >= 2, YST = MODE == 3;
  __shared__ double sP[BC_NS][BC_R];
  __shared__ double sWt[BC_NS][BC_NW];
  __shared__ int sWl[3][BC_NW];
  __shared__ int sCar[3];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
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
  if (tid < BC_H) {
#pragma unroll
    for (int q = 0; q < BC_NS; ++q) sP[q][bslot(tid)] = 0.0;
  }
  if (tid < 3) sCar[tid] = -1;
  for (int t0 = 0; t0 < T; t0 += BC_TT) {
    const int tb = t0 + BC_K * tid, pb = BC_H + BC_K * tid;
    double x[BC_K], y[BC_K];
    {
      double pc = tb >= 1 && tb <= T ? rc[tb - 1] : qnan();
      double pbt = tb >= 1 && tb <= T ? rb[tb - 1] : qnan();
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        const bool ok = tb + k < T;
        const double c = ok ? rc[tb + k] : qnan(), b = ok ? rb[tb + k] : qnan();
        if (PAIRS) {
          x[k] = c;
          y[k] = b;
        } else {
          x[k] = log_return(c, pc);   // NaN at candle 0 (dropna)
          y[k] = BRET ? b : log_return(b, pbt);
        }
        pc = c;
        pbt = b;
      }
    }
    // per-candle terms (a candle without both returns adds nothing) and the
    // lane's inclusive prefix of each
    double q[BC_NS][BC_K];
    int lx = -1, ly = -1, lxy = -1;   // last index where x / y / x*y changed (lane)
    int lcx[BC_K], lcy[BC_K], lcxy[BC_K];
    {
      double acc[BC_NS] = {0, 0, 0, 0, 0};
      double px = qnan(), py = qnan(), pxy = qnan();
      if (tb >= 1 && tb <= T) {   // the previous candle's values for the run test
        // (a neighbour lane's last candle: recomputed, cheaper than a barrier)
        if (PAIRS) {
          px = rc[tb - 1];
          py = rb[tb - 1];
        } else if (tb >= 2) {
          px = log_return(rc[tb - 1], rc[tb - 2]);
          py = BRET ? rb[tb - 1] : log_return(rb[tb - 1], rb[tb - 2]);
        }
        pxy = px * py;
      }
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        const int t = tb + k;
        const bool ok = x[k] == x[k] && y[k] == y[k];
        const double xy = x[k] * y[k];
        if (ok) {
          const double u = x[k] - rx, v = y[k] - ry;
          acc[0] += x[k];
          acc[2] += xy;
          acc[3] = fma(u, u, acc[3]);
          if (!YST) {
            acc[1] += y[k];
            acc[4] = fma(v, v, acc[4]);
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < BC_NS; ++s2) q[s2][k] = acc[s2];
        if (t == 0 || !(x[k] == px)) lx = t;
        if (t == 0 || !(y[k] == py)) ly = t;
        if (t == 0 || !(xy == pxy)) lxy = t;
        lcx[k] = lx;
        lcy[k] = ly;
        lcxy[k] = lxy;
        px = x[k];
        py = y[k];
        pxy = xy;
      }
      // wave scan of the lane totals, wave totals to LDS
#pragma unroll
      for (int s2 = 0; s2 < BC_NS; ++s2) {
        if (YST && (s2 == 1 || s2 == 4)) continue;
        const double inc = wave_scan_f64(acc[s2], lane);
        if (lane == WAVE - 1) sWt[s2][w] = inc;
        const double ex = inc - acc[s2];
#pragma unroll
        for (int k = 0; k < BC_K; ++k) q[s2][k] += ex;
      }
      const int ix = wave_scan_max_dpp(lx + 1, lane) - 1, iy = wave_scan_max_dpp(ly + 1, lane) - 1,
                ixy = wave_scan_max_dpp(lxy + 1, lane) - 1;
      if (lane == WAVE - 1) {
        sWl[0][w] = ix;
        sWl[1][w] = iy;
        sWl[2][w] = ixy;
      }
      const int ex_x = dpp_i32<DPP_WAVE_SHR1>(ix + 1) - 1, ex_y = dpp_i32<DPP_WAVE_SHR1>(iy + 1) - 1,
                ex_xy = dpp_i32<DPP_WAVE_SHR1>(ixy + 1) - 1;
      __syncthreads();
      int cx = max(sCar[0], ex_x), cy = max(sCar[1], ex_y), cxy = max(sCar[2], ex_xy);
      double base[BC_NS] = {0, 0, 0, 0, 0};
      for (int u = 0; u < w; ++u) {
        cx = max(cx, sWl[0][u]);
        cy = max(cy, sWl[1][u]);
        cxy = max(cxy, sWl[2][u]);
#pragma unroll
        for (int s2 = 0; s2 < BC_NS; ++s2)
          if (!(YST && (s2 == 1 || s2 == 4))) base[s2] += sWt[s2][u];
      }
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        lcx[k] = max(lcx[k], cx);
        lcy[k] = max(lcy[k], cy);
        lcxy[k] = max(lcxy[k], cxy);
#pragma unroll
        for (int s2 = 0; s2 < BC_NS; ++s2) {
          if (YST && (s2 == 1 || s2 == 4)) continue;
          q[s2][k] += base[s2];
          sP[s2][bslot(pb + k)] = q[s2][k];
        }
      }
    }
    __syncthreads();
    double beta[BC_K], corr[BC_K];
    const double wd = (double)win;
#pragma unroll
    for (int k = 0; k < BC_K; ++k) {
      const int t = tb + k, o = bslot(pb + k - win);
      if (t < win - (PAIRS ? 1 : 0) || t >= T) {
        beta[k] = corr[k] = qnan();
        continue;
      }
      // the lane's own prefixes are re-read from the ring (not held across the
      // barrier: fewer live registers, more waves per SIMD)
      const int me = bslot(pb + k);
      const double Sx = sP[0][me] - sP[0][o], Sxy = sP[2][me] - sP[2][o];
      const double Suu = sP[3][me] - sP[3][o];
      // pandas: mean_xy, mean_x, mean_y = roll_mean (same-value rule)
      const bool cx = lcx[k] <= t - win + 1, cxy = lcxy[k] <= t - win + 1;
      const double mx = cx ? x[k] : div_exact(Sx, wd, A.inv_w);
      const double mxy = cxy ? x[k] * y[k] : div_exact(Sxy, wd, A.inv_w);
      // variances about the row references: sum (x - rx)^2 - (sum (x - rx))^2 / w
      const double Su = Sx - wd * rx;
      double vx = cx ? 0.0 : (Suu - Su * Su * A.inv_w) * A.inv_w1;
      double my, vy;
      if (YST) {
        my = A.ystat[t];
        vy = A.ystat[T + t];
      } else {
        const double Sy = sP[1][me] - sP[1][o], Svv = sP[4][me] - sP[4][o];
        const bool cy = lcy[k] <= t - win + 1;
        my = cy ? y[k] : div_exact(Sy, wd, A.inv_w);
        const double Sv = Sy - wd * ry;
        vy = cy ? 0.0 : (Svv - Sv * Sv * A.inv_w) * A.inv_w1;
      }
      const double cov = (mxy - mx * my) * A.bias;
      vx = vx < 0.0 ? 0.0 : vx;
      vy = vy < 0.0 ? 0.0 : vy;
      // reciprocal / reciprocal square root with Newton refinement (a few ulps,
      // well inside the 1e-9 bar) instead of IEEE divides: cov / vy, and
      // cov / sqrt(vx vy) (+-inf / NaN when vx vy == 0, as pandas' division)
      beta[k] = vy == 0.0 ? qnan() : cov * rcp_nr(vy);
      corr[k] = cov * rsq_nr(vx * vy);
    }
    const int64_t orow = sym * A.ld_out;
#pragma unroll
    for (int k = 0; k < BC_K; ++k) {
      if (tb + k < T) {
        if (A.beta) A.beta[orow + tb + k] = beta[k];
        if (A.corr) A.corr[orow + tb + k] = corr[k];
      }
    }
    if (t0 + BC_TT >= T) break;
    // halo for the next tile: the last 128 prefixes, re-based to end at 0
    double last[BC_NS];
#pragma unroll
    for (int s2 = 0; s2 < BC_NS; ++s2) last[s2] = sP[s2][bslot(BC_R - 1)];
    __syncthreads();   // every read of this tile's ring is done
    if (pb >= BC_TT) {
#pragma unroll
      for (int k = 0; k < BC_K; ++k)
#pragma unroll
        for (int s2 = 0; s2 < BC_NS; ++s2) sP[s2][bslot(pb + k - BC_TT)] = q[s2][k] - last[s2];
    }
    if (tid == BC_NT - 1) {
      sCar[0] = lcx[BC_K - 1];
      sCar[1] = lcy[BC_K - 1];
      sCar[2] = lcxy[BC_K - 1];
    }
  }
}

// The benchmark's rolling(w) mean and variance (ddof 1) of its log returns
// at every t (NaN while t < w; pandas' same-value rule: a constant window has
// the value itself as mean and 0 variance): ystat[0][t], ystat[1][t]. One
// 256-thread workgroup walks the row with the prefix scheme of the main
// kernel. y = returns row (y[0] NaN).
__global__ __launch_bounds__(BC_NT) void beta_btc_stats_kernel(const double* __restrict__ y, int T, int win,
                                                               double inv_w, double inv_w1, double* ystat) {
  __shared__ double sP[2][BC_R];
  __shared__ double sWt[2][BC_NW];
  __shared__ int sWl[BC_NW];
  __shared__ int sCar;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  double ry = T > 1 ? y[1] : 0.0;
  if (ry != ry) ry = 0.0;
  if (tid < BC_H) sP[0][bslot(tid)] = sP[1][bslot(tid)] = 0.0;
  if (tid == 0) sCar = -1;
  for (int t0 = 0; t0 < T; t0 += BC_TT) {
    const int tb = t0 + BC_K * tid, pb = BC_H + BC_K * tid;
    double v[BC_K], q[2][BC_K], acc[2] = {0.0, 0.0};
    int lc[BC_K], l = -1;
    double pv = tb >= 1 && tb <= T ? y[tb - 1] : qnan();
#pragma unroll
    for (int k = 0; k < BC_K; ++k) {
      const int t = tb + k;
      v[k] = t < T ? y[t] : qnan();
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
  if (mode == 3) {
    hipLaunchKernelGGL(beta_btc_stats_kernel, dim3(1), dim3(BC_NT), 0, (hipStream_t)stream, btc_close, A.T, window,
                       A.inv_w, A.inv_w1, ystat);
    hipLaunchKernelGGL(beta_corr_kernel<3>, dim3((unsigned)S), dim3(BC_NT), 0, (hipStream_t)stream, A);
  } else if (mode == 1) hipLaunchKernelGGL(beta_corr_kernel<1>, dim3((unsigned)S), dim3(BC_NT), 0, (hipStream_t)stream, A);
  else if (mode == 2) hipLaunchKernelGGL(beta_corr_kernel<2>, dim3((unsigned)S), dim3(BC_NT), 0, (hipStream_t)stream, A);
  else hipLaunchKernelGGL(beta_corr_kernel<0>, dim3((unsigned)S), dim3(BC_NT), 0, (hipStream_t)stream, A);
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

extern "C" int bq_beta_corr_pairs(const double* x, const double* y, int64_t S, int64_t T, int64_t ld_in,
                                  int32_t window, double* beta, double* corr, int64_t ld_out, void* stream) {
  return launch_beta(1, x, y, S, T, ld_in, window, beta, corr, ld_out, stream);
}
