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
// One 256-thread workgroup per symbol, tiles of 2048 candles (8 per lane),
// returns staged in an LDS ring with a 128-candle halo; each lane walks its
// window once and slides it over its 8 candles.
#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

constexpr int BC_NT = 256;
constexpr int BC_K = 8;
constexpr int BC_TT = BC_NT * BC_K;
constexpr int BC_H = 128;
constexpr int BC_R = BC_H + BC_TT;
// LDS index skew: one pad double every 32, so the lanes' stride-4 window
// walks (lane i at 4i + j) spread over all bank pairs instead of 8
__device__ __forceinline__ int bsk(int p) { return p + (p >> 5); }
constexpr int BC_RS = BC_R + (BC_R >> 5) + 1;

struct BetaArgs {
  const double* close;   // PAIRS: symbol returns
  const double* btc;     // PAIRS: benchmark returns, same row stride
  double* beta;
  double* corr;
  int64_t ld_in, ld_out;
  int T, win;
  double inv_w, inv_w1, bias;   // 1/w, 1/(w-1), w/(w-1)
};

__device__ __forceinline__ double log_return(double c, double p) { return log(c / p); }


// PAIRS = false: close / btc prices, returns formed here (first return NaN,
// first full window at t = w). PAIRS = true: rows of dropna'd return pairs
// (bq_join_returns), first full window at t = w - 1.
template <bool PAIRS>
__global__ __launch_bounds__(BC_NT) void beta_corr_kernel(const BetaArgs A) {
  __shared__ double sX[BC_RS], sY[BC_RS];
  const int tid = threadIdx.x;
  const int64_t sym = blockIdx.x;
  const double* __restrict__ rc = A.close + sym * A.ld_in;
  const double* __restrict__ rb = PAIRS ? A.btc + sym * A.ld_in : A.btc;
  const int T = A.T, w = A.win;
  if (tid < BC_H) {
    sX[bsk(tid)] = qnan();
    sY[bsk(tid)] = qnan();
  }
  __syncthreads();
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
          y[k] = log_return(b, pbt);
        }
        sX[bsk(pb + k)] = x[k];
        sY[bsk(pb + k)] = y[k];
        pc = c;
        pbt = b;
      }
    }
    __syncthreads();
    double beta[BC_K], corr[BC_K];
    {
      // window sums over (t - w, t]: x, y, x*y, and squares about lane refs
      const double rx = x[0] == x[0] ? x[0] : 0.0, ry = y[0] == y[0] ? y[0] : 0.0;
      double sx = 0, sy = 0, sxy = 0, dx2 = 0, dy2 = 0, dx1 = 0, dy1 = 0;
      double px = qnan(), py = qnan(), pxy = qnan();
      int runx = 0, runy = 0, runxy = 0;
      auto add = [&](double xi, double yi, double sign) {
        const double xy = xi * yi;
        sx += sign * xi;
        sy += sign * yi;
        sxy += sign * xy;
        const double ex = xi - rx, ey = yi - ry;
        dx1 += sign * ex;
        dy1 += sign * ey;
        dx2 = fma(sign * ex, ex, dx2);
        dy2 = fma(sign * ey, ey, dy2);
      };
      auto track = [&](double xi, double yi) {
        const double xy = xi * yi;
        runx = xi == px ? runx + 1 : 1;
        runy = yi == py ? runy + 1 : 1;
        runxy = xy == pxy ? runxy + 1 : 1;
        px = xi;
        py = yi;
        pxy = xy;
      };
      for (int i = pb - w + 1; i <= pb; ++i) {
        const double xi = sX[bsk(i)], yi = sY[bsk(i)];
        if (xi == xi && yi == yi) add(xi, yi, 1.0);
        track(xi, yi);
      }
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        const int t = tb + k, p = pb + k;
        if (k > 0) {
          const double xo = sX[bsk(p - w)], yo = sY[bsk(p - w)];
          if (xo == xo && yo == yo) add(xo, yo, -1.0);
          add(x[k], y[k], 1.0);
          track(x[k], y[k]);
        }
        if (t < w - (PAIRS ? 1 : 0) || t >= T) {
          beta[k] = corr[k] = qnan();
          continue;
        }
        const double wd = (double)w;
        const double mx = runx >= w ? px : div_exact(sx, wd, A.inv_w);
        const double my = runy >= w ? py : div_exact(sy, wd, A.inv_w);
        const double mxy = runxy >= w ? pxy : div_exact(sxy, wd, A.inv_w);
        const double cov = (mxy - mx * my) * A.bias;
        double vx = runx >= w ? 0.0 : (dx2 - dx1 * dx1 * A.inv_w) * A.inv_w1;
        double vy = runy >= w ? 0.0 : (dy2 - dy1 * dy1 * A.inv_w) * A.inv_w1;
        vx = vx < 0.0 ? 0.0 : vx;
        vy = vy < 0.0 ? 0.0 : vy;
        beta[k] = vy == 0.0 ? qnan() : cov / vy;
        corr[k] = cov / sqrt(vx * vy);
      }
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
    __syncthreads();   // every read of this tile's ring is done
    if (pb >= BC_TT) {   // owners of [TT, R) become the next tile's halo
#pragma unroll
      for (int k = 0; k < BC_K; ++k) {
        sX[bsk(pb + k - BC_TT)] = x[k];
        sY[bsk(pb + k - BC_TT)] = y[k];
      }
    }
  }
}

}  // namespace bq

namespace {
int launch_beta(bool pairs, const double* close, const double* btc_close, int64_t S, int64_t T, int64_t ld_in,
                int32_t window, double* beta, double* corr, int64_t ld_out, void* stream) {
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
  if (pairs) hipLaunchKernelGGL(beta_corr_kernel<true>, dim3((unsigned)S), dim3(BC_NT), 0, (hipStream_t)stream, A);
  else hipLaunchKernelGGL(beta_corr_kernel<false>, dim3((unsigned)S), dim3(BC_NT), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
}  // namespace

extern "C" int bq_beta_corr(const double* close, const double* btc_close, int64_t S, int64_t T, int64_t ld_in,
                            int32_t window, double* beta, double* corr, int64_t ld_out, void* stream) {
  return launch_beta(false, close, btc_close, S, T, ld_in, window, beta, corr, ld_out, stream);
}

extern "C" int bq_beta_corr_pairs(const double* x, const double* y, int64_t S, int64_t T, int64_t ld_in,
                                  int32_t window, double* beta, double* corr, int64_t ld_out, void* stream) {
  return launch_beta(true, x, y, S, T, ld_in, window, beta, corr, ld_out, stream);
}
