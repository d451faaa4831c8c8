// Time-parallel ("panel mode") rolling sums / means and ewm (gfx950) for the
// strategy pipelines of SURVEY §8a a17-a19 on a [S][T] panel, at the
// north_star tolerance (1e-9 of pandas) instead of the bit-exact replay:
//
//   x.shift(shift).rolling(window, min_periods).sum() / .mean()
//       strategies/failed_spike_fade.py:260-318, liquidation_sweep_pump.py:220
//   x.ewm(alpha, adjust=False, min_periods).mean()
//       strategies/liquidation_sweep_pump.py:215-217, 252-253, 265-266
//
// The exact replays of bq_rolling.hip are lane = symbol, sequential along T:
// 12.5k symbols are 196 waves per series for 1 024 SIMDs, each a 2 000-step
// dependent chain. Here one 256-thread workgroup per (row, series) walks the
// row in tiles of 2 048 candles (8 per lane, 64-byte loads, the next tile in
// flight), the values in an LDS ring with a 128-candle halo (window + shift
// <= 128), lane-interleaved (conflict-free):
//
// * sum / mean: one sliding walk per lane (window + 8 ring reads per 8
//   outputs), NaN skipped with pandas' observation count and min_periods, the
//   same-value rule (the window's values all equal -> the value itself, x
//   nobs for sums) from the run starts of the row (a block max-scan of the
//   last index where the value changed) — a window holding a NaN compares its
//   values directly — and calc_mean's sign rule from sliding negative counts;
// * ewm: an associative scan of the affine maps y -> la y + lb x (wave
//   shuffles, LDS across waves, a tile carry), then each lane replays its 8
//   steps with pandas' update (weighted = old_wt w + alpha x, / (old_wt +
//   alpha), skipped when w == x). A row with a missing or infinite value
//   continues serially from the first tile that holds one with pandas' own
//   recursion (gap decay of the old weight, the observation count, a late
//   first observation): exact, and only such rows pay for it.
//
// Values agree with pandas to rounding (the replay's Kahan / online sums are
// not reproduced bit for bit); bq_rolling_batch keeps the replays for
// bq_roll_job.panel == 0 (the live path and every bit-exact test).
#include "bq_panel.h"

#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

constexpr int PN_NT = 256;
constexpr int PN_NW = PN_NT / WAVE;
constexpr int PN_K = 8;
constexpr int PN_TT = PN_NT * PN_K;   // 2048
constexpr int PN_H = 128;             // >= window + shift
constexpr int PN_R = PN_H + PN_TT;    // 2176
constexpr int PN_Q = PN_R / PN_K;     // 272

__device__ __forceinline__ int pn_slot(int p) { return (p & (PN_K - 1)) * PN_Q + (p >> 3); }

typedef double pn_dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void pn_load(const double* __restrict__ row, int tb, int T, bool vec, double (&x)[PN_K]) {
  if (vec && tb + PN_K <= T) {
    const pn_dbl2* p = reinterpret_cast<const pn_dbl2*>(row + tb);
#pragma unroll
    for (int j = 0; j < PN_K / 2; ++j) {
      const pn_dbl2 a = p[j];
      x[2 * j] = a.x;
      x[2 * j + 1] = a.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < PN_K; ++k) x[k] = tb + k < T ? row[tb + k] : qnan();
  }
}

__device__ __forceinline__ bool pn_aligned(const void* p, int64_t ld) { return (((uintptr_t)p) & 15u) == 0 && (ld % 2) == 0; }

// exclusive block max of a per-lane int >= -1 combined with the tile carry
// `*carry` — read after the barrier: the previous tile's last thread writes it
// after that tile's final barrier, so a read before this one would race
__device__ __forceinline__ int pn_block_excl_max(int v, const int* carry, int* sW, int lane, int w) {
  const int inc = wave_scan_max_dpp(v + 1, lane) - 1;
  if (lane == WAVE - 1) sW[w] = inc;
  const int lpre = dpp_i32<DPP_WAVE_SHR1>(inc + 1) - 1;
  __syncthreads();
  int c = max(*carry, lpre);
  for (int u = 0; u < w; ++u) c = max(c, sW[u]);
  return c;
}

// ---- sum / mean -----------------------------------------------------------------------
__global__ __launch_bounds__(PN_NT) void panel_window_kernel(const PanelBatch B) {
  __shared__ double sX[PN_R];
  __shared__ int sL[PN_R];   // run start (last index where the value changed) per ring position
  __shared__ int sW[PN_NW];
  __shared__ int sCar;
  const PanelJob& A = B.j[blockIdx.y];
  const int64_t row = blockIdx.x;
  if (row >= A.rows) return;   // the job's own row count (a benchmark row): uniform per block
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const double* __restrict__ x = A.x + row * A.ld_in;
  double* __restrict__ out = A.out + row * A.ld_out;
  const int T = B.T, win = A.win, sh = A.shift, minp = A.minp;
  const bool mean = A.mode == BQ_ROLL_MEAN;
  const bool vin = pn_aligned(A.x, A.ld_in), vout = pn_aligned(A.out, A.ld_out);
  if (tid < PN_H) {   // before the row: missing values
    sX[pn_slot(tid)] = qnan();
    sL[pn_slot(tid)] = -1;
  }
  if (tid == 0) sCar = -1;
  double nx[PN_K];
  pn_load(x, PN_K * tid, T, vin, nx);
  for (int t0 = 0; t0 < T; t0 += PN_TT) {
    const int tb = t0 + PN_K * tid, pb = PN_H + PN_K * tid;
    double c[PN_K];
#pragma unroll
    for (int k = 0; k < PN_K; ++k) c[k] = win_val(nx[k]);   // +-inf is missing (pandas' window ops)
    const double pc0 = tb >= 1 && tb <= T ? win_val(x[tb - 1]) : qnan();
    if (t0 + PN_TT < T) pn_load(x, tb + PN_TT, T, vin, nx);
    // run starts of the values (NaN counts as a change)
    int lcl[PN_K];
    {
      double pv = pc0;
      int run = -1;
#pragma unroll
      for (int k = 0; k < PN_K; ++k) {
        if (tb + k == 0 || !(c[k] == pv)) run = tb + k;
        lcl[k] = run;
        pv = c[k];
      }
      const int carry = pn_block_excl_max(lcl[PN_K - 1], &sCar, sW, lane, w);
#pragma unroll
      for (int k = 0; k < PN_K; ++k) lcl[k] = max(lcl[k], carry);
    }
#pragma unroll
    for (int k = 0; k < PN_K; ++k) {
      sX[pn_slot(pb + k)] = c[k];
      sL[pn_slot(pb + k)] = lcl[k];
    }
    __syncthreads();
    // window of output t = tb + k: ring positions [pb + k - sh - win + 1, pb + k - sh]
    double s = 0.0;
    int nobs = 0, neg = 0;
    const int e0 = pb - sh;   // position of the entering value of output k = 0
    for (int j = 1 - win; j <= 0; ++j) {
      const double v = sX[pn_slot(e0 + j)];
      const bool ok = v == v;
      s += ok ? v : 0.0;
      nobs += ok;
      neg += ok && signbit(v);
    }
    double res[PN_K];
#pragma unroll
    for (int k = 0; k < PN_K; ++k) {
      const int e = e0 + k;   // entering position
      if (k > 0) {
        const double vi = sX[pn_slot(e)], vo = sX[pn_slot(e - win)];
        const bool oi = vi == vi, oo = vo == vo;
        s = (s + (oi ? vi : 0.0)) - (oo ? vo : 0.0);
        nobs += (int)oi - (int)oo;
        neg += (int)(oi && signbit(vi)) - (int)(oo && signbit(vo));
      }
      double r;
      if (!mean && nobs == 0 && minp == 0) r = 0.0;
      else if (nobs < minp || nobs <= 0) r = qnan();
      else {
        // pandas' same-value rule: every value of the window equal to the last one
        bool same;
        double last;
        if (nobs == win) {   // no missing value: the run start decides
          last = sX[pn_slot(e)];
          same = sL[pn_slot(e)] <= tb + k - sh - win + 1;
        } else {             // missing values: compare the observed ones directly
          last = qnan();
          same = true;
          for (int j = 0; j > -win; --j) {
            const double v = sX[pn_slot(e + j)];
            if (v != v) continue;
            if (last != last) last = v;
            else same = same && v == last;
          }
        }
        if (mean) {
          r = s / (double)nobs;
          if (same) r = last;
          else if (neg == 0 && r < 0.0) r = 0.0;
          else if (neg == nobs && r > 0.0) r = 0.0;
        } else {
          r = same ? last * (double)nobs : s;
        }
      }
      res[k] = r;
    }
    store_lines<PN_K>(out, tb, T, vout, res);
    if (t0 + PN_TT >= T) break;
    __syncthreads();   // every read of this tile's ring is done
    if (pb >= PN_TT) {
#pragma unroll
      for (int k = 0; k < PN_K; ++k) {
        sX[pn_slot(pb + k - PN_TT)] = c[k];
        sL[pn_slot(pb + k - PN_TT)] = lcl[k];
      }
    }
    if (tid == PN_NT - 1) sCar = lcl[PN_K - 1];
  }
}

// ---- ewm ------------------------------------------------------------------------------
// TR: the series is the true range max(h - l, |h - c[t-1]|, |l - c[t-1]|) of
// the job's (hi, lo, x = close), formed from the loads (NaN operands skipped,
// as DataFrame.max(axis=1): the first candle's is h - l) — the ATR of
// liquidation_sweep_pump.py:206-217 without a true-range column in HBM
template <bool TR>
__global__ __launch_bounds__(PN_NT) void panel_ewm_kernel(const PanelBatch B) {
  __shared__ double sA[PN_NW], sB[PN_NW];
  __shared__ double sCarry;
  __shared__ double sX[PN_TT];   // the serial replay's tile
  const PanelJob& A = B.j[blockIdx.y];
  const int64_t row = blockIdx.x;
  if (row >= A.rows) return;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const double* __restrict__ x = A.x + row * A.ld_in;
  double* __restrict__ out = A.out + row * A.ld_out;
  const int T = B.T, minp = A.minp;
  const bool vin = pn_aligned(A.x, A.ld_in), vout = pn_aligned(A.out, A.ld_out);
  const double alpha = A.alpha, om = 1.0 - alpha, den = om + alpha;
  const bool div = den != 1.0;
  const double la = om / den, lb = alpha / den;
  if (tid == 0) sCarry = 0.0;
  bool serial = false;
  double wv = qnan(), owt = 1.0;   // pandas' state (thread 0) once the row turns serial
  int nobs = 0;
  double nx[PN_K], nh[TR ? PN_K : 1], nl[TR ? PN_K : 1];
  const double* __restrict__ xh = TR ? A.hi + row * A.ld_in : nullptr;
  const double* __restrict__ xl = TR ? A.lo + row * A.ld_in : nullptr;
  const bool vhl = TR && pn_aligned(A.hi, A.ld_in) && pn_aligned(A.lo, A.ld_in);
  auto load_tile = [&](int tb) {
    pn_load(x, tb, T, vin, nx);
    if constexpr (TR) {
      pn_load(xh, tb, T, vhl, nh);
      pn_load(xl, tb, T, vhl, nl);
    }
  };
  load_tile(PN_K * tid);
  for (int t0 = 0; t0 < T; t0 += PN_TT) {
    const int tb = t0 + PN_K * tid;
    double c[PN_K];
    if constexpr (TR) {
      double pc = tb >= 1 && tb <= T ? x[tb - 1] : qnan();
#pragma unroll
      for (int k = 0; k < PN_K; ++k) {
        c[k] = tb + k < T ? win_val(true_range(nh[k], nl[k], pc)) : qnan();
        pc = nx[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < PN_K; ++k) c[k] = win_val(nx[k]);   // +-inf is missing (pandas' window ops)
    }
    if (t0 + PN_TT < T) load_tile(tb + PN_TT);
    {
      int bad = 0;
#pragma unroll
      for (int k = 0; k < PN_K; ++k) bad |= (tb + k < T) && !(c[k] - c[k] == 0.0);
      if (__syncthreads_or(bad) && !serial) {
        serial = true;
        if (t0 > 0) {   // candles 0 .. t0 - 1 were all observations
          wv = sCarry;
          nobs = t0;
        }
      }
    }
    double res[PN_K];
    if (serial) {
#pragma unroll
      for (int k = 0; k < PN_K; ++k) sX[PN_K * tid + k] = c[k];
      __syncthreads();
      if (tid == 0) {
        const int n = min(PN_TT, T - t0);
        for (int i = 0; i < n; ++i) {
          const double cur = sX[i];
          const bool obs = cur == cur;
          if (t0 + i == 0) {   // pandas: weighted = vals[0], nobs = its observation
            wv = cur;
            nobs = obs ? 1 : 0;
          } else {
            nobs += obs ? 1 : 0;
            if (wv == wv) {
              owt *= om;
              if (obs) {
                if (wv != cur) {
                  wv = owt * wv + alpha * cur;
                  wv /= owt + alpha;
                }
                owt = 1.0;
              }
            } else if (obs) {
              wv = cur;
            }
          }
          sX[i] = nobs >= minp ? wv : qnan();
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < PN_K; ++k) res[k] = sX[PN_K * tid + k];
      store_lines<PN_K>(out, tb, T, vout, res);
      if (t0 + PN_TT >= T) break;
      __syncthreads();
      continue;
    }
    // lane map over its candles from the zero state (candle 0 resets: a = 0, b = x)
    double a_ = 1.0, b_ = 0.0;
#pragma unroll
    for (int k = 0; k < PN_K; ++k) {
      if (tb + k == 0) {
        a_ = 0.0;
        b_ = c[k];
      } else {
        a_ *= la;
        b_ = fma(la, b_, lb * c[k]);
      }
    }
    double sa = a_, sb = b_;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const double pa = __shfl_up(sa, d, WAVE), pbv = __shfl_up(sb, d, WAVE);
      if (lane >= d) {
        sb = fma(sa, pbv, sb);
        sa *= pa;
      }
    }
    if (lane == WAVE - 1) {
      sA[w] = sa;
      sB[w] = sb;
    }
    double ea = __shfl_up(sa, 1, WAVE), eb = __shfl_up(sb, 1, WAVE);
    if (lane == 0) {
      ea = 1.0;
      eb = 0.0;
    }
    __syncthreads();
    double y = sCarry;
    for (int u = 0; u < w; ++u) y = fma(sA[u], y, sB[u]);
    y = fma(ea, y, eb);
    // exact replay of the lane's steps
#pragma unroll
    for (int k = 0; k < PN_K; ++k) {
      const int t = tb + k;
      const double v = c[k];
      if (t == 0) y = v;
      else if (y != v) {
        y = om * y + alpha * v;
        if (div) y = y / den;
      }
      res[k] = t + 1 >= minp ? y : qnan();
    }
    store_lines<PN_K>(out, tb, T, vout, res);
    if (t0 + PN_TT >= T) break;
    __syncthreads();
    if (tid == PN_NT - 1) sCarry = y;
    __syncthreads();
  }
}

bool panel_supported(int mode, int window, int shift) {
  if (mode == BQ_ROLL_EWM) return true;
  return (mode == BQ_ROLL_SUM || mode == BQ_ROLL_MEAN) && window >= 1 && shift >= 0 && window + shift <= PN_H;
}

void launch_panel(const PanelBatch& B, int n, hipStream_t st) {
  PanelBatch win, ewm;
  win.S = ewm.S = B.S;
  win.T = ewm.T = B.T;
  PanelBatch etr;
  etr.S = B.S;
  etr.T = B.T;
  int nw = 0, ne = 0, nt = 0;
  for (int i = 0; i < n; ++i) {
    if (B.j[i].mode == BQ_ROLL_EWM && B.j[i].hi) etr.j[nt++] = B.j[i];
    else if (B.j[i].mode == BQ_ROLL_EWM) ewm.j[ne++] = B.j[i];
    else win.j[nw++] = B.j[i];
  }
  if (nw) hipLaunchKernelGGL(panel_window_kernel, dim3((unsigned)B.S, (unsigned)nw), dim3(PN_NT), 0, st, win);
  if (ne) hipLaunchKernelGGL(panel_ewm_kernel<false>, dim3((unsigned)B.S, (unsigned)ne), dim3(PN_NT), 0, st, ewm);
  if (nt) hipLaunchKernelGGL(panel_ewm_kernel<true>, dim3((unsigned)B.S, (unsigned)nt), dim3(PN_NT), 0, st, etr);
}

// LiquidationSweepPump's three ewm columns in ONE pass per row
// (bq_pump_ewm): high / low / close loaded once, the true range formed from
// them, and the three series scanned side by side on the same tiles —
// panel_ewm_kernel's map scan + exact replay per series (series 1 and 2 share
// the close values; pandas' recursion on thread 0 for a series from the first
// tile with a missing / infinite value, one series at a time through sX).
// trend_score = (ema20 - ema50) / ema50 (liquidation_sweep_pump.py:254, the
// staged program's operation) leaves with them when asked, so the pump pass
// does not read the two ema columns back.
struct PumpEwmArgs {
  const double *h, *l, *c;
  double* out[3];   // atr, ema20, ema50
  double* trend;    // NULL: skip
  int64_t ld_in, ld_out;
  int T, vin, vout;
  double alpha[3];
  int minp[3];
};

// 256 threads x 8 candles (the panel kernels' 2 048-candle tile and lane maps:
// the same association as panel_ewm_kernel, so the same bits), the series one
// after another, the serial state in LDS: 111 VGPRs, 4 waves per SIMD. At
// 12.5k x 2k 0.257 ms against 0.31 / 0.30 for 512 x 4 at 4 / 8 waves per SIMD
// and 0.27 for the two panel_ewm launches it replaces (tools/ab_kernel.sh).
#ifndef BQ_P3_K
#define BQ_P3_K 8
#endif
#ifndef BQ_P3_WPS
#define BQ_P3_WPS 4
#endif
constexpr int P3_K = BQ_P3_K;
constexpr int P3_NT = 2048 / P3_K;
constexpr int P3_NW = P3_NT / WAVE;
constexpr int P3_TT = P3_NT * P3_K;

__device__ __forceinline__ void p3_load(const double* __restrict__ row, int tb, int T, bool vec, double (&x)[P3_K]) {
  if (vec && tb + P3_K <= T) {
    const pn_dbl2* p = reinterpret_cast<const pn_dbl2*>(row + tb);
#pragma unroll
    for (int j = 0; j < P3_K / 2; ++j) {
      const pn_dbl2 a = p[j];
      x[2 * j] = a.x;
      x[2 * j + 1] = a.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < P3_K; ++k) x[k] = tb + k < T ? row[tb + k] : qnan();
  }
}

__global__ __launch_bounds__(P3_NT, BQ_P3_WPS) void pump_ewm3_kernel(const PumpEwmArgs A) {
  __shared__ double sA[P3_NW], sB[P3_NW];
  __shared__ double sCarry[3];
  __shared__ double sX[P3_TT];   // the serial replay's tile (one series at a time)
  __shared__ double sWv[3], sOwt[3];   // pandas' state of a serial series (thread 0)
  __shared__ int sNobs[3];
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const double* __restrict__ xh = A.h + row * A.ld_in;
  const double* __restrict__ xl = A.l + row * A.ld_in;
  const double* __restrict__ xc = A.c + row * A.ld_in;
  const int64_t orow = row * A.ld_out;
  const int T = A.T;
  const bool vin = A.vin != 0, vout = A.vout != 0;
  if (tid < 3) {
    sCarry[tid] = 0.0;
    sWv[tid] = qnan();
    sOwt[tid] = 1.0;
    sNobs[tid] = 0;
  }
  unsigned serial = 0;   // bit e: series e runs pandas' recursion (block-uniform)
  for (int t0 = 0; t0 < T; t0 += P3_TT) {
    const int tb = t0 + P3_K * tid;
    // loaded at the tile start, not a tile ahead: registers are occupancy
    // here, and a row of up to 2 048 candles is one tile anyway
    double v[2][P3_K];   // the true range; the close (+-inf: missing)
    {
      double nh[P3_K], nl[P3_K], nc[P3_K];
      p3_load(xh, tb, T, vin, nh);
      p3_load(xl, tb, T, vin, nl);
      p3_load(xc, tb, T, vin, nc);
      double pc = tb >= 1 && tb <= T ? xc[tb - 1] : qnan();
#pragma unroll
      for (int k = 0; k < P3_K; ++k) {
        v[0][k] = tb + k < T ? win_val(true_range(nh[k], nl[k], pc)) : qnan();
        v[1][k] = win_val(nc[k]);
        pc = nc[k];
      }
    }
    {
      int b0 = 0, b1 = 0;
#pragma unroll
      for (int k = 0; k < P3_K; ++k) {
        b0 |= (tb + k < T) && !(v[0][k] - v[0][k] == 0.0);
        b1 |= (tb + k < T) && !(v[1][k] - v[1][k] == 0.0);
      }
      const unsigned bad = (__syncthreads_or(b0) ? 1u : 0u) | (__syncthreads_or(b1) ? 6u : 0u);
      const unsigned turn = bad & ~serial;   // these series turn serial here
      if (turn && tid == 0 && t0 > 0)        // candles 0 .. t0 - 1 were all observations
        for (int e = 0; e < 3; ++e)
          if ((turn >> e) & 1) {
            sWv[e] = sCarry[e];
            sNobs[e] = t0;
          }
      serial |= bad;
    }
    double r20[P3_K];
    // one series at a time: the lane maps over its candles from the zero
    // state (candle 0 resets), their wave scans, the waves' totals through
    // LDS, then each lane's exact replay (or pandas' recursion on thread 0)
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const double al = A.alpha[e], om = 1.0 - al, den = om + al;
      const bool div = den != 1.0;
      const double* c = v[e == 0 ? 0 : 1];
      double res[P3_K];
      if ((serial >> e) & 1) {
#pragma unroll
        for (int k = 0; k < P3_K; ++k) sX[P3_K * tid + k] = c[k];
        __syncthreads();
        if (tid == 0) {
          const int n = min(P3_TT, T - t0);
          double y = sWv[e], ow = sOwt[e];
          int no = sNobs[e];
          for (int i = 0; i < n; ++i) {
            const double cur = sX[i];
            const bool obs = cur == cur;
            if (t0 + i == 0) {   // pandas: weighted = vals[0], nobs = its observation
              y = cur;
              no = obs ? 1 : 0;
            } else {
              no += obs ? 1 : 0;
              if (y == y) {
                ow *= om;
                if (obs) {
                  if (y != cur) {
                    y = ow * y + al * cur;
                    y /= ow + al;
                  }
                  ow = 1.0;
                }
              } else if (obs) {
                y = cur;
              }
            }
            sX[i] = no >= A.minp[e] ? y : qnan();
          }
          sWv[e] = y;
          sOwt[e] = ow;
          sNobs[e] = no;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < P3_K; ++k) res[k] = sX[P3_K * tid + k];
        __syncthreads();   // sX free for the next series
      } else {
        const double la = om / den, lb = al / den;
        double a_ = 1.0, b_ = 0.0;
#pragma unroll
        for (int k = 0; k < P3_K; ++k) {
          if (tb + k == 0) {
            a_ = 0.0;
            b_ = c[k];
          } else {
            a_ *= la;
            b_ = fma(la, b_, lb * c[k]);
          }
        }
        double sa = a_, sb = b_;
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
          const double pa = __shfl_up(sa, d, WAVE), pbv = __shfl_up(sb, d, WAVE);
          if (lane >= d) {
            sb = fma(sa, pbv, sb);
            sa *= pa;
          }
        }
        if (lane == WAVE - 1) {
          sA[w] = sa;
          sB[w] = sb;
        }
        double ea = __shfl_up(sa, 1, WAVE), eb = __shfl_up(sb, 1, WAVE);
        if (lane == 0) {
          ea = 1.0;
          eb = 0.0;
        }
        __syncthreads();
        double y = sCarry[e];
        for (int u = 0; u < w; ++u) y = fma(sA[u], y, sB[u]);
        y = fma(ea, y, eb);
#pragma unroll
        for (int k = 0; k < P3_K; ++k) {   // exact replay of the lane's steps
          const int t = tb + k;
          const double x = c[k];
          if (t == 0) y = x;
          else if (y != x) {
            y = om * y + al * x;
            if (div) y = y / den;
          }
          res[k] = t + 1 >= A.minp[e] ? y : qnan();
        }
        __syncthreads();   // sA / sB (and sCarry[e]) read by every wave
        if (tid == P3_NT - 1) sCarry[e] = y;   // the next tile's carry (nothing reads it before then)
      }
      store_lines<P3_K>(A.out[e] + orow, tb, T, vout, res);   // each column leaves as formed
      if (e == 1) {
#pragma unroll
        for (int k = 0; k < P3_K; ++k) r20[k] = res[k];
      }
      if (e == 2 && A.trend) {
#pragma unroll
        for (int k = 0; k < P3_K; ++k) r20[k] = (r20[k] - res[k]) / res[k];
        store_lines<P3_K>(A.trend + orow, tb, T, vout, r20);
      }
    }
  }
}

}  // namespace bq

// LiquidationSweepPump's per-symbol ewm columns in panel mode
// (liquidation_sweep_pump.py:206-217, 252-254): candidate_atr =
// TR.ewm(alpha = 1/14, min_periods = 14), ema20 / ema50 of close and, when
// asked, trend_score — one pass per row (pump_ewm3_kernel).
extern "C" int bq_pump_ewm(const double* high, const double* low, const double* close, int64_t S, int64_t T,
                           int64_t ld_in, double* atr, double* ema20, double* ema50, double* trend_score,
                           int64_t ld_out, void* stream) {
  using namespace bq;
  if (!high || !low || !close || !atr || !ema20 || !ema50 || S < 0 || T < 0 || ld_in < T || ld_out < T ||
      S > 0x7fffffff || T > 0x7fffffff - 2 * P3_TT)
    return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  PumpEwmArgs A;
  memset(&A, 0, sizeof(A));
  A.h = high;
  A.l = low;
  A.c = close;
  A.out[0] = atr;
  A.out[1] = ema20;
  A.out[2] = ema50;
  A.trend = trend_score;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  auto aligned = [](const void* p, int64_t ld) { return (((uintptr_t)p) & 15u) == 0 && (ld % 2) == 0; };
  A.vin = aligned(high, ld_in) && aligned(low, ld_in) && aligned(close, ld_in);
  A.vout = aligned(atr, ld_out) && aligned(ema20, ld_out) && aligned(ema50, ld_out) &&
           (!trend_score || aligned(trend_score, ld_out));
  // pandas: alpha = 1 / (1 + com), com = 1 / alpha - 1 or (span - 1) / 2
  const double coms[3] = {1.0 / (1.0 / 14.0) - 1.0, (20.0 - 1.0) / 2.0, (50.0 - 1.0) / 2.0};
  const int minp[3] = {14, 0, 0};
  for (int i = 0; i < 3; ++i) {
    A.alpha[i] = 1.0 / (1.0 + coms[i]);
    A.minp[i] = minp[i];
  }
  hipLaunchKernelGGL(pump_ewm3_kernel, dim3((unsigned)S), dim3(P3_NT), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
