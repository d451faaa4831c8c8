// Time-parallel kernels for the signal generators' inline helpers (SURVEY
// §8a a20) on a [S][T] panel, gfx950:
//
//   bq_wilder_rsi  MeanReversionFade._rsi          strategies/mean_reversion_fade.py:88-109
//   bq_zscore      RangeBbRsiMeanReversion._compute_zscore
//                                                  strategies/range_bb_rsi_mean_reversion.py:132-138
//   bq_adx         RangeBbRsiMeanReversion._compute_adx  (:101-130)
//
// evaluated at every candle t (column t = the helper on the prefix frame
// df.iloc[:t + 1]). The replay composition in binquant_amd.signals (exact=True)
// reproduces pandas bit for bit but is sequential per symbol (one lane per
// symbol: 12.5k symbols fill under 20 % of the SIMDs); these kernels split the
// time axis instead, at the north_star tolerance (1e-9 relative):
//
// One 256-thread workgroup per symbol walks the row in tiles of 2048 candles
// (8 consecutive candles per lane, 64-byte vector loads, the next tile
// prefetched into registers). Per-candle quantities go to an LDS ring (tile +
// 128-candle halo from the previous tile), stored lane-interleaved
// (position i at (i % 8) * (R / 8) + i / 8, so the lanes' k-th candles are
// adjacent: conflict-free). Rolling windows are one sliding walk per lane
// (w + 8 ring reads per 8 outputs). The Wilder EWMs are an associative scan of
// affine maps (wave shuffles + LDS across waves + a tile carry), after which
// each lane replays its 8 steps with pandas' exact ewm(adjust=False) update.
// pandas' rules are kept: constant windows (rolling mean returns the value,
// var returns 0), min_periods warm-up NaN, the helpers' fillna / where.
//
// Missing candles (NaN) follow pandas' rules: the z-score / ADX sliding sums
// exclude a missing value and count it (NaN while the window holds it, finite
// again once it has left); the Wilder RSI row is replayed serially with
// pandas' ewm update from the first tile holding a non-finite close (gap
// decay, observation count, a late first observation).
#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

constexpr int SG_NT = 256;
constexpr int SG_NW = SG_NT / WAVE;
constexpr int SG_K = 8;
constexpr int SG_TT = SG_NT * SG_K;   // 2048
constexpr int SG_H = 128;
constexpr int SG_R = SG_H + SG_TT;    // 2176
constexpr int SG_Q = SG_R / SG_K;     // 272
static_assert(SG_R % SG_K == 0 && SG_H % SG_K == 0, "ring shape");

// ring position p -> LDS slot (lane-interleaved)
__device__ __forceinline__ int sg_slot(int p) { return (p & (SG_K - 1)) * SG_Q + (p >> 3); }

typedef double sg_dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void sg_load(const double* __restrict__ row, int tb, int T, bool vec, double (&x)[SG_K]) {
  if (vec && tb + SG_K <= T) {
    const sg_dbl2* p = reinterpret_cast<const sg_dbl2*>(row + tb);
#pragma unroll
    for (int j = 0; j < SG_K / 2; ++j) {
      const sg_dbl2 a = p[j];
      x[2 * j] = a.x;
      x[2 * j + 1] = a.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < SG_K; ++k) x[k] = tb + k < T ? row[tb + k] : qnan();
  }
}

// whole-line stores (bq_device.h store_lines); every thread of the block calls it
__device__ __forceinline__ void sg_store(double* __restrict__ row, int tb, int T, bool vec, const double (&x)[SG_K]) {
  store_lines<SG_K>(row, tb, T, vec, x);
}

// Block-wide inclusive max of a per-lane int (>= -1): wave DPP scan, wave
// totals through LDS. Returns the exclusive prefix max over lower lanes
// combined with `carry` (the value carried from previous tiles).
__device__ __forceinline__ int sg_block_excl_max(int v, int carry, int* sW, int lane, int w) {
  const int inc = wave_scan_max_dpp(v + 1, lane) - 1;
  if (lane == WAVE - 1) sW[w] = inc;
  const int lpre = dpp_i32<DPP_WAVE_SHR1>(inc + 1) - 1;   // lane 0 -> -1
  __syncthreads();
  int c = max(carry, lpre);
  for (int u = 0; u < w; ++u) c = max(c, sW[u]);
  return c;
}

struct SigArgs {
  const double* in[3];   // close | high, low, close
  double* out;
  int64_t ld_in, ld_out;
  int T, win;
  int vin, vout;   // 16-byte aligned rows: vector loads / stores
  double inv_w;
  double alpha, om, den;   // Wilder EWM: alpha = 1 / win, om = 1 - alpha, den = om + alpha
};

// ---- zscore ----------------------------------------------------------------------
// mean = close.rolling(w, min_periods=w).mean(), std = .std(ddof=0);
// z = 0 where std == 0 or NaN (incl. the warm-up), else (c - mean) / std.
// W > 0: the window is the reference's (20), known at compile time, so the
// window walks unroll completely (same operations, same order); W = 0: any.
template <int W>
__global__ __launch_bounds__(SG_NT) void zscore_kernel(const SigArgs A) {
  __shared__ double sC[SG_R];
  __shared__ int sW[SG_NW];
  __shared__ int sCar;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t sym = blockIdx.x;
  const double* __restrict__ rc = A.in[0] + sym * A.ld_in;
  double* __restrict__ ro = A.out + sym * A.ld_out;
  const int T = A.T;
  const int win = W ? W : __builtin_amdgcn_readfirstlane(A.win);
  if (tid < SG_H) sC[sg_slot(tid)] = qnan();
  if (tid == 0) sCar = -1;
  double nx[SG_K];
  sg_load(rc, SG_K * tid, T, A.vin, nx);
  for (int t0 = 0; t0 < T; t0 += SG_TT) {
    const int tb = t0 + SG_K * tid, pb = SG_H + SG_K * tid;
    double c[SG_K];
#pragma unroll
    for (int k = 0; k < SG_K; ++k) c[k] = nx[k];
    if (t0 + SG_TT < T) sg_load(rc, tb + SG_TT, T, A.vin, nx);
#pragma unroll
    for (int k = 0; k < SG_K; ++k) sC[sg_slot(pb + k)] = c[k];
    __syncthreads();
    // last index where the close changed (pandas' same-value rule)
    int lcl[SG_K];
    {
      double pc = sC[sg_slot(pb - 1)];
      int run = -1;
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        if (tb + k == 0 || c[k] != pc) run = tb + k;
        lcl[k] = run;
        pc = c[k];
      }
      const int carry = sg_block_excl_max(lcl[SG_K - 1], sCar, sW, lane, w);
#pragma unroll
      for (int k = 0; k < SG_K; ++k) lcl[k] = max(lcl[k], carry);
    }
    double z[SG_K];
    {
      // windows reaching before candle 0 (first tile only) hold only the
      // candles from 0 on; those outputs are warm-up, but the sliding sums
      // must not carry the halo's NaN into the first complete window
      const int gs = SG_H - t0;   // ring position of candle 0
      // a finite lane-local reference (a missing candle is excluded from the
      // sums and counted: pandas' rolling(w, min_periods=w) is NaN while the
      // window holds one, z = 0 there, and finite again once it has left)
      double r = c[0];
#pragma unroll
      for (int k = 1; k < SG_K; ++k) r = r == r ? r : c[k];
      r = r == r ? r : 0.0;
      double s1 = 0.0, s2 = 0.0;
      int nn = 0;
      auto walk = [&](int x0) {
        const double v = sC[sg_slot(pb + x0)];
        const bool ok = v == v;
        const double d = ok ? v - r : 0.0;
        nn += ok ? 0 : 1;
        s1 += d;
        s2 = fma(d, d, s2);
      };
      if (W && gs - pb <= 1 - W) {
#pragma unroll
        for (int x = 1 - W; x <= 0; ++x) walk(x);
      } else {
        for (int x = max(1 - win, gs - pb); x <= 0; ++x) walk(x);
      }
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        const int t = tb + k;
        if (k > 0) {
          const bool oi = c[k] == c[k];
          const double dn = oi ? c[k] - r : 0.0;
          const double vo = pb + k - win >= gs ? sC[sg_slot(pb + k - win)] : r;
          const bool oo = vo == vo;
          const double dol = oo ? vo - r : 0.0;
          nn += (oi ? 0 : 1) - (oo ? 0 : 1);
          s1 = (s1 + dn) - dol;
          s2 = fma(-dol, dol, fma(dn, dn, s2));
        }
        double v = 0.0;
        if (t >= win - 1 && lcl[k] > t - win + 1 && nn == 0) {
          const double var = (s2 - s1 * s1 * A.inv_w) * A.inv_w;
          const double sd = var > 0.0 ? sqrt(var) : 0.0;
          const double mean = r + s1 * A.inv_w;
          if (sd > 0.0 && sd == sd) v = (c[k] - mean) / sd;
        }
        z[k] = v;
      }
    }
    sg_store(ro, tb, T, A.vout, z);
    if (t0 + SG_TT >= T) break;
    __syncthreads();
    if (pb >= SG_TT) {
#pragma unroll
      for (int k = 0; k < SG_K; ++k) sC[sg_slot(pb + k - SG_TT)] = c[k];
    }
    if (tid == SG_NT - 1) sCar = lcl[SG_K - 1];
  }
}

// ---- ADX --------------------------------------------------------------------------
// tr = max(h - l, |h - pc|, |l - pc|) (skip NaN), +DM / -DM, rolling(w) sums,
// DI = 100 * sum / atr_sum, dx = 100 |DI+ - DI-| / (DI+ + DI-) (0 for a zero
// or NaN denominator, fillna(0)), adx = dx.rolling(w).mean(), 100 where NaN.
template <int W>   // as zscore_kernel (the reference's window: 14)
__global__ __launch_bounds__(SG_NT) void adx_kernel(const SigArgs A) {
  __shared__ double sTR[SG_R], sPD[SG_R], sMD[SG_R], sDX[SG_R];
  __shared__ int sW[SG_NW], sW2[SG_NW];
  __shared__ int sCar[2];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t sym = blockIdx.x;
  const double* __restrict__ rh = A.in[0] + sym * A.ld_in;
  const double* __restrict__ rl = A.in[1] + sym * A.ld_in;
  const double* __restrict__ rc = A.in[2] + sym * A.ld_in;
  double* __restrict__ ro = A.out + sym * A.ld_out;
  const int T = A.T;
  const int win = W ? W : __builtin_amdgcn_readfirstlane(A.win);
  if (tid < SG_H) {
    sTR[sg_slot(tid)] = sPD[sg_slot(tid)] = sMD[sg_slot(tid)] = sDX[sg_slot(tid)] = 0.0;
  }
  if (tid < 2) sCar[tid] = -1;
  double nh[SG_K], nl[SG_K], nc[SG_K];
  sg_load(rh, SG_K * tid, T, A.vin, nh);
  sg_load(rl, SG_K * tid, T, A.vin, nl);
  sg_load(rc, SG_K * tid, T, A.vin, nc);
  for (int t0 = 0; t0 < T; t0 += SG_TT) {
    const int tb = t0 + SG_K * tid, pb = SG_H + SG_K * tid;
    double h[SG_K], l[SG_K], c[SG_K];
#pragma unroll
    for (int k = 0; k < SG_K; ++k) {
      h[k] = nh[k];
      l[k] = nl[k];
      c[k] = nc[k];
    }
    const double ph0 = tb >= 1 && tb <= T ? rh[tb - 1] : qnan();
    const double pl0 = tb >= 1 && tb <= T ? rl[tb - 1] : qnan();
    const double pc0 = tb >= 1 && tb <= T ? rc[tb - 1] : qnan();
    if (t0 + SG_TT < T) {
      sg_load(rh, tb + SG_TT, T, A.vin, nh);
      sg_load(rl, tb + SG_TT, T, A.vin, nl);
      sg_load(rc, tb + SG_TT, T, A.vin, nc);
    }
    double tr[SG_K], pd[SG_K], md[SG_K];
    {
      double ph = ph0, pl = pl0, pc = pc0;
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        tr[k] = true_range(h[k], l[k], pc);
        const double hd = h[k] - ph, ld = -(l[k] - pl);   // high.diff(), -low.diff()
        pd[k] = (hd > ld && hd > 0.0) ? hd : 0.0;
        md[k] = (ld > hd && ld > 0.0) ? ld : 0.0;
        sTR[sg_slot(pb + k)] = tr[k];
        sPD[sg_slot(pb + k)] = pd[k];
        sMD[sg_slot(pb + k)] = md[k];
        ph = h[k];
        pl = l[k];
        pc = c[k];
      }
    }
    __syncthreads();   // the ring (incl. the neighbour lanes' candles) is visible
    // constant-run starts of the three series (pandas' same-value rule for sums)
    int ltr[SG_K];
    {
      double ptr = sTR[sg_slot(pb - 1)], ppd = sPD[sg_slot(pb - 1)], pmd = sMD[sg_slot(pb - 1)];
      int run = -1;
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        if (tb + k == 0 || tr[k] != ptr || pd[k] != ppd || md[k] != pmd) run = tb + k;
        ltr[k] = run;
        ptr = tr[k];
        ppd = pd[k];
        pmd = md[k];
      }
      const int carry = sg_block_excl_max(ltr[SG_K - 1], sCar[0], sW, lane, w);
#pragma unroll
      for (int k = 0; k < SG_K; ++k) ltr[k] = max(ltr[k], carry);
    }
    // dx of the lane's candles
    double dx[SG_K];
    {
      // a true range that is NaN (a missing high / low / previous close the
      // skip-NaN max cannot cover) is excluded from the sliding sum and
      // counted: pandas' rolling(w).sum() is NaN while the window holds it
      // (dx = 0) and finite again once it has left
      double st = 0.0, sp = 0.0, sm = 0.0;
      int nn = 0;
      walk_window<(W > 0)>(1 - win, [&](int x) {
        const double a = sTR[sg_slot(pb + x)];
        st += a == a ? a : 0.0;
        nn += a == a ? 0 : 1;
        sp += sPD[sg_slot(pb + x)];
        sm += sMD[sg_slot(pb + x)];
      });
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        const int t = tb + k;
        if (k > 0) {
          const int o = sg_slot(pb + k - win);
          const double ai = tr[k], ao = sTR[o];
          st = (st + (ai == ai ? ai : 0.0)) - (ao == ao ? ao : 0.0);
          nn += (ai == ai ? 0 : 1) - (ao == ao ? 0 : 1);
          sp = (sp + pd[k]) - sPD[o];
          sm = (sm + md[k]) - sMD[o];
        }
        double v = 0.0;
        if (t >= win - 1) {
          double a = nn ? qnan() : st, p = sp, m = sm;
          if (ltr[k] <= t - win + 1) {   // constant window: value * nobs
            a = tr[k] * (double)win;
            p = pd[k] * (double)win;
            m = md[k] * (double)win;
          }
          const double pdi = 100.0 * p / a, mdi = 100.0 * m / a;
          const double tot = pdi + mdi;
          v = tot != 0.0 ? 100.0 * fabs(pdi - mdi) / tot : qnan();
          if (v != v) v = 0.0;
        }
        dx[k] = v;
        sDX[sg_slot(pb + k)] = v;
      }
    }
    __syncthreads();   // dx of every lane visible
    int ldx[SG_K];
    {
      double pv = sDX[sg_slot(pb - 1)];
      int run = -1;
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        if (tb + k == 0 || dx[k] != pv) run = tb + k;
        ldx[k] = run;
        pv = dx[k];
      }
      const int carry = sg_block_excl_max(ldx[SG_K - 1], sCar[1], sW2, lane, w);
#pragma unroll
      for (int k = 0; k < SG_K; ++k) ldx[k] = max(ldx[k], carry);
    }
    double adx[SG_K];
    {
      double s = 0.0;
      walk_window<(W > 0)>(1 - win, [&](int x) { s += sDX[sg_slot(pb + x)]; });
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        const int t = tb + k;
        if (k > 0) s = (s + dx[k]) - sDX[sg_slot(pb + k - win)];
        double v = 100.0;
        if (t >= win - 1) {
          if (ldx[k] <= t - win + 1) v = dx[k];
          else v = div_exact(s < 0.0 ? 0.0 : s, (double)win, A.inv_w);
        }
        adx[k] = v;
      }
    }
    sg_store(ro, tb, T, A.vout, adx);
    if (t0 + SG_TT >= T) break;
    __syncthreads();
    if (pb >= SG_TT) {
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        const int d = sg_slot(pb + k - SG_TT);
        sTR[d] = tr[k];
        sPD[d] = pd[k];
        sMD[d] = md[k];
        sDX[d] = dx[k];
      }
    }
    if (tid == SG_NT - 1) {
      sCar[0] = ltr[SG_K - 1];
      sCar[1] = ldx[SG_K - 1];
    }
  }
}

// ---- Wilder RSI ----------------------------------------------------------------
// gain / loss = delta.clip(lower=0) / -delta.clip(upper=0) (NaN at candle 0),
// avg = ewm(alpha = 1 / w, min_periods = w, adjust=False).mean() (the first
// observation, candle 1, starts the average), rsi = 100 avg_g / (avg_g +
// avg_l), 50 where the denominator is 0, NaN during the warm-up.
template <bool DIV>
__device__ __forceinline__ double wilder_step(double y, double x, const SigArgs& A) {
  if (y != x) {
    y = A.om * y + A.alpha * x;
    if (DIV) y = y / A.den;
  }
  return y;
}

template <bool DIV>
__global__ __launch_bounds__(SG_NT) void wilder_rsi_kernel(const SigArgs A) {
  __shared__ double sA[SG_NW], sB[2][SG_NW];
  __shared__ double sCarry[2];
  __shared__ double sX[SG_TT];   // the serial replay's tile (rows with missing candles)
  __shared__ double sSt[4];      // its pandas state: avg gain, avg loss, old weight, previous close
  __shared__ int sNobs;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t sym = blockIdx.x;
  const double* __restrict__ rc = A.in[0] + sym * A.ld_in;
  double* __restrict__ ro = A.out + sym * A.ld_out;
  const int T = A.T;
  // the scan's per-candle map: y -> la * y + lb * x (la = om / den, lb = alpha / den)
  const double la = A.om / A.den, lb = A.alpha / A.den;
  if (tid < 2) sCarry[tid] = 0.0;
  // pandas' ewm state once the row turns serial (LDS, thread 0): averages,
  // old weight, previous close, observation count
  bool serial = false;
  if (tid == 0) {
    sSt[0] = sSt[1] = sSt[3] = qnan();
    sSt[2] = 1.0;
    sNobs = 0;
  }
  double nx[SG_K];
  sg_load(rc, SG_K * tid, T, A.vin, nx);
  for (int t0 = 0; t0 < T; t0 += SG_TT) {
    const int tb = t0 + SG_K * tid;
    double c[SG_K];
#pragma unroll
    for (int k = 0; k < SG_K; ++k) c[k] = nx[k];
    const double pc0 = tb >= 1 && tb <= T ? rc[tb - 1] : qnan();
    if (t0 + SG_TT < T) sg_load(rc, tb + SG_TT, T, A.vin, nx);
    // A missing (NaN) or infinite close breaks the scan's fixed per-candle
    // map: pandas' ewm(ignore_na=False) decays the old weight across a gap
    // and divides by (old_wt + alpha), counts only observations toward
    // min_periods and starts at the first observation wherever it is. From
    // the first tile holding one, the row is replayed serially with pandas'
    // own update (thread 0; the carry so far seeds it) — exact, and only the
    // rows with gaps pay for it.
    {
      int bad = 0;
#pragma unroll
      for (int k = 0; k < SG_K; ++k) bad |= (tb + k < T) && !(c[k] - c[k] == 0.0);
      if (__syncthreads_or(bad) && !serial) {
        serial = true;
        if (t0 > 0 && tid == 0) {   // candles 1 .. t0 - 1 were all observations
          sSt[0] = sCarry[0];
          sSt[1] = sCarry[1];
          sSt[3] = rc[t0 - 1];
          sNobs = t0 - 1;
        }
      }
    }
    if (serial) {
#pragma unroll
      for (int k = 0; k < SG_K; ++k) sX[SG_K * tid + k] = c[k];
      __syncthreads();
      if (tid == 0) {
        double wg = sSt[0], wl = sSt[1], owt = sSt[2], prev = sSt[3];
        int nobs = sNobs;
        const int n = min(SG_TT, T - t0);
        for (int i = 0; i < n; ++i) {
          const double cur = sX[i];
          const double d = cur - prev;
          prev = cur;
          const double g = d != d ? d : (d > 0.0 ? d : 0.0);
          const double l = d != d ? d : (d < 0.0 ? -d : 0.0);
          const bool obs = g == g;
          nobs += obs ? 1 : 0;
          if (wg == wg) {
            owt *= A.om;
            if (obs) {
              if (wg != g) {
                wg = owt * wg + A.alpha * g;
                wg /= owt + A.alpha;
              }
              if (wl != l) {
                wl = owt * wl + A.alpha * l;
                wl /= owt + A.alpha;
              }
              owt = 1.0;
            }
          } else if (obs) {
            wg = g;
            wl = l;
          }
          double v = qnan();
          if (nobs >= A.win) {
            const double den = wg + wl;
            v = den != 0.0 ? (100.0 * wg) / den : 50.0;
          }
          sX[i] = v;
        }
        sSt[0] = wg;
        sSt[1] = wl;
        sSt[2] = owt;
        sSt[3] = prev;
        sNobs = nobs;
      }
      __syncthreads();
      double rsi[SG_K];
#pragma unroll
      for (int k = 0; k < SG_K; ++k) rsi[k] = sX[SG_K * tid + k];
      sg_store(ro, tb, T, A.vout, rsi);
      if (t0 + SG_TT >= T) break;
      __syncthreads();
      continue;
    }
    double g[SG_K], l[SG_K];
    {
      double pc = pc0;
#pragma unroll
      for (int k = 0; k < SG_K; ++k) {
        const double d = c[k] - pc;
        g[k] = d != d ? d : (d > 0.0 ? d : 0.0);
        l[k] = d != d ? d : (d < 0.0 ? -d : 0.0);
        pc = c[k];
      }
    }
    // lane map over its K candles from the zero state; candle 1 (the first
    // observation) resets the state: a = 0, b = x
    double A_ = 1.0, Bg = 0.0, Bl = 0.0;
#pragma unroll
    for (int k = 0; k < SG_K; ++k) {
      const int t = tb + k;
      if (t == 0) continue;   // NaN observation before any: no state
      if (t == 1) {
        A_ = 0.0;
        Bg = g[k];
        Bl = l[k];
      } else {
        A_ *= la;
        Bg = fma(la, Bg, lb * g[k]);
        Bl = fma(la, Bl, lb * l[k]);
      }
    }
    // block exclusive scan of (A, Bg, Bl): wave Hillis-Steele with shuffles
    double sa = A_, sg = Bg, sl = Bl;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const double pa = __shfl_up(sa, d, WAVE), pg = __shfl_up(sg, d, WAVE), pl = __shfl_up(sl, d, WAVE);
      if (lane >= d) {   // (sa, sg) after (pa, pg)
        sg = fma(sa, pg, sg);
        sl = fma(sa, pl, sl);
        sa *= pa;
      }
    }
    if (lane == WAVE - 1) {
      sA[w] = sa;
      sB[0][w] = sg;
      sB[1][w] = sl;
    }
    // exclusive within the wave
    double ea = __shfl_up(sa, 1, WAVE), eg = __shfl_up(sg, 1, WAVE), el = __shfl_up(sl, 1, WAVE);
    if (lane == 0) {
      ea = 1.0;
      eg = el = 0.0;
    }
    __syncthreads();
    double yg = sCarry[0], yl = sCarry[1];
    for (int u = 0; u < w; ++u) {
      yg = fma(sA[u], yg, sB[0][u]);
      yl = fma(sA[u], yl, sB[1][u]);
    }
    yg = fma(ea, yg, eg);
    yl = fma(ea, yl, el);
    // exact replay of the lane's K steps
    double rsi[SG_K];
#pragma unroll
    for (int k = 0; k < SG_K; ++k) {
      const int t = tb + k;
      if (t == 1) {
        yg = g[k];
        yl = l[k];
      } else if (t > 1) {
        yg = wilder_step<DIV>(yg, g[k], A);
        yl = wilder_step<DIV>(yl, l[k], A);
      }
      double v = qnan();
      if (t >= A.win && t < T) {   // nobs (candles 1..t) >= min_periods
        const double den = yg + yl;
        v = den != 0.0 ? (100.0 * yg) / den : 50.0;
      }
      rsi[k] = v;
    }
    sg_store(ro, tb, T, A.vout, rsi);
    if (t0 + SG_TT >= T) break;
    __syncthreads();
    if (tid == SG_NT - 1) {
      sCarry[0] = yg;
      sCarry[1] = yl;
    }
    __syncthreads();
  }
}

// 16-byte vector access needs every row start 16-byte aligned
static void set_vec(SigArgs& A, int64_t ld_in, int64_t ld_out, int n_in) {
  auto al = [](const void* p) { return (((uintptr_t)p) & 15u) == 0; };
  A.vin = (ld_in % 2) == 0;
  for (int i = 0; i < n_in; ++i) A.vin &= al(A.in[i]);
  A.vout = (ld_out % 2) == 0 && al(A.out);
}

static bool sig_ok(const void* a, int64_t S, int64_t T, int64_t ld_in, int64_t ld_out, const void* out, int w,
                   int wmax) {
  return a && out && S >= 0 && T >= 0 && ld_in >= T && ld_out >= T && T <= 0x7fffffff - 2 * SG_TT &&
         S <= 0x7fffffff && w >= 1 && w <= wmax;
}

}  // namespace bq

extern "C" {

int bq_zscore(const double* close, int64_t S, int64_t T, int64_t ld_in, int32_t window, double* out, int64_t ld_out,
              void* stream) {
  using namespace bq;
  if (!sig_ok(close, S, T, ld_in, ld_out, out, window, BQ_MAX_WINDOW)) return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  SigArgs A;
  memset(&A, 0, sizeof A);
  A.in[0] = close;
  A.out = out;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.win = window;
  A.inv_w = 1.0 / (double)window;
  set_vec(A, ld_in, ld_out, 1);
  if (window == 20) hipLaunchKernelGGL(zscore_kernel<20>, dim3((unsigned)S), dim3(SG_NT), 0, (hipStream_t)stream, A);
  else hipLaunchKernelGGL(zscore_kernel<0>, dim3((unsigned)S), dim3(SG_NT), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_adx(const double* high, const double* low, const double* close, int64_t S, int64_t T, int64_t ld_in,
           int32_t window, double* out, int64_t ld_out, void* stream) {
  using namespace bq;
  // the mean of dx reaches 2 (w - 1) candles back: inside the 128-candle halo
  if (!high || !low || !sig_ok(close, S, T, ld_in, ld_out, out, window, SG_H / 2)) return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  SigArgs A;
  memset(&A, 0, sizeof A);
  A.in[0] = high;
  A.in[1] = low;
  A.in[2] = close;
  A.out = out;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.win = window;
  A.inv_w = 1.0 / (double)window;
  set_vec(A, ld_in, ld_out, 3);
  if (window == 14) hipLaunchKernelGGL(adx_kernel<14>, dim3((unsigned)S), dim3(SG_NT), 0, (hipStream_t)stream, A);
  else hipLaunchKernelGGL(adx_kernel<0>, dim3((unsigned)S), dim3(SG_NT), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_wilder_rsi(const double* close, int64_t S, int64_t T, int64_t ld_in, int32_t window, double* out,
                  int64_t ld_out, void* stream) {
  using namespace bq;
  if (!sig_ok(close, S, T, ld_in, ld_out, out, window, 1 << 20)) return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  SigArgs A;
  memset(&A, 0, sizeof A);
  A.in[0] = close;
  A.out = out;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.win = window;
  // pandas: ewm(alpha = 1 / w) keeps com = 1 / alpha - 1 and recomputes
  // alpha = 1 / (1 + com); old_wt_factor = 1 - alpha, new_wt = alpha
  A.alpha = 1.0 / (1.0 + (1.0 / (1.0 / (double)window) - 1.0));
  A.om = 1.0 - A.alpha;
  A.den = A.om + A.alpha;
  set_vec(A, ld_in, ld_out, 1);
  if (A.den != 1.0)
    hipLaunchKernelGGL(wilder_rsi_kernel<true>, dim3((unsigned)S), dim3(SG_NT), 0, (hipStream_t)stream, A);
  else
    hipLaunchKernelGGL(wilder_rsi_kernel<false>, dim3((unsigned)S), dim3(SG_NT), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
