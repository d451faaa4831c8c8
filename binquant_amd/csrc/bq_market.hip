// Market-context kernels for gfx950: per-symbol features at every timestamp and
// the deterministic cross-symbol breadth partial sums.
//
// bq_market_features restates, for every timestamp t of a [S][T] panel,
//   LiveMarketContextAccumulator._compute_symbol_features
//   (market_regime/live_market_context_accumulator.py:244-297)
// applied to the history the MarketStateStore would hold at t: the last
// `max_bars` candles (market_regime/market_state_store.py:25-29 tail()).
//   * ema20/ema50 = ewm(span, adjust=False, min_periods=1) seeded at the first
//     candle of that window. Computed from the full-history EMA Y (affine scan,
//     as in bq_enrich) with the exact windowing identity
//       y_t = Y_t - a^(M-1) * (Y_s - c_s),  s = t - M + 1,
//     which needs Y_s - c_s M-1 candles back: that difference is kept in
//     LDS with a 512-candle halo; close and the prefix sums only need the
//     short windows' 32-candle halo (LDS 50 KB: 3 workgroups per CU).
//   * ATR = TR.rolling(14, min_periods=1).mean(); BB mid/std(ddof=0) over
//     rolling(20, min_periods=1): compensated prefix-sum differences with the
//     pandas constant-window rules, two-pass variance.
// One 256-thread workgroup per symbol, tiles of 1024 candles (4 per lane).
//
// bq_breadth_partial sums the per-symbol features over the symbols of the
// shard for every t (the counts and sums of _build_context,
// live_market_context_accumulator.py:135-163) in a fixed order.
#include "bq_device.h"
#include "binquant_amd.h"

#include <stdlib.h>
#include <string.h>

namespace bq {

constexpr int MF_NT = 256;
constexpr int MF_NW = MF_NT / WAVE;
constexpr int MF_K = 4;
constexpr int MF_TT = MF_NT * MF_K;
constexpr int MF_H = BQ_MAX_HISTORY;   // halo of the window-seeded EMA terms
constexpr int MF_R = MF_H + MF_TT;
constexpr int MF_HS = 32;              // halo of the short windows (ATR 14, BB 20)
constexpr int MF_RS = MF_HS + MF_TT;
#ifndef BQ_MF_LDSPERM
#define BQ_MF_LDSPERM 1   // lane-interleaved short-halo arrays (as bq_enrich's LX)
#endif
// slot of short-halo ring position i: lanes own 4 consecutive positions, so
// in the natural layout the 64 lanes of a wave touch slots 4 doubles apart (a
// 4-way bank conflict on every access); position i at (i % 4) * (RS / 4) +
// i / 4 puts the lanes' k-th candles side by side. qb is a multiple of 4, so
// for a constant offset x the slot of qb + x is (qb / 4) + a constant.
#if BQ_MF_LDSPERM
#define FX(i) (((((i) & 3)) * (MF_RS / 4)) + ((i) >> 2))
#else
#define FX(i) (i)
#endif
#ifndef BQ_MF_PREFETCH
#define BQ_MF_PREFETCH 0   // register prefetch of the next tile's inputs
#endif
constexpr int ATR_W = 14;   // live_market_context_accumulator.py:268
constexpr int BB_W = 20;    // :269-270

struct FeatArgs {
  const double* h;
  const double* l;
  const double* c;
  double* out[BQ_NUM_FEATURES];
  int64_t ld_in, ld_out;
  int T, M;
  double alpha[2], om[2], den[2], lin_a[2], lin_b[2];
  double apow[2][8];
  double corr[2];   // lin_a^(M-1)
};

__device__ __forceinline__ void mf_load(const double* __restrict__ row, int tb, int T, bool vec,
                                        double (&x)[MF_K]) {
  if (vec && tb + MF_K <= T) {
    const double2* p = reinterpret_cast<const double2*>(row + tb);
    double2 a = p[0], b = p[1];
    x[0] = a.x; x[1] = a.y; x[2] = b.x; x[3] = b.y;
  } else {
#pragma unroll
    for (int k = 0; k < MF_K; ++k) x[k] = (tb + k < T) ? row[tb + k] : 0.0;
  }
}

typedef double mdbl2 __attribute__((ext_vector_type(2)));

// whole-line stores (bq_device.h store_lines); called by every thread of the block
__device__ __forceinline__ void mf_store(double* __restrict__ row, int tb, int T, bool vec,
                                         const double (&x)[MF_K]) {
  store_lines<MF_K>(row, tb, T, vec, x);
}

#ifndef BQ_MF_WPS
#define BQ_MF_WPS 1   // __launch_bounds__ min waves per SIMD
#endif
// DIV: the EMAs need pandas' `/ (old_wt + new_wt)` (a non-unit sum; for the
// reference's spans 20 / 50 the sum is exactly 1.0 and the divide is the
// identity — checked on the host with the same IEEE arithmetic)
template <bool DIV>
__global__ __launch_bounds__(MF_NT, BQ_MF_WPS) void features_kernel(const FeatArgs A, int vec_in, int vec_out) {
  __shared__ double sPc[MF_RS], sPt[MF_RS], sC[MF_RS];
  __shared__ double sD[2][MF_R];   // Y_e - close (EMA window identity)
  __shared__ double sX[4][MF_NW + 1];   // c, c[-2], h, l of each wave's last candle
  __shared__ double sWh[2][MF_NW], sWl[2][MF_NW], sWe[2][MF_NW];
  __shared__ int sWlc[2][MF_NW];
  __shared__ double sEcar[2];
  __shared__ int sLcar[2];

  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t sym = blockIdx.x;
  const int T = A.T, M = A.M;
  const double* __restrict__ rH = A.h + sym * A.ld_in;
  const double* __restrict__ rL = A.l + sym * A.ld_in;
  const double* __restrict__ rC = A.c + sym * A.ld_in;
  const bool vin = vec_in != 0, vout = vec_out != 0;

  if (tid < 2) {
    sEcar[tid] = 0.0;
    sLcar[tid] = -1;
  }
  if (tid < 4) sX[tid][0] = qnan();
  for (int i = tid; i < MF_H; i += MF_NT) {
    sD[0][i] = qnan();
    sD[1][i] = qnan();
  }
  if (tid < MF_HS) {
    sPc[FX(tid)] = 0.0;
    sPt[FX(tid)] = 0.0;
    sC[FX(tid)] = qnan();
  }
  __syncthreads();

#if BQ_MF_PREFETCH
  double nh[MF_K], nl[MF_K], nc[MF_K];   // the next tile's inputs, in flight during this one
  mf_load(rH, MF_K * tid, T, vin, nh);
  mf_load(rL, MF_K * tid, T, vin, nl);
  mf_load(rC, MF_K * tid, T, vin, nc);
#endif
  for (int t0 = 0; t0 < T; t0 += MF_TT) {
    const int tb = t0 + MF_K * tid;
    const int pb = MF_H + MF_K * tid;     // position in the long-halo arrays
    const int qb = MF_HS + MF_K * tid;    // position in the short-halo arrays
    double h[MF_K], l[MF_K], c[MF_K];
#if BQ_MF_PREFETCH
#pragma unroll
    for (int k = 0; k < MF_K; ++k) {
      h[k] = nh[k];
      l[k] = nl[k];
      c[k] = nc[k];
    }
    if (t0 + MF_TT < T) {
      mf_load(rH, tb + MF_TT, T, vin, nh);
      mf_load(rL, tb + MF_TT, T, vin, nl);
      mf_load(rC, tb + MF_TT, T, vin, nc);
    }
#else
    mf_load(rH, tb, T, vin, h);
    mf_load(rL, tb, T, vin, l);
    mf_load(rC, tb, T, vin, c);
#endif

    // neighbour values and scans on DPP (VALU) moves; lane 0's are replaced below
    double pc1 = dpp_f64<DPP_WAVE_SHR1>(c[MF_K - 1]);
    double pc2 = dpp_f64<DPP_WAVE_SHR1>(c[MF_K - 2]);
    double ph = dpp_f64<DPP_WAVE_SHR1>(h[MF_K - 1]);
    double pl = dpp_f64<DPP_WAVE_SHR1>(l[MF_K - 1]);
    if (lane == WAVE - 1) {
      sX[0][w + 1] = c[MF_K - 1];
      sX[1][w + 1] = c[MF_K - 2];
      sX[2][w + 1] = h[MF_K - 1];
      sX[3][w + 1] = l[MF_K - 1];
    }
#pragma unroll
    for (int k = 0; k < MF_K; ++k) sC[FX(qb + k)] = c[k];
    __syncthreads();   // B1
    if (lane == 0) {
      pc1 = sX[0][w];
      pc2 = sX[1][w];
      ph = sX[2][w];
      pl = sX[3][w];
    }

    double tr[MF_K];
    int lcc[MF_K], lct[MF_K];
    {
      double pcv = pc1, ptr = true_range(ph, pl, pc2), cp = pc1;
      int rc = -1, rt = -1;
#pragma unroll
      for (int k = 0; k < MF_K; ++k) {
        const int t = tb + k;
        tr[k] = true_range(h[k], l[k], cp);
        if (t == 0 || c[k] != pcv) rc = t;
        if (t == 0 || tr[k] != ptr) rt = t;
        lcc[k] = rc;
        lct[k] = rt;
        pcv = c[k];
        ptr = tr[k];
        cp = c[k];
      }
    }

    // ---- wave scans ---------------------------------------------------------
    dd preC, preT;
    {
      dd tc = {0.0, 0.0}, tt = {0.0, 0.0};
#pragma unroll
      for (int k = 0; k < MF_K; ++k) {
        tc = dd_add1(tc, c[k]);
        tt = dd_add1(tt, tr[k]);
      }
      dd ic = wave_scan_dd_dpp(tc, lane), it = wave_scan_dd_dpp(tt, lane);
      if (lane == WAVE - 1) {
        sWh[0][w] = ic.hi; sWl[0][w] = ic.lo;
        sWh[1][w] = it.hi; sWl[1][w] = it.lo;
      }
      double a0 = dpp_f64<DPP_WAVE_SHR1>(ic.hi), a1 = dpp_f64<DPP_WAVE_SHR1>(ic.lo);
      double b0 = dpp_f64<DPP_WAVE_SHR1>(it.hi), b1 = dpp_f64<DPP_WAVE_SHR1>(it.lo);
      preC = lane == 0 ? dd{0.0, 0.0} : dd{a0, a1};
      preT = lane == 0 ? dd{0.0, 0.0} : dd{b0, b1};
    }
    double epre[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      double y = 0.0;
#pragma unroll
      for (int k = 0; k < MF_K; ++k) y = (tb + k == 0) ? c[k] : fma(A.lin_a[e], y, A.lin_b[e] * c[k]);
      double inc = wave_scan_affine_dpp(y, A.apow[e], lane);
      if (lane == WAVE - 1) sWe[e][w] = inc;
      double ex = dpp_f64<DPP_WAVE_SHR1>(inc);
      epre[e] = lane == 0 ? 0.0 : ex;
    }
    int lpc, lpt;
    {
      // indices >= -1: scanned as index + 1 so DPP's zero fill is the identity
      int ic = wave_scan_max_dpp(lcc[MF_K - 1] + 1, lane) - 1, it = wave_scan_max_dpp(lct[MF_K - 1] + 1, lane) - 1;
      if (lane == WAVE - 1) {
        sWlc[0][w] = ic;
        sWlc[1][w] = it;
      }
      int a = dpp_i32<DPP_WAVE_SHR1>(ic + 1) - 1, b = dpp_i32<DPP_WAVE_SHR1>(it + 1) - 1;
      lpc = lane == 0 ? -1 : a;
      lpt = lane == 0 ? -1 : b;
    }
    __syncthreads();   // B2

    {
      dd bc = {0.0, 0.0}, bt = {0.0, 0.0};
      for (int u = 0; u < w; ++u) {
        bc = dd_add(bc, dd{sWh[0][u], sWl[0][u]});
        bt = dd_add(bt, dd{sWh[1][u], sWl[1][u]});
      }
      bc = dd_add(bc, preC);
      bt = dd_add(bt, preT);
#pragma unroll
      for (int k = 0; k < MF_K; ++k) {
        bc = dd_add1(bc, c[k]);
        bt = dd_add1(bt, tr[k]);
        sPc[FX(qb + k)] = dd_round(bc);
        sPt[FX(qb + k)] = dd_round(bt);
      }
      int cc = sLcar[0], ct = sLcar[1];
      for (int u = 0; u < w; ++u) {
        cc = max(cc, sWlc[0][u]);
        ct = max(ct, sWlc[1][u]);
      }
      cc = max(cc, lpc);
      ct = max(ct, lpt);
#pragma unroll
      for (int k = 0; k < MF_K; ++k) {
        lcc[k] = max(lcc[k], cc);
        lct[k] = max(lct[k], ct);
      }
    }
    double Y[2][MF_K];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      double C = sEcar[e];
      for (int u = 0; u < w; ++u) C = fma(A.apow[e][6], C, sWe[e][u]);
      double y = lane == 0 ? C : fma(pow_bits<6>(A.apow[e], lane), C, epre[e]);
      const double al = A.alpha[e], om = A.om[e], dn = A.den[e];
#pragma unroll
      for (int k = 0; k < MF_K; ++k) {
        const double x = c[k];
        if (tb + k == 0) y = x;
        else if (y != x) y = DIV ? (om * y + al * x) / dn : om * y + al * x;
        Y[e][k] = y;
        sD[e][pb + k] = y - x;
      }
    }
    __syncthreads();   // B3

    // ---- features ----------------------------------------------------------
    double fr[MF_K], fe20[MF_K], fe50[MF_K], ftr[MF_K], fap[MF_K], fbw[MF_K];
    // Steady state (the lane's first candle has a full 20-candle window under
    // the history cap, so all four do): the four Bollinger windows share one pass over the 23
    // ring values they cover — each value read once and folded into every
    // window holding it, each window's squares still summed in ascending
    // order — and the divisions by the window lengths are div_count (IEEE-
    // exact): the same results as the per-candle path below.
    const bool steady = M >= BB_W && tb >= BB_W - 1;   // (history cap >= both windows)
    double bmid[MF_K], bacc[MF_K];
    if (steady) {
#pragma unroll
      for (int k = 0; k < MF_K; ++k) {
        bmid[k] = div_count(sPc[FX(qb + k)] - sPc[FX(qb + k - BB_W)], (double)BB_W, 1.0 / BB_W);
        bacc[k] = 0.0;
      }
#pragma unroll
      for (int m = 0; m < BB_W + MF_K - 1; ++m) {
        const double v = sC[FX(qb - (BB_W - 1) + m)];
#pragma unroll
        for (int k = 0; k < MF_K; ++k) {
          if (m - k >= 0 && m - k < BB_W) {
            const double d = v - bmid[k];
            bacc[k] = fma(d, d, bacc[k]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < MF_K; ++k) {
      const int t = tb + k, p = pb + k, q = qb + k;
      const int n = min(t + 1, M);
      if (n < 2) {   // history.empty or len < 2 -> None (:248-249)
        fr[k] = fe20[k] = fe50[k] = ftr[k] = fap[k] = fbw[k] = qnan();
        continue;
      }
      const double cl = c[k];
      const double prev = k > 0 ? c[k - 1] : pc1;
      double e20 = Y[0][k], e50 = Y[1][k];
      if (t + 1 > M) {   // history window starts at s = t - M + 1 > 0
        const int ps = p - M + 1;
        e20 = e20 - A.corr[0] * sD[0][ps];
        e50 = e50 - A.corr[1] * sD[1][ps];
      }
      // ATR: TR.rolling(14, min_periods=1).mean() at the last row (:268)
      const int ma = min(ATR_W, n);
      double atr;
      if (lct[k] <= t - ma + 1) atr = tr[k];
      else {
        double S = sPt[FX(q)] - sPt[FX(q - ma)];
        S = S < 0.0 ? 0.0 : S;
        atr = steady ? div_count(S, (double)ATR_W, 1.0 / ATR_W) : S / (double)ma;
      }
      // BB: rolling(20, min_periods=1) mean / std(ddof=0).fillna(0) (:269-272)
      const int mb = min(BB_W, n);
      double mid, sd;
      if (lcc[k] <= t - mb + 1) {
        mid = cl;
        sd = 0.0;
      } else if (steady) {
        mid = bmid[k];
        sd = sqrt(div_count(bacc[k], (double)BB_W, 1.0 / BB_W));
      } else {
        mid = (sPc[FX(q)] - sPc[FX(q - mb)]) / (double)mb;
        double acc = 0.0;
        if (mb == BB_W) {   // every candle past the warm-up: a compile-time walk,
                            // all 20 ring reads issued ahead of the sum (same order)
#pragma unroll
          for (int j = 1 - BB_W; j <= 0; ++j) {
            const double d = sC[FX(q + j)] - mid;
            acc = fma(d, d, acc);
          }
        } else {
          for (int i = q - mb + 1; i <= q; ++i) {
            const double d = sC[FX(i)] - mid;
            acc = fma(d, d, acc);
          }
        }
        sd = sqrt(acc / (double)mb);
      }
      const double up = mid + (2.0 * sd), lo = mid - (2.0 * sd);
      fr[k] = safe_pct(cl, prev);
      fe20[k] = e20;
      fe50[k] = e50;
      ftr[k] = e50 != 0.0 ? (e20 - e50) / fabs(e50) : 0.0;
      fap[k] = cl != 0.0 ? atr / cl : 0.0;
      fbw[k] = mid != 0.0 ? (up - lo) / fabs(mid) : 0.0;
    }
    const int64_t orow = sym * A.ld_out;
    if (A.out[BQ_F_RETURN]) mf_store(A.out[BQ_F_RETURN] + orow, tb, T, vout, fr);
    if (A.out[BQ_F_EMA20]) mf_store(A.out[BQ_F_EMA20] + orow, tb, T, vout, fe20);
    if (A.out[BQ_F_EMA50]) mf_store(A.out[BQ_F_EMA50] + orow, tb, T, vout, fe50);
    if (A.out[BQ_F_TREND]) mf_store(A.out[BQ_F_TREND] + orow, tb, T, vout, ftr);
    if (A.out[BQ_F_ATR_PCT]) mf_store(A.out[BQ_F_ATR_PCT] + orow, tb, T, vout, fap);
    if (A.out[BQ_F_BB_WIDTH]) mf_store(A.out[BQ_F_BB_WIDTH] + orow, tb, T, vout, fbw);

    if (t0 + MF_TT >= T) break;
    __syncthreads();   // B4
    for (int i = tid; i < MF_H; i += MF_NT) {
      sD[0][i] = sD[0][MF_TT + i];
      sD[1][i] = sD[1][MF_TT + i];
    }
    if (tid < MF_HS) {   // short halos; prefixes re-based to the tile end
      const int src = MF_TT + tid;
      sPc[FX(tid)] = sPc[FX(src)] - sPc[FX(MF_RS - 1)];
      sPt[FX(tid)] = sPt[FX(src)] - sPt[FX(MF_RS - 1)];
      sC[FX(tid)] = sC[FX(src)];
    }
    if (tid < 4) sX[tid][0] = sX[tid][MF_NW];
    if (tid == MF_NT - 1) {
      sEcar[0] = Y[0][MF_K - 1];
      sEcar[1] = Y[1][MF_K - 1];
      sLcar[0] = lcc[MF_K - 1];
      sLcar[1] = lct[MF_K - 1];
    }
    __syncthreads();   // B5
  }
}

// ---- breadth partials ---------------------------------------------------------
// One workgroup of BR_NW waves owns BR_TW consecutive timestamps; wave u sums
// symbols s = u, u + BR_NW, ... in ascending order, lane = timestamp. The wave
// partials are then combined in wave order: a fixed, placement-independent
// reduction order (bitwise reproducible run to run).
constexpr int BR_TW = 64;
constexpr int BR_NW = 16;

struct BreadthArgs {
  const double* c;
  const double* f[BQ_NUM_FEATURES];
  int64_t S, ld_c, ld_f;
  int T;
  double* partial;
};

__global__ __launch_bounds__(BR_TW * BR_NW) void breadth_kernel(const BreadthArgs A) {
  __shared__ double sAcc[BR_NW][BQ_NUM_PARTIALS][BR_TW + 1];
  const int lane = threadIdx.x & (WAVE - 1), u = threadIdx.x / WAVE;
  const int t = blockIdx.x * BR_TW + lane;
  double acc[BQ_NUM_PARTIALS];
#pragma unroll
  for (int i = 0; i < BQ_NUM_PARTIALS; ++i) acc[i] = 0.0;
  if (t < A.T) {
    for (int64_t s = u; s < A.S; s += BR_NW) {
      const double r = A.f[BQ_F_RETURN][s * A.ld_f + t];
      if (r != r) continue;   // no features at this t (history < 2 bars)
      const double cl = A.c[s * A.ld_c + t];
      acc[BQ_P_COUNT] += 1.0;
      acc[BQ_P_ADV] += r > 0.0 ? 1.0 : 0.0;
      acc[BQ_P_DEC] += r < 0.0 ? 1.0 : 0.0;
      acc[BQ_P_ABOVE20] += cl > A.f[BQ_F_EMA20][s * A.ld_f + t] ? 1.0 : 0.0;
      acc[BQ_P_ABOVE50] += cl > A.f[BQ_F_EMA50][s * A.ld_f + t] ? 1.0 : 0.0;
      acc[BQ_P_SUM_RET] += r;
      acc[BQ_P_SUM_TREND] += A.f[BQ_F_TREND][s * A.ld_f + t];
      acc[BQ_P_SUM_ATR_PCT] += A.f[BQ_F_ATR_PCT][s * A.ld_f + t];
      acc[BQ_P_SUM_BB_WIDTH] += A.f[BQ_F_BB_WIDTH][s * A.ld_f + t];
    }
  }
#pragma unroll
  for (int i = 0; i < BQ_NUM_PARTIALS; ++i) sAcc[u][i][lane] = acc[i];
  __syncthreads();
  if (u == 0 && t < A.T) {
    for (int v = 1; v < BR_NW; ++v)
#pragma unroll
      for (int i = 0; i < BQ_NUM_PARTIALS; ++i) acc[i] += sAcc[v][i][lane];
#pragma unroll
    for (int i = 0; i < BQ_NUM_PARTIALS; ++i) A.partial[(int64_t)t * BQ_NUM_PARTIALS + i] = acc[i];
  }
}

// Few timestamps (the live tick: T = 1). The kernel above gives one lane per
// timestamp, so at T = 1 each of its 16 waves walks S / 16 symbols with one
// active lane (≈0.5 ms at S = 10k). Here a workgroup of BS_NT threads owns one
// timestamp: thread k sums symbols k, k + BS_NT, ... in ascending order, then
// xor-butterflies over the wave and over the waves combine the threads. Again a
// fixed, placement-independent order: bitwise reproducible run to run.
constexpr int BS_NT = 1024;
constexpr int BS_MAX_T = 256;

__device__ __forceinline__ double wave_sum(double v, int width) {
#pragma unroll
  for (int d = WAVE / 2; d >= 1; d >>= 1)
    if (d < width) v += __shfl_xor(v, d, WAVE);
  return v;
}

__global__ __launch_bounds__(BS_NT) void breadth_small_kernel(const BreadthArgs A) {
  __shared__ double sRed[BQ_NUM_PARTIALS][BS_NT / WAVE];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t t = blockIdx.x;
  double acc[BQ_NUM_PARTIALS];
#pragma unroll
  for (int i = 0; i < BQ_NUM_PARTIALS; ++i) acc[i] = 0.0;
  for (int64_t s = tid; s < A.S; s += BS_NT) {
    const double r = A.f[BQ_F_RETURN][s * A.ld_f + t];
    if (r != r) continue;   // no features at this t (history < 2 bars)
    const double cl = A.c[s * A.ld_c + t];
    acc[BQ_P_COUNT] += 1.0;
    acc[BQ_P_ADV] += r > 0.0 ? 1.0 : 0.0;
    acc[BQ_P_DEC] += r < 0.0 ? 1.0 : 0.0;
    acc[BQ_P_ABOVE20] += cl > A.f[BQ_F_EMA20][s * A.ld_f + t] ? 1.0 : 0.0;
    acc[BQ_P_ABOVE50] += cl > A.f[BQ_F_EMA50][s * A.ld_f + t] ? 1.0 : 0.0;
    acc[BQ_P_SUM_RET] += r;
    acc[BQ_P_SUM_TREND] += A.f[BQ_F_TREND][s * A.ld_f + t];
    acc[BQ_P_SUM_ATR_PCT] += A.f[BQ_F_ATR_PCT][s * A.ld_f + t];
    acc[BQ_P_SUM_BB_WIDTH] += A.f[BQ_F_BB_WIDTH][s * A.ld_f + t];
  }
#pragma unroll
  for (int i = 0; i < BQ_NUM_PARTIALS; ++i) {
    const double v = wave_sum(acc[i], WAVE);
    if (lane == 0) sRed[i][w] = v;
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int i = 0; i < BQ_NUM_PARTIALS; ++i) {
      const double v = wave_sum(lane < BS_NT / WAVE ? sRed[i][lane] : 0.0, BS_NT / WAVE);
      if (lane == 0) A.partial[t * BQ_NUM_PARTIALS + i] = v;
    }
  }
}

static double alpha_from_span(double span) {
  const double com = (span - 1.0) / 2.0;
  return 1.0 / (1.0 + com);
}

// bq_context.hip: the features through the one-wave-per-symbol context kernel
int context_features(const double* const* hlc, int64_t S, int64_t T, int64_t ld_in, int32_t max_bars,
                     double* const* feat, int64_t ld_out, hipStream_t st);

// BQ_MARKET_FEATURES_IMPL=block / wave forces the workgroup-per-symbol
// features_kernel below / the context kernel's feature pass (default: by rows)
int market_features_impl() {   // 0 auto, 1 block, 2 wave
  static const int v = [] {
    const char* e = getenv("BQ_MARKET_FEATURES_IMPL");
    if (e && strcmp(e, "block") == 0) return 1;
    if (e && strcmp(e, "wave") == 0) return 2;
    return 0;
  }();
  return v;
}

}  // namespace bq

extern "C" {

int bq_market_features(const double* const* hlc, int64_t S, int64_t T, int64_t ld_in, int32_t max_bars,
                       double* const* feat, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!hlc || !feat || !hlc[0] || !hlc[1] || !hlc[2] || S < 0 || T < 0 || ld_in < T || ld_out < T ||
      max_bars < 15 || max_bars > BQ_MAX_HISTORY + 1 || T > (int64_t)0x7fffffff - MF_TT)
    return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  // one wave per row once the rows fill the chip (3 waves per SIMD x 1 024
  // SIMDs); fewer rows — the C5 step's one benchmark row — walk faster on a
  // workgroup each (1 x 10 000: 0.10 against 0.18 ms)
  const int impl = market_features_impl();
  if (impl != 1 && (impl == 2 || S >= 4096) && T <= (int64_t)0x7fffffff - 256 && S <= (int64_t)0x7fffffff)
    return context_features(hlc, S, T, ld_in, max_bars, feat, ld_out, (hipStream_t)stream);
  FeatArgs A;
  memset(&A, 0, sizeof(A));
  A.h = hlc[0];
  A.l = hlc[1];
  A.c = hlc[2];
  bool any = false;
  for (int i = 0; i < BQ_NUM_FEATURES; ++i) {
    A.out[i] = feat[i];
    any |= feat[i] != nullptr;
  }
  if (!any) return BQ_OK;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.M = max_bars;
  const double spans[2] = {20.0, 50.0};   // live_market_context_accumulator.py:266-267
  for (int e = 0; e < 2; ++e) {
    const double al = alpha_from_span(spans[e]);
    A.alpha[e] = al;
    A.om[e] = 1.0 - al;
    A.den[e] = A.om[e] + al;
    A.lin_a[e] = A.om[e] / A.den[e];
    A.lin_b[e] = al / A.den[e];
    double ak = 1.0;
    for (int k = 0; k < MF_K; ++k) ak *= A.lin_a[e];
    for (int j = 0; j < 8; ++j) {
      A.apow[e][j] = ak;
      ak *= ak;
    }
    double cp = 1.0;
    for (int k = 0; k < max_bars - 1; ++k) cp *= A.lin_a[e];
    A.corr[e] = cp;
  }
  auto aligned = [](const void* p) { return (((uintptr_t)p) & 15u) == 0; };
  int vin = (ld_in % 2) == 0 && aligned(A.h) && aligned(A.l) && aligned(A.c);
  int vout = (ld_out % 2) == 0;
  for (int i = 0; i < BQ_NUM_FEATURES; ++i)
    if (feat[i]) vout &= aligned(feat[i]);
  if (A.den[0] != 1.0 || A.den[1] != 1.0)
    hipLaunchKernelGGL(features_kernel<true>, dim3((unsigned)S), dim3(MF_NT), 0, (hipStream_t)stream, A, vin, vout);
  else
    hipLaunchKernelGGL(features_kernel<false>, dim3((unsigned)S), dim3(MF_NT), 0, (hipStream_t)stream, A, vin, vout);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_breadth_partial(const double* close, const double* const* feat, int64_t S, int64_t T,
                       int64_t ld_close, int64_t ld_feat, double* partial, void* stream) {
  using namespace bq;
  if (!close || !feat || !partial || S < 0 || T < 0 || ld_close < T || ld_feat < T || T > 0x7fffffff)
    return BQ_EINVAL;
  for (int i = 0; i < BQ_NUM_FEATURES; ++i)
    if (!feat[i]) return BQ_EINVAL;
  if (T == 0) return BQ_OK;
  BreadthArgs A;
  A.c = close;
  for (int i = 0; i < BQ_NUM_FEATURES; ++i) A.f[i] = feat[i];
  A.S = S;
  A.ld_c = ld_close;
  A.ld_f = ld_feat;
  A.T = (int)T;
  A.partial = partial;
  if (T <= BS_MAX_T) {
    hipLaunchKernelGGL(breadth_small_kernel, dim3((unsigned)T), dim3(BS_NT), 0, (hipStream_t)stream, A);
  } else {
    const unsigned blocks = (unsigned)((T + BR_TW - 1) / BR_TW);
    hipLaunchKernelGGL(breadth_kernel, dim3(blocks), dim3(BR_TW * BR_NW), 0, (hipStream_t)stream, A);
  }
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
