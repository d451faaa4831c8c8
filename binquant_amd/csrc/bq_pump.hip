// Fused pump-score features (gfx950): LiquidationSweepPump.compute_pump_score
// (strategies/liquidation_sweep_pump.py:195-269) on an [S][T] panel, every
// element-wise column and the short rolling windows in ONE pass over the row:
//
//   volume.shift(1).rolling(20).mean()          (:220-222, pandas' roll_mean
//                                                 rules: min_periods = window,
//                                                 same-value and sign rules)
//   high.shift(1).rolling(6).max(), low ... min (:223-226, :248)
//   close.pct_change(3) (pandas 2.3.3 fill_method='pad': the ffilled close)
//   relative_volume, pre_breakout_compression, pump_score, prior_high,
//   close_location, trend_score, momentum_atr, btc_momentum_3,
//   btc_trend_score, relative_strength     (:218-268)
//
// The benchmark's ffill / ewm rows come from bq_rolling_batch (panel mode)
// and are inputs here; the two rolling quantiles and score_cross follow
// (strategies.pump_score_features). The per-symbol ewm columns (candidate_atr
// = TR.ewm(alpha = 1/14, min_periods = 14), ema20, ema50) are either inputs
// (bq_pump_features) or formed in the pass (bq_pump_features_ewm): per tile,
// the lanes' affine maps y -> a y + b x over their 4 candles, a DPP wave scan
// on the lane-constant powers of a, the waves' totals through LDS, then each
// lane replays its 4 steps with pandas' update (as bq_panel.hip's ewm); a
// series with a missing or infinite value in a tile continues serially from
// there with pandas' own recursion (thread 0, from the ring; its results reach
// the lanes through the output column). No ewm column crosses HBM twice.
// Composed from separate stages the pipeline wrote and re-read every
// intermediate (TR aside: the volume mean, the highs / lows window, the
// ffilled close, momentum_3, pump_score ...): ~2.4x its algorithmic bytes.
//
// Mapping (as bq_enrich): one 256-thread workgroup per symbol walks its row in
// tiles of 1024 candles (4 per lane, 3 workgroups per CU); an LDS
// ring with a 32-candle halo holds high, low, close, volume, the ffilled
// close and the volume's run starts (the same-value rule), so every window
// reads the ring and every input byte crosses HBM once. Outputs leave through
// whole-line stores (store_lines). The element-wise arithmetic is the
// reference's operation order (the JIT stages' IEEE operations), so those
// columns equal the staged pipeline given the same window values; the volume
// mean's sliding sum agrees with pandas' Kahan roll_mean to rounding.
#include "bq_device.h"
#include "binquant_amd.h"

#include <stdint.h>
#include <string.h>

namespace bq {

constexpr int PF_NT = 256;
constexpr int PF_NW = PF_NT / WAVE;
constexpr int PF_K = 4;
constexpr int PF_TT = PF_NT * PF_K;   // 1024
constexpr int PF_H = 32;              // halo >= the longest lookback (volume window + shift)
constexpr int PF_R = PF_H + PF_TT;
constexpr int PF_Q = PF_R / PF_K;
constexpr int PF_MAXW = PF_H - 1;
// lane-interleaved ring (conflict-free: the lanes' k-th candles side by side)
__device__ __forceinline__ int pf_slot(int p) { return (p & (PF_K - 1)) * PF_Q + (p >> 2); }

enum { PF_H_IN = 0, PF_L_IN, PF_C_IN, PF_V_IN, PF_ATR_IN, PF_E20_IN, PF_E50_IN, PF_NIN };

// one ewm series of the fused variant: pandas' alpha / old-weight factor /
// divisor, the affine map y -> la y + lb x, apow[j] = la^(4 * 2^j) (the wave
// scan's lane powers), mw = la^(4 * 64) (one wave's span)
struct PumpEwm {
  double alpha, om, den, la, lb, mw;
  double apow[8];
  int minp, div;
};

struct PumpArgs {
  const double* in[PF_NIN];            // high, low, close, volume, candidate_atr, ema20, ema50 [S][ld_in]
  const double *bf, *be20, *be50;      // benchmark rows [T]: ffilled close, ewm 20, ewm 50
  double* out[BQ_NUM_PUMP_COLS];       // NULL: skip
  int64_t S, ld_in, ld_out;
  int T, mom, vol_w, comp_w;
  PumpEwm ew[3];                       // EWM_IN: TR (atr), close span 20, close span 50
};

typedef double pf_dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void pf_load(const double* __restrict__ row, int tb, int T, bool vec, double (&x)[PF_K]) {
  if (vec && tb + PF_K <= T) {
    const pf_dbl2* p = reinterpret_cast<const pf_dbl2*>(row + tb);
    const pf_dbl2 a = p[0], b = p[1];
    x[0] = a.x;
    x[1] = a.y;
    x[2] = b.x;
    x[3] = b.y;
  } else {
#pragma unroll
    for (int k = 0; k < PF_K; ++k) x[k] = tb + k < T ? row[tb + k] : qnan();
  }
}

// Series.clip(lower=0) / .replace(0, nan) as the staged programs evaluate them
__device__ __forceinline__ double clip0(double x) { return x < 0.0 ? 0.0 : x; }
__device__ __forceinline__ double rep0(double x) { return x == 0.0 ? qnan() : x; }

// 3 workgroups per CU for the default pass (168 VGPRs, 8 B of spill): its
// inputs are loaded at the tile start instead of a tile ahead (the prefetch's
// 32 registers cost a workgroup per CU) — a18 1.91-2.01 -> 1.86-1.87 ms (A/B).
// MC / VWC / CWC > 0: the momentum lag, volume lookback and compression
// window as compile-time constants (PumpParams' defaults 3 / 20 / 6): the
// window walks unroll, their ring slots become immediate offsets
template <bool EWM_IN, int MC = 0, int VWC = 0, int CWC = 0>
__global__ __launch_bounds__(PF_NT, EWM_IN ? 2 : 3) void pump_features_kernel(const PumpArgs A, int vin, int vout) {
  __shared__ double sH[PF_R], sL[PF_R], sC[PF_R], sV[PF_R], sF[PF_R];
  __shared__ double sEB[EWM_IN ? 3 : 1][PF_NW];   // the waves' scan totals
  __shared__ double sEC[EWM_IN ? 3 : 1];          // the ewm values at the previous tile's last candle
  __shared__ int sBad;                            // series (bits) with a non-finite value in this tile
  __shared__ int sRV[PF_R];   // volume run start (last index where the value changed; NaN counts)
  __shared__ int sWv[PF_NW], sWc[PF_NW];
  __shared__ int sCv, sCc;    // carries: volume run start, last valid close index
  __shared__ double sFV;      // ffilled close at the end of the previous tile
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t sym = blockIdx.x;
  const int T = A.T, M = MC > 0 ? MC : A.mom, VW = VWC > 0 ? VWC : A.vol_w, CW = CWC > 0 ? CWC : A.comp_w;
  const int64_t irow = sym * A.ld_in, orow = sym * A.ld_out;
  if (tid < PF_H) {   // before the row: missing values
    sH[pf_slot(tid)] = sL[pf_slot(tid)] = sC[pf_slot(tid)] = sV[pf_slot(tid)] = sF[pf_slot(tid)] = qnan();
    sRV[pf_slot(tid)] = -1;
  }
  if (tid == 0) {
    sCv = -1;
    sCc = -1;
    sFV = qnan();
    sBad = 0;
    if (EWM_IN)
      for (int e = 0; e < 3; ++e) sEC[e] = 0.0;
  }
  // the ewm scans' lane-constant powers, and the serial state (thread 0) of a
  // series once it has met a missing / infinite value
  double lpow[3], rpow[3];
  bool serial[3] = {false, false, false};
  double swv[3], sowt[3];
  int snobs[3];
  if (EWM_IN) {
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      lpow[e] = pow_bits<6>(A.ew[e].apow, lane);
      rpow[e] = pow_bits<5>(A.ew[e].apow, (lane & 15) + 1);
      swv[e] = qnan();
      sowt[e] = 1.0;
      snobs[e] = 0;
    }
  }
  // high, low, close, volume and the ewm columns: loaded at the start of
  // their own tile (no prefetch: see the launch bounds)
  constexpr int NP = PF_V_IN + 1;

  for (int t0 = 0; t0 < T; t0 += PF_TT) {
    const int tb = t0 + PF_K * tid, pb = PF_H + PF_K * tid;
    double x[NP][PF_K], atr[PF_K], e20[PF_K], e50[PF_K], ewy[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int f = 0; f < NP; ++f) pf_load(A.in[f] + irow, tb, T, vin, x[f]);
    if (!EWM_IN) {
      pf_load(A.in[PF_ATR_IN] + irow, tb, T, vin, atr);
      if (A.in[PF_E20_IN]) {   // NULL: trend_score came with the ewm columns (bq_pump_ewm)
        pf_load(A.in[PF_E20_IN] + irow, tb, T, vin, e20);
        pf_load(A.in[PF_E50_IN] + irow, tb, T, vin, e50);
      } else {
#pragma unroll
        for (int k = 0; k < PF_K; ++k) e20[k] = e50[k] = qnan();
      }
    }
    const double pv0 = tb >= 1 && tb <= T ? A.in[PF_V_IN][irow + tb - 1] : qnan();
    // ---- phase A: ring, run starts of the volume, last valid close (and the
    // ewm series' lane maps / wave scans)
    int lrv[PF_K], lvc[PF_K];
    double ewx[3], ewv[3][PF_K];
    {
      double pv = pv0;
      int run = -1, val = -1;
#pragma unroll
      for (int k = 0; k < PF_K; ++k) {
        const int t = tb + k;
        const double v = x[PF_V_IN][k];
        if (t == 0 || !(v == pv)) run = t;
        lrv[k] = run;
        pv = v;
        const double c = x[PF_C_IN][k];
        if (c == c && t < T) val = t;
        lvc[k] = val;
        sH[pf_slot(pb + k)] = x[PF_H_IN][k];
        sL[pf_slot(pb + k)] = x[PF_L_IN][k];
        sC[pf_slot(pb + k)] = c;
        sV[pf_slot(pb + k)] = v;
      }
      const int iv = wave_scan_max_dpp(lrv[PF_K - 1] + 1, lane);   // +1: DPP's zero fill is the identity
      const int ic = wave_scan_max_dpp(lvc[PF_K - 1] + 1, lane);
      if (lane == WAVE - 1) {
        sWv[w] = iv - 1;
        sWc[w] = ic - 1;
      }
      const int ev = dpp_i32<DPP_WAVE_SHR1>(iv) - 1, ec = dpp_i32<DPP_WAVE_SHR1>(ic) - 1;
      __syncthreads();   // A: ring, wave totals
      if (EWM_IN) {
        // the series' values: the true range (previous close from the ring)
        // and the close; lane maps from the zero state (candle 0 resets)
        double sv[3][PF_K];
        {
          double pc = sC[pf_slot(pb - 1)];
#pragma unroll
          for (int k = 0; k < PF_K; ++k) {
            const double c = x[PF_C_IN][k];
            sv[0][k] = tb + k < T ? win_val(true_range(x[PF_H_IN][k], x[PF_L_IN][k], pc)) : qnan();
            sv[1][k] = sv[2][k] = win_val(c);   // ewm: +-inf is missing
            pc = c;
          }
        }
        int bad = 0;
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          double y = 0.0;
#pragma unroll
          for (int k = 0; k < PF_K; ++k) {
            const double v = sv[e][k];
            bad |= (tb + k < T && !(v - v == 0.0)) ? (1 << e) : 0;
            y = tb + k == 0 ? v : fma(A.ew[e].la, y, A.ew[e].lb * v);
          }
          const double inc = wave_scan_affine_dpp_rp(y, A.ew[e].apow, rpow[e], lane);
          if (lane == WAVE - 1) sEB[e][w] = inc;
          ewx[e] = dpp_f64<DPP_WAVE_SHR1>(inc);   // exclusive (lane 0: the carry alone)
#pragma unroll
          for (int k = 0; k < PF_K; ++k) ewv[e][k] = sv[e][k];
        }
        if (bad) atomicOr(&sBad, bad);
      }
      int cv = max(sCv, ev), cc = max(sCc, ec);
      for (int u = 0; u < w; ++u) {
        cv = max(cv, sWv[u]);
        cc = max(cc, sWc[u]);
      }
#pragma unroll
      for (int k = 0; k < PF_K; ++k) {
        lrv[k] = max(lrv[k], cv);
        lvc[k] = max(lvc[k], cc);
        sRV[pf_slot(pb + k)] = lrv[k];
        // ffill: the last valid close at or before t (in the ring, or carried)
        const int i = lvc[k];
        sF[pf_slot(pb + k)] = i < 0 ? qnan() : (i >= t0 - PF_H ? sC[pf_slot(i - t0 + PF_H)] : sFV);
      }
    }
    __syncthreads();   // B: ffilled close and run starts visible (and the ewm wave totals)
    if (EWM_IN) {
      const int bad = sBad;
      double* eo[3] = {A.out[BQ_PUMP_CANDIDATE_ATR], A.out[BQ_PUMP_EMA20], A.out[BQ_PUMP_EMA50]};
      double* res[3] = {atr, e20, e50};
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const PumpEwm& P = A.ew[e];
        if (((bad >> e) & 1) && !serial[e]) {   // wave-uniform (from LDS): this series turns serial here
          serial[e] = true;
          if (t0 > 0) {   // candles 0 .. t0 - 1 were all observations
            swv[e] = sEC[e];
            snobs[e] = t0;
            sowt[e] = 1.0;
          }
        }
        if (serial[e]) {
          // pandas' recursion over the tile (thread 0, values from the ring),
          // results through the output column
          if (tid == 0) {
            const int n = min(PF_TT, T - t0);
            double wv = swv[e], owt = sowt[e];
            int nobs = snobs[e];
            for (int i = 0; i < n; ++i) {
              const int p = PF_H + i;
              const double c = sC[pf_slot(p)];
              const double cur = win_val(
                  e == 0 ? true_range(sH[pf_slot(p)], sL[pf_slot(p)], t0 + i > 0 ? sC[pf_slot(p - 1)] : qnan()) : c);
              const bool obs = cur == cur;
              if (t0 + i == 0) {
                wv = cur;
                nobs = obs ? 1 : 0;
              } else {
                nobs += obs ? 1 : 0;
                if (wv == wv) {
                  owt *= P.om;
                  if (obs) {
                    if (wv != cur) {
                      wv = owt * wv + P.alpha * cur;
                      wv /= owt + P.alpha;
                    }
                    owt = 1.0;
                  }
                } else if (obs) {
                  wv = cur;
                }
              }
              __hip_atomic_store(reinterpret_cast<unsigned long long*>(eo[e] + orow + t0 + i),
                                 (unsigned long long)__double_as_longlong(nobs >= P.minp ? wv : qnan()),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            swv[e] = wv;
            sowt[e] = owt;
            snobs[e] = nobs;
          }
          __threadfence();
          __syncthreads();
#pragma unroll
          for (int k = 0; k < PF_K; ++k)
            res[e][k] = tb + k < T ? __longlong_as_double((long long)__hip_atomic_load(
                                         reinterpret_cast<unsigned long long*>(eo[e] + orow + tb + k), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT))
                                   : qnan();
        } else {
          // the value at candle tb - 1: the carry through the earlier waves'
          // totals, then this lane's exclusive prefix
          double y = sEC[e];
          for (int u = 0; u < w; ++u) y = fma(P.mw, y, sEB[e][u]);
          y = lane == 0 ? y : fma(lpow[e], y, ewx[e]);
#pragma unroll
          for (int k = 0; k < PF_K; ++k) {   // pandas' update, step by step
            const int t = tb + k;
            const double v = ewv[e][k];
            if (t == 0) y = v;
            else if (y != v) {
              y = P.om * y + P.alpha * v;
              if (P.div) y = y / P.den;
            }
            res[e][k] = t + 1 >= P.minp ? y : qnan();
          }
          ewy[e] = y;
        }
      }
    }

    // ---- phase C: the lane's 4 candles; each column stored as soon as formed
    const bool whole = t0 + PF_TT <= T, vo = vout != 0;
    auto put = [&](int col, const double (&r)[PF_K]) {
      if (A.out[col]) store_lines<PF_K>(A.out[col] + orow, tb, T, vo, r, whole);
    };
    double m3[PF_K], rv[PF_K], comp[PF_K], hmax[PF_K], bm3[PF_K], r[PF_K];
    {
      // volume.shift(1).rolling(VW).mean(): window = ring [p - VW, p - 1]
      double s = 0.0;
      int nobs = 0, neg = 0;
      for (int j = -VW; j <= -1; ++j) {
        const double v = sV[pf_slot(pb + j)];
        const bool ok = win_ok(v);   // NaN and +-inf are missing (window op)
        s += ok ? v : 0.0;
        nobs += ok;
        neg += ok && signbit(v);
      }
      double pc = sC[pf_slot(pb - 1)];
#pragma unroll
      for (int k = 0; k < PF_K; ++k) {
        const int t = tb + k, p = pb + k;
        if (k > 0) {
          const double vi = sV[pf_slot(p - 1)], vo_ = sV[pf_slot(p - 1 - VW)];
          const bool oi = win_ok(vi), oo = win_ok(vo_);
          s = (s + (oi ? vi : 0.0)) - (oo ? vo_ : 0.0);
          nobs += (int)oi - (int)oo;
          neg += (int)(oi && signbit(vi)) - (int)(oo && signbit(vo_));
        }
        double vmean;
        if (nobs < VW || nobs <= 0) vmean = qnan();   // min_periods = window
        else {
          const double last = sV[pf_slot(p - 1)];
          const bool same = sRV[pf_slot(p - 1)] <= t - VW;   // every value equal to the last
          vmean = s / (double)nobs;
          if (same) vmean = last;
          else if (neg == 0 && vmean < 0.0) vmean = 0.0;
          else if (neg == nobs && vmean > 0.0) vmean = 0.0;
        }
        // high.shift(1).rolling(CW).max(), low ... .min() (min_periods = window:
        // a window with a missing value is NaN whatever else it holds, so the
        // extremes take every value unmasked — v_max / v_min skip a NaN — and
        // the observed counts decide; NaN and +-inf are missing, window op)
        double hm = -__builtin_inf(), lm = __builtin_inf();
        int nh = 0, nl = 0;
        for (int j = -CW; j <= -1; ++j) {
          const double hv = sH[pf_slot(p + j)], lv = sL[pf_slot(p + j)];
          nh += win_ok(hv);
          nl += win_ok(lv);
          hm = fmax(hm, hv);
          lm = fmin(lm, lv);
        }
        hmax[k] = nh >= CW ? hm : qnan();
        const double lmin = nl >= CW ? lm : qnan();
        const double prev = pc;   // close.shift(1)
        pc = x[PF_C_IN][k];
        const double cf = sF[pf_slot(p)], cf3 = t >= M ? sF[pf_slot(p - M)] : qnan();
        m3[k] = cf / cf3 - 1.0;
        rv[k] = x[PF_V_IN][k] / vmean;
        comp[k] = (hmax[k] - lmin) / prev;
        const bool tin = t < T;
        const double bf = tin ? A.bf[t] : qnan(), bf3 = tin && t >= M ? A.bf[t - M] : qnan();
        bm3[k] = bf / bf3 - 1.0;
      }
    }
    put(BQ_PUMP_CANDIDATE_ATR, atr);
    put(BQ_PUMP_MOMENTUM_3, m3);
    put(BQ_PUMP_RELATIVE_VOLUME, rv);
    put(BQ_PUMP_COMPRESSION, comp);
#pragma unroll
    for (int k = 0; k < PF_K; ++k) r[k] = rv[k] * clip0(m3[k]) / rep0(comp[k]);
    put(BQ_PUMP_SCORE, r);
    put(BQ_PUMP_PRIOR_HIGH, hmax);
#pragma unroll
    for (int k = 0; k < PF_K; ++k) r[k] = (x[PF_C_IN][k] - x[PF_L_IN][k]) / rep0(x[PF_H_IN][k] - x[PF_L_IN][k]);
    put(BQ_PUMP_CLOSE_LOCATION, r);
    put(BQ_PUMP_EMA20, e20);
    put(BQ_PUMP_EMA50, e50);
#pragma unroll
    for (int k = 0; k < PF_K; ++k) r[k] = (e20[k] - e50[k]) / e50[k];
    put(BQ_PUMP_TREND_SCORE, r);
#pragma unroll
    for (int k = 0; k < PF_K; ++k) r[k] = m3[k] / (atr[k] / x[PF_C_IN][k]);
    put(BQ_PUMP_MOMENTUM_ATR, r);
    put(BQ_PUMP_BTC_MOMENTUM_3, bm3);
#pragma unroll
    for (int k = 0; k < PF_K; ++k) {
      const int t = tb + k;
      const double b20 = t < T ? A.be20[t] : qnan(), b50 = t < T ? A.be50[t] : qnan();
      r[k] = (b20 - b50) / b50;
    }
    put(BQ_PUMP_BTC_TREND_SCORE, r);
#pragma unroll
    for (int k = 0; k < PF_K; ++k) r[k] = m3[k] - bm3[k];
    put(BQ_PUMP_RELATIVE_STRENGTH, r);

    if (t0 + PF_TT >= T) break;
    __syncthreads();   // every read of this tile's ring is done
    if (pb >= PF_TT) {   // halo of the next tile: the last PF_H positions
#pragma unroll
      for (int k = 0; k < PF_K; ++k) {
        const int a = pf_slot(pb + k), d = pf_slot(pb + k - PF_TT);
        sH[d] = sH[a];
        sL[d] = sL[a];
        sC[d] = sC[a];
        sV[d] = sV[a];
        sF[d] = sF[a];
        sRV[d] = sRV[a];
      }
    }
    if (tid == PF_NT - 1) {
      sCv = lrv[PF_K - 1];
      sCc = lvc[PF_K - 1];
      sFV = sF[pf_slot(pb + PF_K - 1)];
      if (EWM_IN)
#pragma unroll
        for (int e = 0; e < 3; ++e) sEC[e] = ewy[e];   // (serial series: unused)
    }
    if (EWM_IN && tid == 0) sBad = 0;
    __syncthreads();
  }
}

}  // namespace bq

extern "C" int bq_pump_features(const double* const* in, int64_t S, int64_t T, int64_t ld_in, const double* const* bench,
                                int32_t momentum_bars, int32_t volume_lookback, int32_t compression_bars,
                                double* const* out, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!in || !bench || !out || S < 0 || T < 0 || ld_in < T || ld_out < T || T > 0x7fffffff - 2 * PF_TT ||
      S > 0x7fffffff)
    return BQ_EINVAL;
  if (momentum_bars < 1 || momentum_bars > PF_MAXW || volume_lookback < 1 || compression_bars < 1 ||
      volume_lookback + 1 > PF_H || compression_bars + 1 > PF_H)
    return BQ_EINVAL;
  PumpArgs A;
  memset(&A, 0, sizeof(A));
  for (int f = 0; f < PF_NIN; ++f) {
    // ema20 / ema50 may both be NULL when no column reads them
    const bool opt = (f == PF_E20_IN || f == PF_E50_IN) && !out[BQ_PUMP_EMA20] && !out[BQ_PUMP_EMA50] &&
                     !out[BQ_PUMP_TREND_SCORE] && !in[PF_E20_IN] && !in[PF_E50_IN];
    if (!in[f] && !opt) return BQ_EINVAL;
    A.in[f] = in[f];
  }
  for (int i = 0; i < 3; ++i)
    if (!bench[i]) return BQ_EINVAL;
  A.bf = bench[0];
  A.be20 = bench[1];
  A.be50 = bench[2];
  bool any = false;
  for (int c = 0; c < BQ_NUM_PUMP_COLS; ++c) {
    A.out[c] = out[c];
    any |= out[c] != nullptr;
  }
  if (S == 0 || T == 0 || !any) return BQ_OK;
  A.S = S;
  A.T = (int)T;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.mom = momentum_bars;
  A.vol_w = volume_lookback;
  A.comp_w = compression_bars;
  auto aligned = [](const void* p) { return (((uintptr_t)p) & 15u) == 0; };
  int vin = (ld_in % 2) == 0, vout = (ld_out % 2) == 0;
  for (int f = 0; f < PF_NIN; ++f)
    if (in[f]) vin &= aligned(in[f]);
  for (int c = 0; c < BQ_NUM_PUMP_COLS; ++c)
    if (out[c]) vout &= aligned(out[c]);
  if (momentum_bars == 3 && volume_lookback == 20 && compression_bars == 6)   // PumpParams' defaults
    hipLaunchKernelGGL((pump_features_kernel<false, 3, 20, 6>), dim3((unsigned)S), dim3(PF_NT), 0, (hipStream_t)stream, A,
                       vin, vout);
  else
    hipLaunchKernelGGL(pump_features_kernel<false>, dim3((unsigned)S), dim3(PF_NT), 0, (hipStream_t)stream, A, vin,
                       vout);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

namespace {
// pandas: alpha = 1 / (1 + com); com = 1 / alpha - 1 (alpha given) or (span - 1) / 2
void pump_ewm_consts(bq::PumpEwm& E, double com, int minp) {
  E.alpha = 1.0 / (1.0 + com);
  E.om = 1.0 - E.alpha;
  E.den = E.om + E.alpha;
  E.div = E.den != 1.0;
  E.la = E.om / E.den;
  E.lb = E.alpha / E.den;
  double a4 = E.la * E.la;
  a4 *= a4;   // la^4
  E.apow[0] = a4;
  for (int j = 1; j < 8; ++j) E.apow[j] = E.apow[j - 1] * E.apow[j - 1];
  E.mw = E.apow[6];   // la^(4 * 64)
  E.minp = minp;
}
}  // namespace

extern "C" int bq_pump_features_ewm(const double* const* in, int64_t S, int64_t T, int64_t ld_in,
                                    const double* const* bench, int32_t momentum_bars, int32_t volume_lookback,
                                    int32_t compression_bars, double* const* out, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!in || !bench || !out || S < 0 || T < 0 || ld_in < T || ld_out < T || T > 0x7fffffff - 2 * PF_TT ||
      S > 0x7fffffff)
    return BQ_EINVAL;
  if (momentum_bars < 1 || momentum_bars > PF_MAXW || volume_lookback < 1 || compression_bars < 1 ||
      volume_lookback + 1 > PF_H || compression_bars + 1 > PF_H)
    return BQ_EINVAL;
  PumpArgs A;
  memset(&A, 0, sizeof(A));
  for (int f = 0; f <= PF_V_IN; ++f) {   // high, low, close, volume
    if (!in[f]) return BQ_EINVAL;
    A.in[f] = in[f];
  }
  for (int i = 0; i < 3; ++i)
    if (!bench[i]) return BQ_EINVAL;
  A.bf = bench[0];
  A.be20 = bench[1];
  A.be50 = bench[2];
  for (int c = 0; c < BQ_NUM_PUMP_COLS; ++c) A.out[c] = out[c];
  // the ewm columns are formed here and read back by the serial path
  if (!out[BQ_PUMP_CANDIDATE_ATR] || !out[BQ_PUMP_EMA20] || !out[BQ_PUMP_EMA50]) return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  A.S = S;
  A.T = (int)T;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.mom = momentum_bars;
  A.vol_w = volume_lookback;
  A.comp_w = compression_bars;
  pump_ewm_consts(A.ew[0], 1.0 / (1.0 / 14.0) - 1.0, 14);   // TR.ewm(alpha=1/14, min_periods=14) (:206-217)
  pump_ewm_consts(A.ew[1], (20.0 - 1.0) / 2.0, 0);          // close.ewm(span=20) (:252)
  pump_ewm_consts(A.ew[2], (50.0 - 1.0) / 2.0, 0);          // close.ewm(span=50) (:253)
  auto aligned = [](const void* p) { return (((uintptr_t)p) & 15u) == 0; };
  int vin = (ld_in % 2) == 0, vout = (ld_out % 2) == 0;
  for (int f = 0; f <= PF_V_IN; ++f) vin &= aligned(in[f]);
  for (int c = 0; c < BQ_NUM_PUMP_COLS; ++c)
    if (out[c]) vout &= aligned(out[c]);
  hipLaunchKernelGGL(pump_features_kernel<true>, dim3((unsigned)S), dim3(PF_NT), 0, (hipStream_t)stream, A, vin, vout);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
