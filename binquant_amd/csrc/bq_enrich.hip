// Fused full-indicator-set kernel for gfx950 (MI355X).
//
// Replaces the per-symbol pandas path of
//   producers/context_evaluator.py:240-263  (ContextEvaluator.indicators_enrichment)
// i.e. pybinbot.Indicators.moving_averages(7/25/100), macd, rsi,
// bollinguer_spreads, set_twap, atr(14) — plus Indicators.mfi(14)
// (strategies/coinrule/price_tracker.py:185) and the ema20/ema50 columns of
// market_regime/live_market_context_accumulator.py:266-267 — on a [S][T] panel.
//
// Mapping: one 256-thread workgroup (4 waves) owns one symbol and walks its
// candles in tiles of TT = 1024 (K = 4 consecutive candles per thread, so each
// lane's 32-byte slice is contiguous and a wave covers 2 KiB per field).
// Per tile:
//   * rolling windows = differences of a compensated (double-double) prefix
//     sum. The prefix is scanned across the wave with __shfl_up, across the 4
//     waves through LDS, rounded once to fp64 and kept in LDS for the tile plus
//     a 128-candle halo (re-based each tile so magnitudes stay tile-local);
//   * pandas' constant-window exactness (rolling().mean() returns the value
//     itself and std() returns 0 when every value in the window is identical)
//     is reproduced by a max-scan of "last index where the value changed";
//   * EMA / MACD recurrences are associative scans of the affine maps
//     y -> a*y + b (wave scan + LDS cross-wave + per-tile carry), after which
//     each lane replays its 4 steps with pandas' exact ewm(adjust=False)
//     update so per-element rounding matches pandas;
//   * Bollinger std is an exact two-pass variance over the window in LDS.
// Every input byte is read from HBM once and every output byte written once.
#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

constexpr int EN_NT = 256;
constexpr int EN_NW = EN_NT / WAVE;
constexpr int EN_K = 4;
constexpr int EN_TT = EN_NT * EN_K;
constexpr int EN_H = 128;
constexpr int EN_R = EN_H + EN_TT;

// prefix-summed quantities
enum { QC = 0, QG, QL, QTR, QO4, QPF, QNF, NQ };
constexpr int NLC = 5;   // constant-run tracking for QC..QO4
// EMA slots: 0 macd fast, 1 macd slow, 2 ema span0, 3 ema span1, 4 macd signal
constexpr int NE = 5;

struct EnrichArgs {
  const double* in[BQ_NUM_INPUTS];
  double* out[BQ_NUM_ENRICH_COLS];
  int64_t ld_in, ld_out;
  int T;
  int ma[3];
  int rsi_w, bb_w, bb_ddof, atr_w, twap_w, mfi_w;
  double bb_k;
  double alpha[NE], om[NE], den[NE];   // pandas ewm: new_wt, old_wt, old_wt+new_wt
  double lin_a[NE], lin_b[NE];         // linearised step y -> lin_a*y + lin_b*x
  double apow[NE][8];                  // (lin_a^K)^(2^j)
  int need_macd, need_sig;
};

__device__ __forceinline__ void load_k(const double* __restrict__ row, int tb, int T, bool vec,
                                       double (&x)[EN_K]) {
  if (vec && tb + EN_K <= T) {
    const double2* p = reinterpret_cast<const double2*>(row + tb);
    double2 a = p[0], b = p[1];
    x[0] = a.x; x[1] = a.y; x[2] = b.x; x[3] = b.y;
  } else {
#pragma unroll
    for (int k = 0; k < EN_K; ++k) x[k] = (tb + k < T) ? row[tb + k] : 0.0;
  }
}

typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void store_k(double* __restrict__ row, int tb, int T, bool vec,
                                        const double (&x)[EN_K]) {
  if (vec && tb + EN_K <= T) {
    dbl2* p = reinterpret_cast<dbl2*>(row + tb);
    dbl2 a = {x[0], x[1]}, b = {x[2], x[3]};
    __builtin_nontemporal_store(a, p);
    __builtin_nontemporal_store(b, p + 1);
  } else {
#pragma unroll
    for (int k = 0; k < EN_K; ++k)
      if (tb + k < T) row[tb + k] = x[k];
  }
}

__global__ __launch_bounds__(EN_NT) void enrich_kernel(const EnrichArgs A, int vec_in, int vec_out) {
  __shared__ double sP[NQ][EN_R];      // tile-local prefix sums (+ halo)
  __shared__ double sC[EN_R];          // raw close (+ halo) for the two-pass std
  __shared__ double sX[5][EN_NW + 1];  // neighbour exchange: c, c[-2], h, l, o of last candle
  __shared__ double sWh[NQ][EN_NW], sWl[NQ][EN_NW];
  __shared__ double sWe[NE][EN_NW];
  __shared__ int sWlc[NLC][EN_NW];
  __shared__ double sEcar[NE];
  __shared__ int sLcar[NLC];

  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t sym = blockIdx.x;
  const int T = A.T;
  const double* __restrict__ rO = A.in[BQ_OPEN] + sym * A.ld_in;
  const double* __restrict__ rH = A.in[BQ_HIGH] + sym * A.ld_in;
  const double* __restrict__ rL = A.in[BQ_LOW] + sym * A.ld_in;
  const double* __restrict__ rC = A.in[BQ_CLOSE] + sym * A.ld_in;
  const double* __restrict__ rV = A.in[BQ_VOLUME] + sym * A.ld_in;

  if (tid < NE) sEcar[tid] = 0.0;
  if (tid < NLC) sLcar[tid] = -1;
  if (tid < 5) sX[tid][0] = qnan();
  if (tid < EN_H) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) sP[q][tid] = 0.0;
    sC[tid] = qnan();
  }
  __syncthreads();

  const bool vin = vec_in != 0, vout = vec_out != 0;

  for (int t0 = 0; t0 < T; t0 += EN_TT) {
    const int tb = t0 + EN_K * tid;
    const int pb = EN_H + EN_K * tid;   // LDS position of element k=0
    double o[EN_K], h[EN_K], l[EN_K], c[EN_K], v[EN_K];
    load_k(rO, tb, T, vin, o);
    load_k(rH, tb, T, vin, h);
    load_k(rL, tb, T, vin, l);
    load_k(rC, tb, T, vin, c);
    load_k(rV, tb, T, vin, v);

    // ---- neighbour exchange (previous candle's raw values) -----------------
    double pc1 = __shfl_up(c[EN_K - 1], 1, WAVE);
    double pc2 = __shfl_up(c[EN_K - 2], 1, WAVE);
    double ph = __shfl_up(h[EN_K - 1], 1, WAVE);
    double pl = __shfl_up(l[EN_K - 1], 1, WAVE);
    double po = __shfl_up(o[EN_K - 1], 1, WAVE);
    if (lane == WAVE - 1) {
      sX[0][w + 1] = c[EN_K - 1];
      sX[1][w + 1] = c[EN_K - 2];
      sX[2][w + 1] = h[EN_K - 1];
      sX[3][w + 1] = l[EN_K - 1];
      sX[4][w + 1] = o[EN_K - 1];
    }
#pragma unroll
    for (int k = 0; k < EN_K; ++k) sC[pb + k] = c[k];
    __syncthreads();   // B1
    if (lane == 0) {
      pc1 = sX[0][w];
      pc2 = sX[1][w];
      ph = sX[2][w];
      pl = sX[3][w];
      po = sX[4][w];
    }

    // ---- derived per-candle quantities --------------------------------------
    double g[EN_K], ls[EN_K], tr[EN_K], o4[EN_K], pf[EN_K], nf[EN_K];
    int lcl[NLC][EN_K];
    {
      // values of candle t-1 (for change detection at k = 0)
      const double dm1 = pc1 - pc2;
      double prv[NLC] = {pc1, gain_of(dm1), loss_of(dm1), true_range(ph, pl, pc2),
                         ohlc4(po, ph, pl, pc1)};
      double cp = pc1, tpp = typical_price(ph, pl, pc1);
      int run[NLC] = {-1, -1, -1, -1, -1};
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        const int t = tb + k;
        const double d = c[k] - cp;
        g[k] = gain_of(d);
        ls[k] = loss_of(d);
        tr[k] = true_range(h[k], l[k], cp);
        o4[k] = ohlc4(o[k], h[k], l[k], c[k]);
        const double tp = typical_price(h[k], l[k], c[k]);
        const double mf = tp * v[k];
        pf[k] = tp > tpp ? mf : 0.0;
        nf[k] = tp < tpp ? mf : 0.0;
        const double cur[NLC] = {c[k], g[k], ls[k], tr[k], o4[k]};
#pragma unroll
        for (int q = 0; q < NLC; ++q) {
          if (t == 0 || cur[q] != prv[q]) run[q] = t;
          lcl[q][k] = run[q];
          prv[q] = cur[q];
        }
        cp = c[k];
        tpp = tp;
      }
    }

    // ---- phase A: per-thread totals, wave scans -----------------------------
    dd pre[NQ];   // exclusive wave prefix (dd)
    {
      const double* qv[NQ] = {c, g, ls, tr, o4, pf, nf};
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        dd tot = {0.0, 0.0};
#pragma unroll
        for (int k = 0; k < EN_K; ++k) tot = dd_add1(tot, qv[q][k]);
        dd inc = wave_incl_scan_dd(tot, lane);
        if (lane == WAVE - 1) {
          sWh[q][w] = inc.hi;
          sWl[q][w] = inc.lo;
        }
        double eh = __shfl_up(inc.hi, 1, WAVE), el = __shfl_up(inc.lo, 1, WAVE);
        pre[q] = lane == 0 ? dd{0.0, 0.0} : dd{eh, el};
      }
    }
    double epre[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < 2 && !A.need_macd) { epre[e] = 0.0; continue; }
      double y = 0.0;
#pragma unroll
      for (int k = 0; k < EN_K; ++k) y = (tb + k == 0) ? c[k] : fma(A.lin_a[e], y, A.lin_b[e] * c[k]);
      double inc = wave_incl_scan_affine(y, A.apow[e], lane);
      if (lane == WAVE - 1) sWe[e][w] = inc;
      double ex = __shfl_up(inc, 1, WAVE);
      epre[e] = lane == 0 ? 0.0 : ex;
    }
    int lpre[NLC];
#pragma unroll
    for (int q = 0; q < NLC; ++q) {
      int inc = wave_incl_scan_max(lcl[q][EN_K - 1], lane);
      if (lane == WAVE - 1) sWlc[q][w] = inc;
      int ex = __shfl_up(inc, 1, WAVE);
      lpre[q] = lane == 0 ? -1 : ex;
    }
    __syncthreads();   // B2

    // ---- phase B: carries, prefix to LDS, EMA replay -------------------------
    {
      const double* qv[NQ] = {c, g, ls, tr, o4, pf, nf};
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        dd base = {0.0, 0.0};   // halo prefix ends at 0 by construction (re-base)
        for (int u = 0; u < w; ++u) base = dd_add(base, dd{sWh[q][u], sWl[q][u]});
        base = dd_add(base, pre[q]);
#pragma unroll
        for (int k = 0; k < EN_K; ++k) {
          base = dd_add1(base, qv[q][k]);
          sP[q][pb + k] = dd_round(base);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NLC; ++q) {
      int carry = sLcar[q];
      for (int u = 0; u < w; ++u) carry = max(carry, sWlc[q][u]);
      carry = max(carry, lpre[q]);
#pragma unroll
      for (int k = 0; k < EN_K; ++k) lcl[q][k] = max(lcl[q][k], carry);
    }
    double ema[4][EN_K];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < 2 && !A.need_macd) {
#pragma unroll
        for (int k = 0; k < EN_K; ++k) ema[e][k] = 0.0;
        continue;
      }
      double C = sEcar[e];
      for (int u = 0; u < w; ++u) C = fma(A.apow[e][6], C, sWe[e][u]);
      double y = lane == 0 ? C : fma(pow_bits<6>(A.apow[e], lane), C, epre[e]);
      const double al = A.alpha[e], om = A.om[e], dn = A.den[e];
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        const double x = c[k];
        if (tb + k == 0) y = x;
        else if (y != x) y = (om * y + al * x) / dn;
        ema[e][k] = y;
      }
    }
    double macd[EN_K], sig[EN_K] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < EN_K; ++k) macd[k] = ema[0][k] - ema[1][k];
    double spre = 0.0;
    if (A.need_sig) {
      double y = 0.0;
#pragma unroll
      for (int k = 0; k < EN_K; ++k) y = (tb + k == 0) ? macd[k] : fma(A.lin_a[4], y, A.lin_b[4] * macd[k]);
      double inc = wave_incl_scan_affine(y, A.apow[4], lane);
      if (lane == WAVE - 1) sWe[4][w] = inc;
      double ex = __shfl_up(inc, 1, WAVE);
      spre = lane == 0 ? 0.0 : ex;
    }
    __syncthreads();   // B3: prefix sums + signal wave totals visible
    if (A.need_sig) {
      double C = sEcar[4];
      for (int u = 0; u < w; ++u) C = fma(A.apow[4][6], C, sWe[4][u]);
      double y = lane == 0 ? C : fma(pow_bits<6>(A.apow[4], lane), C, spre);
      const double al = A.alpha[4], om = A.om[4], dn = A.den[4];
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        const double x = macd[k];
        if (tb + k == 0) y = x;
        else if (y != x) y = (om * y + al * x) / dn;
        sig[k] = y;
      }
    }

    // ---- phase C: window outputs --------------------------------------------
    const double cur_q[NLC][EN_K] = {{c[0], c[1], c[2], c[3]},
                                     {g[0], g[1], g[2], g[3]},
                                     {ls[0], ls[1], ls[2], ls[3]},
                                     {tr[0], tr[1], tr[2], tr[3]},
                                     {o4[0], o4[1], o4[2], o4[3]}};
    auto wmean = [&](int q, int win, int k) -> double {
      const int t = tb + k, p = pb + k;
      if (t < win - 1) return qnan();
      if (lcl[q][k] <= t - win + 1) return cur_q[q][k];
      double S = sP[q][p] - sP[q][p - win];
      if (q != QC && q != QO4) S = S < 0.0 ? 0.0 : S;   // pandas neg_ct clamp
      return S / (double)win;
    };
    auto wsum = [&](int q, int win, int k) -> double {
      const int t = tb + k, p = pb + k;
      if (t < win - 1) return qnan();
      double S = sP[q][p] - sP[q][p - win];
      return S < 0.0 ? 0.0 : S;
    };
    const int64_t orow = sym * A.ld_out;
    double res[EN_K];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (A.out[BQ_MA_FAST + i]) {
#pragma unroll
        for (int k = 0; k < EN_K; ++k) res[k] = wmean(QC, A.ma[i], k);
        store_k(A.out[BQ_MA_FAST + i] + orow, tb, T, vout, res);
      }
    }
    if (A.out[BQ_MACD]) store_k(A.out[BQ_MACD] + orow, tb, T, vout, macd);
    if (A.out[BQ_MACD_SIGNAL]) store_k(A.out[BQ_MACD_SIGNAL] + orow, tb, T, vout, sig);
    if (A.out[BQ_RSI]) {
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        const double gm = wmean(QG, A.rsi_w, k), lm = wmean(QL, A.rsi_w, k);
        res[k] = oscillator(gm, lm);
      }
      store_k(A.out[BQ_RSI] + orow, tb, T, vout, res);
    }
    if (A.out[BQ_BB_UPPER] || A.out[BQ_BB_MID] || A.out[BQ_BB_LOWER]) {
      double mid[EN_K], up[EN_K], lo[EN_K];
      const int win = A.bb_w;
      const double dv = (double)(win - A.bb_ddof);
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        const int t = tb + k, p = pb + k;
        const double m = wmean(QC, win, k);
        double sd;
        if (t < win - 1 || dv <= 0.0) sd = qnan();
        else if (lcl[QC][k] <= t - win + 1) sd = 0.0;
        else {
          double acc = 0.0;
          for (int i = p - win + 1; i <= p; ++i) {
            const double dlt = sC[i] - m;
            acc = fma(dlt, dlt, acc);
          }
          sd = sqrt(acc / dv);
        }
        mid[k] = m;
        up[k] = m + A.bb_k * sd;
        lo[k] = m - A.bb_k * sd;
      }
      if (A.out[BQ_BB_UPPER]) store_k(A.out[BQ_BB_UPPER] + orow, tb, T, vout, up);
      if (A.out[BQ_BB_MID]) store_k(A.out[BQ_BB_MID] + orow, tb, T, vout, mid);
      if (A.out[BQ_BB_LOWER]) store_k(A.out[BQ_BB_LOWER] + orow, tb, T, vout, lo);
    }
    if (A.out[BQ_ATR]) {
#pragma unroll
      for (int k = 0; k < EN_K; ++k) res[k] = wmean(QTR, A.atr_w, k);
      store_k(A.out[BQ_ATR] + orow, tb, T, vout, res);
    }
    if (A.out[BQ_TWAP]) {
#pragma unroll
      for (int k = 0; k < EN_K; ++k) res[k] = wmean(QO4, A.twap_w, k);
      store_k(A.out[BQ_TWAP] + orow, tb, T, vout, res);
    }
    if (A.out[BQ_EMA_FAST]) store_k(A.out[BQ_EMA_FAST] + orow, tb, T, vout, ema[2]);
    if (A.out[BQ_EMA_SLOW]) store_k(A.out[BQ_EMA_SLOW] + orow, tb, T, vout, ema[3]);
    if (A.out[BQ_MFI]) {
#pragma unroll
      for (int k = 0; k < EN_K; ++k) res[k] = oscillator(wsum(QPF, A.mfi_w, k), wsum(QNF, A.mfi_w, k));
      store_k(A.out[BQ_MFI] + orow, tb, T, vout, res);
    }

    if (t0 + EN_TT >= T) break;   // no next tile: skip carry bookkeeping
    __syncthreads();   // B4: every read of this tile's LDS is done

    // ---- carries into the next tile -----------------------------------------
    if (tid < EN_H) {
      const int src = EN_TT + tid;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const double last = sP[q][EN_R - 1];
        sP[q][tid] = sP[q][src] - last;   // re-base: halo prefix ends at 0
      }
      sC[tid] = sC[src];
    }
    if (tid < 5) sX[tid][0] = sX[tid][EN_NW];
    if (tid == EN_NT - 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) sEcar[e] = ema[e][EN_K - 1];
      sEcar[4] = sig[EN_K - 1];
#pragma unroll
      for (int q = 0; q < NLC; ++q) sLcar[q] = lcl[q][EN_K - 1];
    }
    __syncthreads();   // B5
  }
}

// pandas.core.window.ewm: comass from span, alpha = 1 / (1 + comass)
static double ewm_alpha_from_span(double span) {
  const double com = (span - 1.0) / 2.0;
  return 1.0 / (1.0 + com);
}

static void set_ema(EnrichArgs& A, int e, double alpha) {
  const double om = 1.0 - alpha;   // old_wt = 1 * old_wt_factor
  A.alpha[e] = alpha;
  A.om[e] = om;
  A.den[e] = om + alpha;
  A.lin_a[e] = om / A.den[e];
  A.lin_b[e] = alpha / A.den[e];
  double ak = 1.0;
  for (int k = 0; k < EN_K; ++k) ak *= A.lin_a[e];
  for (int j = 0; j < 8; ++j) {
    A.apow[e][j] = ak;
    ak *= ak;
  }
}

static bool window_ok(int w) { return w >= 1 && w <= BQ_MAX_WINDOW; }

}  // namespace bq

extern "C" {

void bq_default_params(bq_params* p) {
  if (!p) return;
  memset(p, 0, sizeof(*p));
  p->ma_periods[0] = 7;
  p->ma_periods[1] = 25;
  p->ma_periods[2] = 100;
  p->macd_fast = 12;
  p->macd_slow = 26;
  p->macd_signal = 9;
  p->rsi_window = 14;
  p->bb_window = 20;
  p->bb_ddof = 1;
  p->atr_window = 14;
  p->twap_window = 12;
  p->ema_spans[0] = 20;
  p->ema_spans[1] = 50;
  p->mfi_window = 14;
  p->bb_k = 2.0;
}

const char* bq_version(void) { return "binquant_amd 0.1.0 (gfx950)"; }

int bq_device_arch(char* buf, int buflen) {
  if (!buf || buflen <= 0) return BQ_EINVAL;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return BQ_EHIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return BQ_EHIP;
  strncpy(buf, prop.gcnArchName, (size_t)buflen - 1);
  buf[buflen - 1] = 0;
  return BQ_OK;
}

int bq_enrich(const double* const* in, int64_t S, int64_t T, int64_t ld_in, const bq_params* params,
              double* const* out, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!in || !out || S < 0 || T < 0 || ld_in < T || ld_out < T || T > (int64_t)0x7fffffff - EN_TT)
    return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  bq_params dp;
  if (!params) {
    bq_default_params(&dp);
    params = &dp;
  }
  EnrichArgs A;
  memset(&A, 0, sizeof(A));
  bool any_out = false;
  for (int i = 0; i < BQ_NUM_INPUTS; ++i) {
    if (!in[i]) return BQ_EINVAL;
    A.in[i] = in[i];
  }
  for (int i = 0; i < BQ_NUM_ENRICH_COLS; ++i) {
    A.out[i] = out[i];
    any_out |= out[i] != nullptr;
  }
  if (!any_out) return BQ_OK;
  const bq_params& P = *params;
  for (int i = 0; i < 3; ++i)
    if (!window_ok(P.ma_periods[i])) return BQ_EINVAL;
  if (!window_ok(P.rsi_window) || !window_ok(P.bb_window) || !window_ok(P.atr_window) ||
      !window_ok(P.twap_window) || !window_ok(P.mfi_window) || P.bb_ddof < 0 ||
      P.macd_fast < 1 || P.macd_slow < 1 || P.macd_signal < 1 || P.ema_spans[0] < 1 ||
      P.ema_spans[1] < 1)
    return BQ_EINVAL;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  for (int i = 0; i < 3; ++i) A.ma[i] = P.ma_periods[i];
  A.rsi_w = P.rsi_window;
  A.bb_w = P.bb_window;
  A.bb_ddof = P.bb_ddof;
  A.atr_w = P.atr_window;
  A.twap_w = P.twap_window;
  A.mfi_w = P.mfi_window;
  A.bb_k = P.bb_k;
  set_ema(A, 0, ewm_alpha_from_span(P.macd_fast));
  set_ema(A, 1, ewm_alpha_from_span(P.macd_slow));
  set_ema(A, 2, ewm_alpha_from_span(P.ema_spans[0]));
  set_ema(A, 3, ewm_alpha_from_span(P.ema_spans[1]));
  set_ema(A, 4, ewm_alpha_from_span(P.macd_signal));
  A.need_sig = out[BQ_MACD_SIGNAL] != nullptr;
  A.need_macd = out[BQ_MACD] != nullptr || A.need_sig;

  // 16-byte vector access needs every row start 16-byte aligned.
  auto aligned = [](const void* p) { return (((uintptr_t)p) & 15u) == 0; };
  int vin = (ld_in % 2) == 0;
  for (int i = 0; i < BQ_NUM_INPUTS; ++i) vin &= aligned(in[i]);
  int vout = (ld_out % 2) == 0;
  for (int i = 0; i < BQ_NUM_ENRICH_COLS; ++i)
    if (out[i]) vout &= aligned(out[i]);

  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(enrich_kernel, dim3((unsigned)S), dim3(EN_NT), 0, st, A, vin, vout);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
