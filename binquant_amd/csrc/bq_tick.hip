// Streaming tick path for gfx950: one new candle per symbol per tick.
//
// The reference re-fetches the last KlinesProvider.LIMIT = 400 candles and
// re-enriches that frame on every closed-kline message
// (consumers/klines_provider.py:40,201-215 -> producers/context_evaluator.py:
// 347-371,416), so every EMA it reports is seeded at the FIRST candle of that
// 400-candle frame. Here each symbol keeps device-resident state instead:
//   * a ring of the last RING candles (o, h, l, c, v), slot-major [RING][S]
//     so that lane = symbol reads are coalesced; the rolling windows
//     (<= BQ_MAX_WINDOW) are re-summed from it each tick (compensated), which
//     keeps them drift-free; pandas' constant-window rules are applied;
//   * frame mode (F > 0, default 400): a close ring of the last F closes and
//     the index of the newest missing close. Each tick replays pandas'
//     ewm(adjust=False) recursion over the frame [t-F+1, t] — seeded at the
//     frame's first candle exactly as the reference's re-enrichment is — so
//     ema20 / ema50 / macd / macd_signal equal the reference's per-message
//     frame bit for bit. The replay is latency-bound (one dependent chain per
//     EMA), so the four chains run on their own waves of the workgroup;
//   * unbounded mode (F = 0): the five EMA carries and their old weights,
//     updated with pandas' exact step (the full-series pandas EMA).
// A NaN candle (a symbol without a candle this tick) follows pandas'
// ignore_na=False rules in both modes.
// One workgroup of 4 waves per 64 symbols; a 10k-symbol tick is one
// ~157-workgroup launch.
#include "bq_device.h"
#include "binquant_amd.h"

#include <stdlib.h>
#include <string.h>

namespace bq {

constexpr int RING = BQ_MAX_WINDOW + 2;   // 128
constexpr int TK_NT = 256;                // 4 waves
constexpr int TK_SYM = 64;                // symbols per workgroup (one per lane)
constexpr int64_t TK_MAX_FRAME = 1 << 20;

struct OutTable {
  double* p[BQ_NUM_ENRICH_COLS];
};

struct TickConsts {
  int ma[3];
  int rsi_w, bb_w, bb_ddof, atr_w, twap_w, mfi_w;
  double bb_k;
  double alpha[5], om[5];   // 0 macd fast, 1 macd slow, 2 ema0, 3 ema1, 4 signal
  int unit[5];              // om + alpha == 1.0 exactly: pandas' divide is the identity
};

}  // namespace bq

struct bq_state {
  int64_t S;
  int64_t count;
  int64_t F;          // frame length (0 = unbounded history)
  bq::TickConsts K;
  double* ring;       // [5][RING][S]
  double* ema;        // F == 0: [10][S]: 5 EMA values, then their 5 old weights
  double* cring;      // F  > 0: [F][S] closes, slot t % F
  int64_t* lastnan;   // F  > 0: [S] index of the newest missing close (-1: none)
};

namespace bq {

__device__ __forceinline__ double ring_at(const double* ring, int f, int64_t S, int64_t i, int64_t s) {
  return ring[((int64_t)f * RING + (i % RING)) * S + s];
}

// Kahan-compensated sum of a derived per-candle quantity over candles
// (t-w, t]; returns NaN if fewer than w candles exist. `all_same` reports
// whether every value in the window equals the newest (pandas same-value rule).
template <class F>
__device__ __forceinline__ double window_sum(F q, int64_t t, int w, bool& all_same) {
  double s = 0.0, comp = 0.0;
  const double last = q(t);
  all_same = true;
  for (int64_t i = t - w + 1; i <= t; ++i) {
    const double x = q(i);
    all_same &= (x == last);
    const double y = x - comp;
    const double z = s + y;
    comp = (z - s) - y;
    s = z;
  }
  return s;
}

// One step of pandas' ewm(adjust=False, ignore_na=False) mean
// (pandas/_libs/window/aggregations.pyx `ewm`; oracle/indicators_ref.py
// ewm_scalar): y = weighted, w = old_wt. pandas' window operations see +-inf
// as missing (_prep_values), hence win_val. With no NaN gap w == 1 before the
// decay and (om * y + al * x) / (om + al) is the plain update; when
// om + al == 1.0 exactly (`unit`, every integer span) the divide is the
// identity and is skipped — the same bits.
__device__ __forceinline__ void ewm_step(double& y, double& w, double x, double al, double om, bool unit,
                                         bool first) {
  x = win_val(x);
  if (first) {
    y = x;
    w = 1.0;
    return;
  }
  const bool obs = x == x;
  if (y == y) {
    w *= om;
    if (obs) {
      if (y != x) {
        const double num = w * y + al * x, den = w + al;
        y = (unit && den == 1.0) ? num : num / den;
      }
      w = 1.0;
    }
  } else if (obs) {
    y = x;
  }
}

// The no-gap step: old weight 1 decayed to om, om + al == 1.
__device__ __forceinline__ double ewm_step_dense(double y, double x, double al, double om) {
  return y != x ? om * y + al * x : y;
}

// Frame-mode EMA replay of one lane's symbol over closes [t0, t] (close ring
// of F slots, slot j % F; the newest close `xt` is passed in, not read).
// NE chains: NE == 3 -> macd fast, macd slow and the signal over their
// difference; NE == 1 -> the single EMA `e`. Dense (no missing close in the
// frame, unit weights) or the general pandas step.
template <int NE>
__device__ __forceinline__ void frame_replay(const TickConsts& K, int e, const double* __restrict__ cring,
                                             int64_t S, int64_t F, int64_t s, int64_t t0, int64_t t, double xt,
                                             bool dense, double* y) {
  constexpr int PF = 16;   // closes loaded ahead of the dependent chain
  const int ea = NE == 3 ? 0 : e;
  const double al0 = K.alpha[ea], om0 = K.om[ea];
  const double al1 = K.alpha[1], om1 = K.om[1];
  const double al4 = K.alpha[4], om4 = K.om[4];
  double w[3] = {1.0, 1.0, 1.0};
  int64_t slot = t0 % F;
  auto at = [&](int64_t j) {
    const double v = j == t ? xt : cring[slot * S + s];
    if (++slot == F) slot = 0;
    return v;
  };
  // first candle of the frame seeds every chain
  {
    const double x = at(t0);
    ewm_step(y[0], w[0], x, al0, om0, true, true);
    if (NE == 3) {
      ewm_step(y[1], w[1], x, al1, om1, true, true);
      ewm_step(y[2], w[2], y[0] - y[1], al4, om4, true, true);
    }
  }
  int64_t j = t0 + 1;
  if (dense) {
    for (; j + PF <= t + 1; j += PF) {
      double xs[PF];
#pragma unroll
      for (int k = 0; k < PF; ++k) xs[k] = at(j + k);
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        y[0] = ewm_step_dense(y[0], xs[k], al0, om0);
        if (NE == 3) {
          y[1] = ewm_step_dense(y[1], xs[k], al1, om1);
          y[2] = ewm_step_dense(y[2], y[0] - y[1], al4, om4);
        }
      }
    }
    for (; j <= t; ++j) {
      const double x = at(j);
      y[0] = ewm_step_dense(y[0], x, al0, om0);
      if (NE == 3) {
        y[1] = ewm_step_dense(y[1], x, al1, om1);
        y[2] = ewm_step_dense(y[2], y[0] - y[1], al4, om4);
      }
    }
  } else {
    const bool u0 = K.unit[ea], u1 = K.unit[1], u4 = K.unit[4];
    for (; j <= t; ++j) {
      const double x = at(j);
      ewm_step(y[0], w[0], x, al0, om0, u0, false);
      if (NE == 3) {
        ewm_step(y[1], w[1], x, al1, om1, u1, false);
        ewm_step(y[2], w[2], y[0] - y[1], al4, om4, u4, false);
      }
    }
  }
}

// Wave 0: ring append + every rolling-window column (+ the EMA carries in
// unbounded mode). Waves 1-3 (frame mode): the EMA replays — wave 1 macd fast
// + slow + signal, wave 2 ema_spans[0], wave 3 ema_spans[1].
__global__ __launch_bounds__(TK_NT) void tick_kernel(const TickConsts K, int64_t S, int64_t n, int64_t F,
                                                     double* ring, double* ema, double* cring, int64_t* lastnan,
                                                     const double* __restrict__ no, const double* __restrict__ nh,
                                                     const double* __restrict__ nl, const double* __restrict__ nc,
                                                     const double* __restrict__ nv, const OutTable outp,
                                                     unsigned outmask) {
  const int wave = threadIdx.x / WAVE;
  const int64_t s = (int64_t)blockIdx.x * TK_SYM + (threadIdx.x % WAVE);
  const int64_t t = n;   // index of the new candle
  const bool live = s < S;
  const double x = live ? nc[s] : 0.0;
  auto put = [&](int col, double v) {
    if (outmask & (1u << col)) outp.p[col][s] = v;
  };

  if (F > 0) {
    // every wave reads the newest-missing index before wave 0 advances it
    const int64_t ln_old = live ? lastnan[s] : 0;
    __syncthreads();
    if (!live) return;
    const bool miss = !win_ok(x);
    if (wave == 0) {
      cring[(t % F) * S + s] = x;
      if (miss) lastnan[s] = t;
    } else {
      const int64_t t0 = t - F + 1 > 0 ? t - F + 1 : 0;
      const bool dense = !miss && ln_old < t0 && K.unit[wave == 1 ? 0 : wave] &&
                         (wave != 1 || (K.unit[1] && K.unit[4]));
      if (wave == 1) {
        if (!(outmask & ((1u << BQ_MACD) | (1u << BQ_MACD_SIGNAL)))) return;
        double y[3];
        frame_replay<3>(K, 0, cring, S, F, s, t0, t, x, dense, y);
        put(BQ_MACD, y[0] - y[1]);
        put(BQ_MACD_SIGNAL, y[2]);
      } else {
        const int col = wave == 2 ? BQ_EMA_FAST : BQ_EMA_SLOW;
        if (!(outmask & (1u << col))) return;
        double y[3];
        frame_replay<1>(K, wave, cring, S, F, s, t0, t, x, dense, y);
        put(col, y[0]);
      }
      return;
    }
  } else {
    if (wave != 0 || !live) return;
  }

  // ---- wave 0 ----
  {
    const int64_t slot = t % RING;
    ring[((int64_t)0 * RING + slot) * S + s] = no[s];
    ring[((int64_t)1 * RING + slot) * S + s] = nh[s];
    ring[((int64_t)2 * RING + slot) * S + s] = nl[s];
    ring[((int64_t)3 * RING + slot) * S + s] = x;
    ring[((int64_t)4 * RING + slot) * S + s] = nv[s];
  }
  if (F == 0) {
    double y[5];
#pragma unroll
    for (int e = 0; e < 5; ++e) {
      double v = ema[(int64_t)e * S + s], wt = ema[(int64_t)(5 + e) * S + s];
      ewm_step(v, wt, e < 4 ? x : y[0] - y[1], K.alpha[e], K.om[e], K.unit[e], t == 0);
      y[e] = v;
      ema[(int64_t)e * S + s] = v;
      ema[(int64_t)(5 + e) * S + s] = wt;
    }
    put(BQ_MACD, y[0] - y[1]);
    put(BQ_MACD_SIGNAL, y[4]);
    put(BQ_EMA_FAST, y[2]);
    put(BQ_EMA_SLOW, y[3]);
  }

  auto O = [&](int64_t i) { return i < 0 ? qnan() : ring_at(ring, 0, S, i, s); };
  auto Hh = [&](int64_t i) { return i < 0 ? qnan() : ring_at(ring, 1, S, i, s); };
  auto Ll = [&](int64_t i) { return i < 0 ? qnan() : ring_at(ring, 2, S, i, s); };
  auto Cc = [&](int64_t i) { return i < 0 ? qnan() : ring_at(ring, 3, S, i, s); };
  auto Vv = [&](int64_t i) { return ring_at(ring, 4, S, i, s); };
  auto close_q = [&](int64_t i) { return Cc(i); };
  auto gain_q = [&](int64_t i) { return gain_of(Cc(i) - Cc(i - 1)); };
  auto loss_q = [&](int64_t i) { return loss_of(Cc(i) - Cc(i - 1)); };
  auto tr_q = [&](int64_t i) { return true_range(Hh(i), Ll(i), Cc(i - 1)); };
  auto o4_q = [&](int64_t i) { return ohlc4(O(i), Hh(i), Ll(i), Cc(i)); };
  auto tp_at = [&](int64_t i) { return typical_price(Hh(i), Ll(i), Cc(i)); };
  auto pf_q = [&](int64_t i) {
    const double tp = tp_at(i), tpp = tp_at(i - 1);
    return tp > tpp ? tp * Vv(i) : 0.0;
  };
  auto nf_q = [&](int64_t i) {
    const double tp = tp_at(i), tpp = tp_at(i - 1);
    return tp < tpp ? tp * Vv(i) : 0.0;
  };
  auto mean_of = [&](auto q, int w, bool nonneg) -> double {
    if (t < w - 1) return qnan();
    bool same;
    double S_ = window_sum(q, t, w, same);
    if (same) return q(t);
    if (nonneg && S_ < 0.0) S_ = 0.0;
    return S_ / (double)w;
  };

#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (outmask & (1u << (BQ_MA_FAST + i))) put(BQ_MA_FAST + i, mean_of(close_q, K.ma[i], false));
  if (outmask & (1u << BQ_RSI)) put(BQ_RSI, oscillator(mean_of(gain_q, K.rsi_w, true), mean_of(loss_q, K.rsi_w, true)));
  if (outmask & ((1u << BQ_BB_UPPER) | (1u << BQ_BB_MID) | (1u << BQ_BB_LOWER))) {
    const int w = K.bb_w;
    double mid = qnan(), sd = qnan();
    if (t >= w - 1) {
      bool same;
      const double sum = window_sum(close_q, t, w, same);
      if (same) {
        mid = x;
        sd = (w - K.bb_ddof) > 0 ? 0.0 : qnan();
      } else {
        mid = sum / (double)w;
        double acc = 0.0;
        for (int64_t i = t - w + 1; i <= t; ++i) {
          const double d = Cc(i) - mid;
          acc = fma(d, d, acc);
        }
        sd = (w - K.bb_ddof) > 0 ? sqrt(acc / (double)(w - K.bb_ddof)) : qnan();
      }
    }
    put(BQ_BB_MID, mid);
    put(BQ_BB_UPPER, mid + K.bb_k * sd);
    put(BQ_BB_LOWER, mid - K.bb_k * sd);
  }
  if (outmask & (1u << BQ_ATR)) put(BQ_ATR, mean_of(tr_q, K.atr_w, true));
  if (outmask & (1u << BQ_TWAP)) put(BQ_TWAP, mean_of(o4_q, K.twap_w, false));
  if (outmask & (1u << BQ_MFI)) {
    double m = qnan();
    if (t >= K.mfi_w - 1) {
      bool same;
      double ps = window_sum(pf_q, t, K.mfi_w, same), ns = window_sum(nf_q, t, K.mfi_w, same);
      m = oscillator(ps < 0.0 ? 0.0 : ps, ns < 0.0 ? 0.0 : ns);
    }
    put(BQ_MFI, m);
  }
}

// Seed: one thread per symbol. Unbounded mode replays the whole history with
// pandas' exact EMA step (bitwise the pandas full-series EMA); frame mode
// copies the last F closes into the close ring and records the newest missing
// close. Both copy the last RING candles into the ring. One-time cost.
__global__ __launch_bounds__(TK_NT) void seed_kernel(const TickConsts K, int64_t S, int T, int64_t ld, int64_t F,
                                                     const double* __restrict__ io, const double* __restrict__ ih,
                                                     const double* __restrict__ il, const double* __restrict__ ic,
                                                     const double* __restrict__ iv, double* ring, double* ema,
                                                     double* cring, int64_t* lastnan) {
  const int64_t s = (int64_t)blockIdx.x * TK_NT + threadIdx.x;
  if (s >= S) return;
  const double* rc = ic + s * ld;
  if (F == 0) {
    double y[5] = {0, 0, 0, 0, 0}, wt[5] = {1, 1, 1, 1, 1};
    for (int t = 0; t < T; ++t) {
      const double x = rc[t];
#pragma unroll
      for (int e = 0; e < 4; ++e) ewm_step(y[e], wt[e], x, K.alpha[e], K.om[e], K.unit[e], t == 0);
      ewm_step(y[4], wt[4], y[0] - y[1], K.alpha[4], K.om[4], K.unit[4], t == 0);
    }
#pragma unroll
    for (int e = 0; e < 5; ++e) {
      ema[(int64_t)e * S + s] = y[e];
      ema[(int64_t)(5 + e) * S + s] = wt[e];
    }
  } else {
    int64_t ln = -1;
    const int64_t first = T > F ? T - F : 0;
    for (int64_t t = first; t < T; ++t) {
      const double x = rc[t];
      cring[(t % F) * S + s] = x;
      if (!win_ok(x)) ln = t;
    }
    lastnan[s] = ln;
  }
  const double* src[5] = {io + s * ld, ih + s * ld, il + s * ld, rc, iv + s * ld};
  const int first = T > RING ? T - RING : 0;
  for (int t = first; t < T; ++t)
#pragma unroll
    for (int f = 0; f < 5; ++f) ring[((int64_t)f * RING + (t % RING)) * S + s] = src[f][t];
}

static double alpha_span(double span) {
  const double com = (span - 1.0) / 2.0;
  return 1.0 / (1.0 + com);
}

static bool win_ok(int w) { return w >= 1 && w <= BQ_MAX_WINDOW; }

}  // namespace bq

extern "C" {

int bq_state_create_frame(bq_state** out, int64_t S, const bq_params* params, int64_t frame) {
  using namespace bq;
  if (!out || S <= 0) return BQ_EINVAL;
  *out = nullptr;
  // the frame must hold every rolling window (they read the RING-candle ring)
  if (frame != 0 && (frame < RING || frame > TK_MAX_FRAME)) return BQ_EINVAL;
  bq_params P;
  if (params) P = *params;
  else bq_default_params(&P);
  for (int i = 0; i < 3; ++i)
    if (!win_ok(P.ma_periods[i])) return BQ_EINVAL;
  if (!win_ok(P.rsi_window) || !win_ok(P.bb_window) || !win_ok(P.atr_window) || !win_ok(P.twap_window) ||
      !win_ok(P.mfi_window) || P.bb_ddof < 0 || P.macd_fast < 1 || P.macd_slow < 1 || P.macd_signal < 1 ||
      P.ema_spans[0] < 1 || P.ema_spans[1] < 1)
    return BQ_EINVAL;
  bq_state* st = (bq_state*)calloc(1, sizeof(bq_state));
  if (!st) return BQ_EINVAL;
  st->S = S;
  st->count = 0;
  st->F = frame;
  TickConsts& K = st->K;
  for (int i = 0; i < 3; ++i) K.ma[i] = P.ma_periods[i];
  K.rsi_w = P.rsi_window;
  K.bb_w = P.bb_window;
  K.bb_ddof = P.bb_ddof;
  K.atr_w = P.atr_window;
  K.twap_w = P.twap_window;
  K.mfi_w = P.mfi_window;
  K.bb_k = P.bb_k;
  const double spans[5] = {(double)P.macd_fast, (double)P.macd_slow, (double)P.ema_spans[0],
                           (double)P.ema_spans[1], (double)P.macd_signal};
  for (int e = 0; e < 5; ++e) {
    K.alpha[e] = alpha_span(spans[e]);
    K.om[e] = 1.0 - K.alpha[e];
    volatile double den = K.om[e] + K.alpha[e];
    K.unit[e] = den == 1.0;
  }
  bool ok = hipMalloc(&st->ring, sizeof(double) * 5 * RING * S) == hipSuccess;
  if (ok && frame == 0) ok = hipMalloc(&st->ema, sizeof(double) * 10 * S) == hipSuccess;
  if (ok && frame > 0) ok = hipMalloc(&st->cring, sizeof(double) * frame * S) == hipSuccess;
  if (ok && frame > 0) ok = hipMalloc(&st->lastnan, sizeof(int64_t) * S) == hipSuccess;
  if (ok && frame > 0) ok = hipMemset(st->lastnan, 0xff, sizeof(int64_t) * S) == hipSuccess;   // -1
  if (!ok) {
    (void)hipFree(st->ring);
    (void)hipFree(st->ema);
    (void)hipFree(st->cring);
    (void)hipFree(st->lastnan);
    free(st);
    return BQ_EHIP;
  }
  *out = st;
  return BQ_OK;
}

int bq_state_create(bq_state** out, int64_t S, const bq_params* params) {
  return bq_state_create_frame(out, S, params, BQ_TICK_FRAME);
}

int bq_state_destroy(bq_state* st) {
  if (!st) return BQ_EINVAL;
  (void)hipFree(st->ring);
  (void)hipFree(st->ema);
  (void)hipFree(st->cring);
  (void)hipFree(st->lastnan);
  free(st);
  return BQ_OK;
}

int64_t bq_state_symbols(const bq_state* st) { return st ? st->S : -1; }
int64_t bq_state_count(const bq_state* st) { return st ? st->count : -1; }
int64_t bq_state_frame(const bq_state* st) { return st ? st->F : -1; }

int bq_state_seed(bq_state* st, const double* const* in, int64_t T, int64_t ld_in, void* stream) {
  using namespace bq;
  if (!st) return BQ_ESTATE;
  if (!in || T < 1 || ld_in < T || T > 0x7fffffff) return BQ_EINVAL;
  for (int i = 0; i < BQ_NUM_INPUTS; ++i)
    if (!in[i]) return BQ_EINVAL;
  const unsigned blocks = (unsigned)((st->S + TK_NT - 1) / TK_NT);
  hipLaunchKernelGGL(seed_kernel, dim3(blocks), dim3(TK_NT), 0, (hipStream_t)stream, st->K, st->S, (int)T, ld_in,
                     st->F, in[0], in[1], in[2], in[3], in[4], st->ring, st->ema, st->cring, st->lastnan);
  if (hipGetLastError() != hipSuccess) return BQ_EHIP;
  st->count = T;
  return BQ_OK;
}

int bq_tick(bq_state* st, const double* const* nw, double* const* out, void* stream) {
  using namespace bq;
  if (!st) return BQ_ESTATE;
  if (!nw || !out) return BQ_EINVAL;
  for (int i = 0; i < BQ_NUM_INPUTS; ++i)
    if (!nw[i]) return BQ_EINVAL;
  unsigned mask = 0;
  for (int i = 0; i < BQ_NUM_ENRICH_COLS; ++i)
    if (out[i]) mask |= 1u << i;
  // The output pointer table travels in kernel-argument space.
  OutTable tab;
  for (int i = 0; i < BQ_NUM_ENRICH_COLS; ++i) tab.p[i] = out[i];
  const unsigned blocks = (unsigned)((st->S + TK_SYM - 1) / TK_SYM);
  hipLaunchKernelGGL(tick_kernel, dim3(blocks), dim3(TK_NT), 0, (hipStream_t)stream, st->K, st->S, st->count,
                     st->F, st->ring, st->ema, st->cring, st->lastnan, nw[0], nw[1], nw[2], nw[3], nw[4], tab, mask);
  if (hipGetLastError() != hipSuccess) return BQ_EHIP;
  st->count += 1;
  return BQ_OK;
}

}  // extern "C"
