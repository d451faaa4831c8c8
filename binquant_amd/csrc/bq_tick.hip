// Streaming tick path for gfx950: one new candle per symbol per tick.
//
// The reference recomputes every indicator column from a freshly fetched
// 400-candle frame on every closed-kline message
// (consumers/klines_provider.py:201-227 -> producers/context_evaluator.py:347-512).
// Here each symbol keeps device-resident state instead:
//   * a ring of the last RING candles (o, h, l, c, v), slot-major [RING][S]
//     so that lane = symbol reads are coalesced;
//   * the five EMA carries (macd fast/slow, ema20, ema50, macd signal) and
//     their old weights, updated with pandas' exact ewm(adjust=False,
//     ignore_na=False) step — a NaN candle (a symbol without a candle this
//     tick) decays the old weight by (1 - alpha) and holds the value, as
//     pandas does across a NaN gap — so tick EMAs equal the full-series
//     pandas EMAs bit for bit once seeded;
//   * rolling windows re-summed from the ring each tick (compensated), which
//     keeps them drift-free; pandas' constant-window rules are applied.
// One thread per symbol; a 10k-symbol tick is a single ~40-workgroup launch.
#include "bq_device.h"
#include "binquant_amd.h"

#include <stdlib.h>
#include <string.h>

namespace bq {

constexpr int RING = BQ_MAX_WINDOW + 2;   // 128
constexpr int TK_NT = 256;

struct OutTable {
  double* p[BQ_NUM_ENRICH_COLS];
};

struct TickConsts {
  int ma[3];
  int rsi_w, bb_w, bb_ddof, atr_w, twap_w, mfi_w;
  double bb_k;
  double alpha[5], om[5];   // 0 macd fast, 1 macd slow, 2 ema0, 3 ema1, 4 signal
};

}  // namespace bq

struct bq_state {
  int64_t S;
  int64_t count;
  bq::TickConsts K;
  double* ring;   // [5][RING][S]
  double* ema;    // [10][S]: 5 EMA values, then their 5 old weights
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
// ewm_scalar): y = weighted, w = old_wt. With no NaN gap w == 1 before the
// decay and (om * y + al * x) / (om + al) is the plain update (om + al == 1.0
// exactly for integer spans, so the divide is the identity).
__device__ __forceinline__ void ewm_step(double& y, double& w, double x, double al, double om, bool first) {
  if (first) {
    y = x;
    w = 1.0;
    return;
  }
  const bool obs = x == x;
  if (y == y) {
    w *= om;
    if (obs) {
      if (y != x) y = (w * y + al * x) / (w + al);
      w = 1.0;
    }
  } else if (obs) {
    y = x;
  }
}

__global__ __launch_bounds__(TK_NT) void tick_kernel(const TickConsts K, int64_t S, int64_t n, double* ring,
                                                     double* ema, const double* __restrict__ no,
                                                     const double* __restrict__ nh, const double* __restrict__ nl,
                                                     const double* __restrict__ nc, const double* __restrict__ nv,
                                                     const OutTable outp, unsigned outmask) {
  const int64_t s = (int64_t)blockIdx.x * TK_NT + threadIdx.x;
  if (s >= S) return;
  const int64_t t = n;   // index of the new candle
  const double x = nc[s];
  {
    const int64_t slot = t % RING;
    ring[((int64_t)0 * RING + slot) * S + s] = no[s];
    ring[((int64_t)1 * RING + slot) * S + s] = nh[s];
    ring[((int64_t)2 * RING + slot) * S + s] = nl[s];
    ring[((int64_t)3 * RING + slot) * S + s] = x;
    ring[((int64_t)4 * RING + slot) * S + s] = nv[s];
  }
  double y[5];
#pragma unroll
  for (int e = 0; e < 5; ++e) {
    double v = ema[(int64_t)e * S + s], wt = ema[(int64_t)(5 + e) * S + s];
    ewm_step(v, wt, e < 4 ? x : y[0] - y[1], K.alpha[e], K.om[e], t == 0);
    y[e] = v;
    ema[(int64_t)e * S + s] = v;
    ema[(int64_t)(5 + e) * S + s] = wt;
  }
  const double macd = y[0] - y[1];

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
  auto put = [&](int col, double v) {
    if (outmask & (1u << col)) outp.p[col][s] = v;
  };

#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (outmask & (1u << (BQ_MA_FAST + i))) put(BQ_MA_FAST + i, mean_of(close_q, K.ma[i], false));
  put(BQ_MACD, macd);
  put(BQ_MACD_SIGNAL, y[4]);
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
  put(BQ_EMA_FAST, y[2]);
  put(BQ_EMA_SLOW, y[3]);
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

// Seed: one thread per symbol replays the whole history sequentially with
// pandas' exact EMA step (bitwise the pandas full-series EMA) and copies the
// last RING candles into the ring. One-time cost.
__global__ __launch_bounds__(TK_NT) void seed_kernel(const TickConsts K, int64_t S, int T, int64_t ld,
                                                     const double* __restrict__ io, const double* __restrict__ ih,
                                                     const double* __restrict__ il, const double* __restrict__ ic,
                                                     const double* __restrict__ iv, double* ring, double* ema) {
  const int64_t s = (int64_t)blockIdx.x * TK_NT + threadIdx.x;
  if (s >= S) return;
  const double* rc = ic + s * ld;
  double y[5] = {0, 0, 0, 0, 0}, wt[5] = {1, 1, 1, 1, 1};
  for (int t = 0; t < T; ++t) {
    const double x = rc[t];
#pragma unroll
    for (int e = 0; e < 4; ++e) ewm_step(y[e], wt[e], x, K.alpha[e], K.om[e], t == 0);
    ewm_step(y[4], wt[4], y[0] - y[1], K.alpha[4], K.om[4], t == 0);
  }
#pragma unroll
  for (int e = 0; e < 5; ++e) {
    ema[(int64_t)e * S + s] = y[e];
    ema[(int64_t)(5 + e) * S + s] = wt[e];
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

int bq_state_create(bq_state** out, int64_t S, const bq_params* params) {
  using namespace bq;
  if (!out || S <= 0) return BQ_EINVAL;
  *out = nullptr;
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
  }
  if (hipMalloc(&st->ring, sizeof(double) * 5 * RING * S) != hipSuccess) {
    free(st);
    return BQ_EHIP;
  }
  if (hipMalloc(&st->ema, sizeof(double) * 10 * S) != hipSuccess) {
    (void)hipFree(st->ring);
    free(st);
    return BQ_EHIP;
  }
  *out = st;
  return BQ_OK;
}

int bq_state_destroy(bq_state* st) {
  if (!st) return BQ_EINVAL;
  (void)hipFree(st->ring);
  (void)hipFree(st->ema);
  free(st);
  return BQ_OK;
}

int64_t bq_state_symbols(const bq_state* st) { return st ? st->S : -1; }
int64_t bq_state_count(const bq_state* st) { return st ? st->count : -1; }

int bq_state_seed(bq_state* st, const double* const* in, int64_t T, int64_t ld_in, void* stream) {
  using namespace bq;
  if (!st) return BQ_ESTATE;
  if (!in || T < 1 || ld_in < T || T > 0x7fffffff) return BQ_EINVAL;
  for (int i = 0; i < BQ_NUM_INPUTS; ++i)
    if (!in[i]) return BQ_EINVAL;
  const unsigned blocks = (unsigned)((st->S + TK_NT - 1) / TK_NT);
  hipLaunchKernelGGL(seed_kernel, dim3(blocks), dim3(TK_NT), 0, (hipStream_t)stream, st->K, st->S, (int)T, ld_in,
                     in[0], in[1], in[2], in[3], in[4], st->ring, st->ema);
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
  const unsigned blocks = (unsigned)((st->S + TK_NT - 1) / TK_NT);
  hipLaunchKernelGGL(tick_kernel, dim3(blocks), dim3(TK_NT), 0, (hipStream_t)stream, st->K, st->S, st->count,
                     st->ring, st->ema, nw[0], nw[1], nw[2], nw[3], nw[4], tab, mask);
  if (hipGetLastError() != hipSuccess) return BQ_EHIP;
  st->count += 1;
  return BQ_OK;
}

}  // extern "C"
