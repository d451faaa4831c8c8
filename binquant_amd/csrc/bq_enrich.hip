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
// candles in tiles of TT = 1024 (K = 4 consecutive candles per lane: a lane's
// 32 bytes per field are contiguous, a wave covers 2 KiB per field). Inputs of
// tile n+1 are prefetched into registers while tile n computes; outputs are
// streamed with non-temporal stores. Two workgroup barriers per tile.
//
// Per tile:
//   * close-based rolling means (ma_7/25/100, bb_mid) are differences of a
//     compensated (double-double) prefix sum: wave scan with __shfl_up, the
//     wave-local prefix rounded once into LDS, wave bases added on lookup;
//   * short windows (RSI, ATR, TWAP, MFI, Bollinger std) are summed directly
//     from per-candle arrays in an LDS ring (tile + 128-candle halo);
//   * pandas' constant-window exactness (rolling().mean() returns the value
//     itself, var() returns 0 when every value in the window is identical)
//     via a max-scan of the last index where close changed (long windows) or
//     an all-equal test while summing (short windows);
//   * the EMA family (macd fast/slow, macd signal, ema20, ema50) is one
//     associative scan of affine maps on the state (y12, y26, signal, y20,
//     y50) — macd's signal EMA makes that a 3x3 lower-triangular system —
//     after which each lane replays its 4 candles with pandas' exact
//     ewm(adjust=False) update, so per-element rounding follows pandas.
// HBM traffic: every input byte read once (plus one 24-byte neighbour read per
// lane and tile), every output byte written once.
#include "bq_device.h"
#include "binquant_amd.h"

#include <stddef.h>
#include <string.h>

#include <type_traits>

namespace bq {

#ifndef BQ_EN_NT
#define BQ_EN_NT 256   // threads per workgroup
#endif
#ifndef BQ_EN_K
#define BQ_EN_K 4      // consecutive candles per lane
#endif
#ifndef BQ_EN_NTSTORE
#define BQ_EN_NTSTORE 1   // non-temporal output stores
#endif
#ifndef BQ_EN_SWIZZLE
#define BQ_EN_SWIZZLE 0   // scattered symbol order (measured slower: 3.85 -> 4.06 ms at 12.5k, 26.2 -> 28.7 ms at 100k)
#endif
#ifndef BQ_EN_WPS
#define BQ_EN_WPS 3    // __launch_bounds__ min waves per SIMD
#endif
constexpr int EN_NT = BQ_EN_NT;
constexpr int EN_NW = EN_NT / WAVE;
constexpr int EN_K = BQ_EN_K;
constexpr int EN_TT = EN_NT * EN_K;   // 1024
constexpr int EN_LK = EN_K == 2 ? 1 : EN_K == 4 ? 2 : 3;   // log2(EN_K)
constexpr int EN_H = 128;             // halo >= BQ_MAX_WINDOW + 2
constexpr int EN_R = EN_H + EN_TT;    // 1152
static_assert(EN_K % 2 == 0 && EN_TT >= EN_H && EN_K * WAVE > BQ_MAX_WINDOW, "tile shape");

#ifndef BQ_EN_LDSPERM
#define BQ_EN_LDSPERM 1   // lane-interleaved LDS ring layout (bank-conflict free)
#endif
// LDS ring position -> physical slot. A lane owns EN_K consecutive ring
// positions, so in the natural layout the 64 lanes of a wave access slots
// EN_K doubles apart (8 dwords): every ds_read/ds_write_b64 of the ring
// serialises 4-way on the 64 banks. Storing position i at
// (i % EN_K) * (R / EN_K) + i / EN_K puts the lanes' k-th candles side by side
// (2 dwords apart, conflict free); every window walk reads the same residue
// class on all lanes at each step (lane positions differ by multiples of
// EN_K), so it stays conflict free too.
#if BQ_EN_LDSPERM
#define LX(i) ((((i) & (EN_K - 1)) * (EN_R / EN_K)) + ((i) >> EN_LK))
// slot of ring position pb + x for the lane whose first position is pb
// (pb % EN_K == 0, lb = pb / EN_K): lb + LX(x), x may be negative (the shift
// floors). Window offsets x are wave-uniform, so LX(x) is scalar arithmetic
// and each access is one VGPR base + an SGPR / immediate offset.
#define RS(x) (lb + LX(x))
#define RS1(x) (pb / EN_K + LX(x))
#else
#define LX(i) (i)
#define RS(x) (pb + (x))
#define RS1(x) (pb + (x))
#endif
static_assert(!BQ_EN_LDSPERM || ((1 << EN_LK) == EN_K && EN_R % EN_K == 0), "LX: power-of-two candles per lane");

// EMA slots in the scan state
enum { E_FAST = 0, E_SLOW, E_SIG, E_0, E_1, NE };

// Power of the per-thread state map M^(K n): lower-triangular 3x3 block for
// (fast, slow, signal) + two scalars.  Applied to v: (a0 v0, a1 v1,
// p v0 + q v1 + a2 v2, a3 v3, a4 v4).
struct Pow {
  double a0, a1, p, q, a2, a3, a4;
};

__host__ __device__ __forceinline__ Pow pow_mul(const Pow& T, const Pow& U) {   // T after U
  Pow r;
  r.a0 = T.a0 * U.a0;
  r.a1 = T.a1 * U.a1;
  r.p = fma(T.p, U.a0, T.a2 * U.p);
  r.q = fma(T.q, U.a1, T.a2 * U.q);
  r.a2 = T.a2 * U.a2;
  r.a3 = T.a3 * U.a3;
  r.a4 = T.a4 * U.a4;
  return r;
}

// the EMA constants a launch shares, formed once on the host (ema_consts):
// pandas' weights per EMA and the powers of the scan's state map
struct EmaHost {
  double al[NE], om[NE], den[NE], la[NE], lb[NE];
  Pow step;            // M (one candle)
  Pow wstep[6];        // (M^K)^(2^j)
  Pow wave[EN_NW + 1]; // (M^K)^(64 m)
};

struct EnrichArgs {
  EmaHost ema;
  const double* in[BQ_NUM_INPUTS];
  double* out[BQ_NUM_ENRICH_COLS];
  int64_t ld_in, ld_out;
  int64_t S, swz;   // symbol of workgroup b = (b * swz) % S (swz coprime to S)
  int T;
  int ma[3];
  int rsi_w, bb_w, bb_ddof, atr_w, twap_w, mfi_w;
  int span[NE];   // macd fast, macd slow, macd signal, ema0, ema1
  double bb_k;
  double inv_ma[3], inv_rsi, inv_bb, inv_bb_dv, inv_atr, inv_twap;   // 1.0 / window (host)
};

// per-workgroup LDS copy: the host's constants, then the lane powers
struct EmaConsts {
  double al[NE], om[NE], den[NE], la[NE], lb[NE];
  Pow step;            // M (one candle)
  Pow wstep[6];        // (M^K)^(2^j)
  Pow wave[EN_NW + 1]; // (M^K)^(64 m)
  Pow lane[WAVE];      // (M^K)^lane
};
static_assert(sizeof(EmaHost) % sizeof(double) == 0 && offsetof(EmaConsts, lane) == sizeof(EmaHost),
              "EmaConsts begins with EmaHost's layout");

// pandas: comass = (span - 1) / 2, alpha = 1 / (1 + comass); the scan's
// state map and its powers (host: the same IEEE operations the kernel used to
// form per workgroup — one thread's serial chain ahead of every row)
static EmaHost ema_consts(const int (&span)[NE]) {
  EmaHost E;
  for (int e = 0; e < NE; ++e) {
    const double com = ((double)span[e] - 1.0) / 2.0;
    const double al = 1.0 / (1.0 + com);
    E.al[e] = al;
    E.om[e] = 1.0 - al;
    E.den[e] = E.om[e] + al;
    E.la[e] = E.om[e] / E.den[e];
    E.lb[e] = al / E.den[e];
  }
  Pow m;
  m.a0 = E.la[E_FAST];
  m.a1 = E.la[E_SLOW];
  m.a2 = E.la[E_SIG];
  m.p = E.lb[E_SIG] * E.la[E_FAST];
  m.q = -(E.lb[E_SIG] * E.la[E_SLOW]);
  m.a3 = E.la[E_0];
  m.a4 = E.la[E_1];
  E.step = m;
  Pow mk = m;
  for (int k = 1; k < EN_K; ++k) mk = pow_mul(m, mk);
  for (int j = 0; j < 6; ++j) {
    E.wstep[j] = mk;
    mk = pow_mul(mk, mk);
  }
  Pow r = {1.0, 1.0, 0.0, 0.0, 1.0, 1.0, 1.0};
  const Pow w64 = pow_mul(E.wstep[5], E.wstep[5]);   // (M^K)^64
  for (int k = 0; k <= EN_NW; ++k) {
    E.wave[k] = r;
    r = pow_mul(w64, r);
  }
  return E;
}

__device__ __forceinline__ void pow_apply(const Pow& A, const double (&v)[NE], double (&r)[NE]) {
  r[E_FAST] = A.a0 * v[E_FAST];
  r[E_SLOW] = A.a1 * v[E_SLOW];
  r[E_SIG] = fma(A.p, v[E_FAST], fma(A.q, v[E_SLOW], A.a2 * v[E_SIG]));
  r[E_0] = A.a3 * v[E_0];
  r[E_1] = A.a4 * v[E_1];
}

// pandas ewm(adjust=False): weighted = old_wt*weighted + new_wt*cur;
// weighted /= old_wt + new_wt; skipped when weighted == cur. For every integer
// span old_wt + new_wt == 1.0 exactly and the divide is the identity: DIV=false
// compiles it out (the host checks this with the same IEEE arithmetic).
template <bool DIV>
__device__ __forceinline__ double ema_step(double y, double x, const EmaConsts& E, int e) {
  if (y != x) {
    y = E.om[e] * y + E.al[e] * x;
    if (DIV) y = y / E.den[e];
  }
  return y;
}

typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void load4(const double* __restrict__ row, int tb, int T, bool vec, double (&x)[EN_K]) {
  if (vec && tb + EN_K <= T) {
    const dbl2* p = reinterpret_cast<const dbl2*>(row + tb);
#pragma unroll
    for (int j = 0; j < EN_K / 2; ++j) {
      const dbl2 a = p[j];
      x[2 * j] = a.x;
      x[2 * j + 1] = a.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < EN_K; ++k) x[k] = (tb + k < T) ? row[tb + k] : 0.0;
  }
}

// Output pointers are re-read from LDS each tile (see sA), which leaves the
// compiler with generic pointers; casting to the global address space keeps
// the stores global_store (flat stores would also count against lgkmcnt and
// serialise the LDS reads that follow them).
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) dbl2 gdbl2;

#ifndef BQ_EN_SWAPST
#define BQ_EN_SWAPST 1   // whole-line output stores through v_permlane32_swap
#endif

__device__ __forceinline__ void put2(gdouble* row, int t, int T, bool full, dbl2 v) {
  if (full || t + 2 <= T) {
#if BQ_EN_NTSTORE
    __builtin_nontemporal_store(v, reinterpret_cast<gdbl2*>(row + t));
#else
    *reinterpret_cast<gdbl2*>(row + t) = v;
#endif
  } else if (t < T) {
    row[t] = v.x;
  }
}

// Output stores. A lane holds 4 consecutive candles, so its natural pair of
// 16-byte stores covers every other 16 bytes of the wave's 2 KiB per
// instruction — half of each 128-byte line, the other half a separate
// instruction. At the headline shape that pattern caps the 5-in / 14-out
// stream at ~5.3 TB/s, whole-line coverage per instruction reaches ~6.4
// (tools/coalesce_ceiling.hip, 100k x 10k). v_permlane32_swap exchanges the
// upper half-wave's first pair with the lower half-wave's second pair: then
// register A holds candles [0, 128) of the wave's slice (lane a < 32 its own
// 4a, 4a+1; lane 32 + a lane a's 4a+2, 4a+3) and register B candles
// [128, 256), so each store instruction writes one contiguous KiB (lanes
// permuted within it). `vec` is wave-uniform (a kernel argument), so every
// lane takes part in the swap; `full` (every candle of the tile in range)
// drops the range checks.
__device__ __forceinline__ void store4(double* __restrict__ row_, int tb, int T, bool vec, const double (&x)[EN_K],
                                       bool full = false) {
  gdouble* row = (gdouble*)row_;
#if BQ_EN_SWAPST
  if constexpr (EN_K == 4) {
    if (vec) {
      union {
        dbl2 d;
        unsigned u[4];
      } a, b;
      a.d = dbl2{x[0], x[1]};
      b.d = dbl2{x[2], x[3]};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto r = __builtin_amdgcn_permlane32_swap(a.u[i], b.u[i], false, false);
        a.u[i] = r[0];
        b.u[i] = r[1];
      }
      const int lane = __lane_id();
      const int ta = lane < 32 ? tb : tb - 126;   // lane 32 + a: wave base + 4a + 2
      put2(row, ta, T, full, a.d);
      put2(row, ta + 128, T, full, b.d);
      return;
    }
  }
#endif
  if (vec && tb + EN_K <= T) {
    gdbl2* p = reinterpret_cast<gdbl2*>(row + tb);
#pragma unroll
    for (int j = 0; j < EN_K / 2; ++j) {
#if BQ_EN_NTSTORE
      __builtin_nontemporal_store(dbl2{x[2 * j], x[2 * j + 1]}, p + j);
#else
      p[j] = dbl2{x[2 * j], x[2 * j + 1]};
#endif
    }
  } else {
#pragma unroll
    for (int k = 0; k < EN_K; ++k)
      if (tb + k < T) row[tb + k] = x[k];
  }
}

struct Tile {
  double o[EN_K], h[EN_K], l[EN_K], c[EN_K], v[EN_K];
  double ph, pl, pc;   // candle tb-1 (NaN before the series start)
};

#ifndef BQ_EN_LINELOAD
#define BQ_EN_LINELOAD 0   // line-covering input loads (bq_device.h load_pieces): measured 0.5-1.6% slower here
#endif

__device__ __forceinline__ void load_tile(const EnrichArgs& A, int64_t row, int tb, bool vin, Tile& t) {
  const int T = A.T;
  if (BQ_EN_LINELOAD && vin) {   // wave-uniform; exchanged into place at use (tile_arrived)
    load_pieces<EN_K>(A.in[BQ_OPEN] + row, tb, T, t.o, 0.0);
    load_pieces<EN_K>(A.in[BQ_HIGH] + row, tb, T, t.h, 0.0);
    load_pieces<EN_K>(A.in[BQ_LOW] + row, tb, T, t.l, 0.0);
    load_pieces<EN_K>(A.in[BQ_CLOSE] + row, tb, T, t.c, 0.0);
    load_pieces<EN_K>(A.in[BQ_VOLUME] + row, tb, T, t.v, 0.0);
  } else {
    load4(A.in[BQ_OPEN] + row, tb, T, vin, t.o);
    load4(A.in[BQ_HIGH] + row, tb, T, vin, t.h);
    load4(A.in[BQ_LOW] + row, tb, T, vin, t.l);
    load4(A.in[BQ_CLOSE] + row, tb, T, vin, t.c);
    load4(A.in[BQ_VOLUME] + row, tb, T, vin, t.v);
  }
  if (tb >= 1 && tb <= T) {
    t.ph = A.in[BQ_HIGH][row + tb - 1];
    t.pl = A.in[BQ_LOW][row + tb - 1];
    t.pc = A.in[BQ_CLOSE][row + tb - 1];
  } else {
    t.ph = t.pl = t.pc = qnan();
  }
}

// the prefetched tile's pieces -> each lane's EN_K consecutive candles
__device__ __forceinline__ void tile_arrived(bool vin, Tile& t) {
  if (BQ_EN_LINELOAD && vin) {
    line_unexchange_x<EN_K>(t.o);
    line_unexchange_x<EN_K>(t.h);
    line_unexchange_x<EN_K>(t.l);
    line_unexchange_x<EN_K>(t.c);
    line_unexchange_x<EN_K>(t.v);
  }
}

// VOUT: every output row 16-byte aligned (a template argument, so the
// unaligned element-wise store path is not compiled into the common kernel)
// DEF: the windows are the reference's (ma 7/25/100, rsi 14, bb 20, atr 14,
// twap 12, mfi 14): compile-time window lengths let every window walk unroll
// completely (all ring reads issued before the dependent sums, immediate LDS
// offsets) — the same operations in the same order as the generic kernel.
template <bool DEF>
__device__ __forceinline__ int win_of(int def, int v) {
  return DEF ? def : __builtin_amdgcn_readfirstlane(v);
}

// ---- rows holding a missing or non-finite input ------------------------------
// The tile walk assumes finite candles: a NaN close would poison the close
// prefix and the EMA scan for the rest of the row, and the sliding window sums
// for the rest of a lane's block. pandas instead treats a missing value (and,
// through _prep_values, +-inf) as an absent observation: a rolling window
// holding one is NaN (min_periods = window), ewm(adjust=False, ignore_na=False)
// decays its old weight across the gap and resumes (aggregations.pyx ewm).
// A workgroup whose row held one recomputes the whole row here after the walk
// — pandas' elementwise series and window definitions candle by candle
// (oracle/indicators_ref.py: SMA RSI via delta.where, MFI flows via tp.where,
// skip-NaN true range, the same-value rule of rolling mean / var), the EMA
// family as pandas' serial recursion (bit for bit) — and overwrites its
// outputs. Real klines never take this path (Binance candles always carry
// prices); it exists so that a drop-in frame with gaps gets pandas' answer.
struct WinAgg {
  double sum, first;
  bool ok, same;
};

template <typename F>
__device__ __forceinline__ WinAgg win_agg(F val, int t, int w) {
  WinAgg a = {0.0, 0.0, t >= w - 1, true};
  if (!a.ok) return a;
  a.first = val(t - w + 1);
  for (int j = t - w + 1; j <= t; ++j) {
    const double x = val(j);
    if (!__builtin_isfinite(x)) {
      a.ok = false;
      return a;
    }
    a.same &= x == a.first;
    a.sum += x;
  }
  return a;
}

// pandas ewm(adjust=False, ignore_na=False) state: weighted (NaN before the
// first observation), old_wt
__device__ __forceinline__ double ewm_gap_step(double& wt, double& old, double x, double al, double om) {
  const bool obs = __builtin_isfinite(x);   // _prep_values: +-inf -> NaN
  if (wt == wt) {
    old *= om;
    if (obs) {
      if (wt != x) {
        wt = old * wt + al * x;
        wt /= (old + al);
      }
      old = 1.0;
    }
  } else if (obs) {
    wt = x;
  }
  return wt;
}

__device__ __forceinline__ void enrich_row_missing(const EnrichArgs& P, const EmaConsts& E, int64_t irow, int64_t orow,
                                                double* bc, double* b0, double* b1, double* b2, double* b3) {
  const int tid = threadIdx.x, T = P.T;
  const double* __restrict__ po = P.in[BQ_OPEN] + irow;
  const double* __restrict__ ph = P.in[BQ_HIGH] + irow;
  const double* __restrict__ pl = P.in[BQ_LOW] + irow;
  const double* __restrict__ pc = P.in[BQ_CLOSE] + irow;
  const double* __restrict__ pv = P.in[BQ_VOLUME] + irow;
  auto C = [&](int j) { return j >= 0 ? pc[j] : qnan(); };
  auto TP = [&](int j) { return j >= 0 ? typical_price(ph[j], pl[j], pc[j]) : qnan(); };
  auto put = [&](int col, int t, double v) {
    if (P.out[col]) P.out[col][orow + t] = v;
  };
  auto mean_of = [&](const WinAgg& a, int w) { return !a.ok ? qnan() : (a.same ? a.first : a.sum / (double)w); };
  for (int t = tid; t < T; t += EN_NT) {
    for (int i = 0; i < 3; ++i)
      if (P.out[BQ_MA_FAST + i]) put(BQ_MA_FAST + i, t, mean_of(win_agg(C, t, P.ma[i]), P.ma[i]));
    if (P.out[BQ_BB_UPPER] || P.out[BQ_BB_MID] || P.out[BQ_BB_LOWER]) {
      const int w = P.bb_w;
      const WinAgg a = win_agg(C, t, w);
      double m = qnan(), sd = qnan();
      if (a.ok) {
        m = mean_of(a, w);
        double ss = 0.0;
        if (!a.same)
          for (int j = t - w + 1; j <= t; ++j) {
            const double d = pc[j] - m;
            ss += d * d;
          }
        sd = w - P.bb_ddof > 0 ? sqrt(ss / (double)(w - P.bb_ddof)) : qnan();
      }
      put(BQ_BB_MID, t, m);
      put(BQ_BB_UPPER, t, m + (P.bb_k * sd));
      put(BQ_BB_LOWER, t, m - (P.bb_k * sd));
    }
    if (P.out[BQ_TWAP])
      put(BQ_TWAP, t, mean_of(win_agg([&](int j) { return ohlc4(po[j], ph[j], pl[j], pc[j]); }, t, P.twap_w),
                              P.twap_w));
    if (P.out[BQ_ATR])
      put(BQ_ATR, t, mean_of(win_agg([&](int j) { return true_range(ph[j], pl[j], C(j - 1)); }, t, P.atr_w),
                             P.atr_w));
    if (P.out[BQ_RSI]) {   // delta.where(delta > 0, 0.0): a missing delta is a 0 gain and loss
      const int w = P.rsi_w;
      const WinAgg g = win_agg([&](int j) { const double d = C(j) - C(j - 1); return d > 0.0 ? d : 0.0; }, t, w);
      const WinAgg l = win_agg([&](int j) { const double d = C(j) - C(j - 1); return d < 0.0 ? -d : 0.0; }, t, w);
      const double rs = mean_of(g, w) / mean_of(l, w);
      put(BQ_RSI, t, 100.0 - (100.0 / (1.0 + rs)));
    }
    if (P.out[BQ_MFI]) {   // mf.where(tp > prev, 0.0) / mf.where(tp < prev, 0.0), rolling sums
      const int w = P.mfi_w;
      const WinAgg p = win_agg([&](int j) { const double tp = TP(j); return tp > TP(j - 1) ? tp * pv[j] : 0.0; }, t, w);
      const WinAgg n = win_agg([&](int j) { const double tp = TP(j); return tp < TP(j - 1) ? tp * pv[j] : 0.0; }, t, w);
      const double ps = p.ok ? p.sum : qnan(), ns = n.ok ? n.sum : qnan();
      put(BQ_MFI, t, 100.0 - (100.0 / (1.0 + ps / ns)));
    }
  }
  // the EMA family: pandas' recursion, serial, closes staged through LDS
  const bool ema = P.out[BQ_MACD] || P.out[BQ_MACD_SIGNAL] || P.out[BQ_EMA_FAST] || P.out[BQ_EMA_SLOW];
  if (!ema) return;
  double wf = qnan(), of = 1.0, ws = qnan(), os = 1.0, wg = qnan(), og = 1.0, we = qnan(), oe = 1.0;
  for (int c0 = 0; c0 < T; c0 += EN_TT) {
    const int n = min(EN_TT, T - c0);
    __syncthreads();   // the previous chunk's results are stored
    for (int i = tid; i < n; i += EN_NT) bc[i] = pc[c0 + i];
    __syncthreads();
    if (tid == 0) {   // macd fast / slow and the signal EMA of their difference
      for (int i = 0; i < n; ++i) {
        const double x = bc[i];
        const double f = ewm_gap_step(wf, of, x, E.al[E_FAST], E.om[E_FAST]);
        const double s = ewm_gap_step(ws, os, x, E.al[E_SLOW], E.om[E_SLOW]);
        const double m = f - s;
        b0[i] = m;
        b1[i] = ewm_gap_step(wg, og, m, E.al[E_SIG], E.om[E_SIG]);
      }
    } else if (tid == WAVE || tid == 2 * WAVE) {   // ema_spans[0] / [1] on waves 1 / 2
      const int e = tid == WAVE ? E_0 : E_1;
      double* dst = tid == WAVE ? b2 : b3;
      for (int i = 0; i < n; ++i) dst[i] = ewm_gap_step(we, oe, bc[i], E.al[e], E.om[e]);
    }
    __syncthreads();
    for (int i = tid; i < n; i += EN_NT) {
      put(BQ_MACD, c0 + i, b0[i]);
      put(BQ_MACD_SIGNAL, c0 + i, b1[i]);
      put(BQ_EMA_FAST, c0 + i, b2[i]);
      put(BQ_EMA_SLOW, c0 + i, b3[i]);
    }
  }
}

template <bool DIV, bool VOUT, bool DEF>
__global__ __launch_bounds__(EN_NT, BQ_EN_WPS) void enrich_kernel(const EnrichArgs A, int vec_in) {
  // LDS ring (positions [0, H) = halo from the previous tile, [H, R) = tile)
  __shared__ double sP[EN_R];    // close prefix: halo re-based, tile wave-local
  __shared__ double sC[EN_R];    // close
  __shared__ double sTR[EN_R];   // true range
  __shared__ double sO4[EN_R];   // (o+h+l+c)/4
  __shared__ double sMF[EN_R];   // signed money flow: +tp*v up-tick, -tp*v down-tick, 0 flat
  __shared__ double sWh[EN_NW], sWl[EN_NW];
  __shared__ double sWe[EN_NW][NE];
  __shared__ int sWlc[EN_NW];
  __shared__ double sEcar[NE];
  __shared__ int sLcar, sMiss;
  __shared__ EmaConsts E;
  __shared__ EnrichArgs sA;   // window sizes / output table, re-read from LDS each
                              // tile so the compiler cannot hoist them into registers

  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  // Concurrently resident workgroups take scattered symbols: row streams of
  // neighbouring symbols (one HBM row pitch apart) otherwise pile onto the
  // same channels in lockstep (tools/row_ceiling.hip: +9% on the pure
  // streaming structure).
  const int64_t sym = BQ_EN_SWIZZLE ? ((int64_t)blockIdx.x * A.swz) % A.S : (int64_t)blockIdx.x;
  const int64_t irow = sym * A.ld_in;
  const int64_t orow = sym * A.ld_out;
  const int T = A.T;
  const bool vin = vec_in != 0, vout = VOUT;

  // the first tile's loads go out before anything else: their HBM latency
  // overlaps the serial constant set-up below (a workgroup's fixed start-up
  // cost otherwise adds ~5% to a 10k-candle row)
  Tile nx;
  load_tile(A, irow, EN_K * tid, vin, nx);

  // ---- per-workgroup constants: the host's (kernel arguments) copied into
  // LDS in parallel, the lane powers (M^K)^lane formed by the first wave
  {
    const double* src = reinterpret_cast<const double*>(&A.ema);
    double* dst = reinterpret_cast<double*>(&E);
    for (int i = tid; i < (int)(sizeof(EmaHost) / sizeof(double)); i += EN_NT) dst[i] = src[i];
  }
  if (tid < WAVE) {
    Pow r = {1.0, 1.0, 0.0, 0.0, 1.0, 1.0, 1.0};
    for (int j = 0; j < 6; ++j)
      if (tid & (1 << j)) r = pow_mul(A.ema.wstep[j], r);
    E.lane[tid] = r;
  }
  if (tid < NE) sEcar[tid] = 0.0;
  if (tid == 0) {
    sLcar = -1;
    sMiss = 0;
    sA = A;
  }
  if (tid < EN_H) {   // candles before the series start: NaN close, zero sums
    sP[LX(tid)] = 0.0;
    sC[LX(tid)] = qnan();
    sTR[LX(tid)] = 0.0;
    sO4[LX(tid)] = 0.0;
    sMF[LX(tid)] = 0.0;
  }
  __syncthreads();

  // EMA carry into candle 0 = (x0, x0, 0, x0, x0): pandas starts every EMA at
  // its first value (output[0] = x0, macd signal[0] = macd[0] = 0), and the
  // generic step from y == x leaves y unchanged, so no first-candle branch.
  if (tid == 0) {
    const double x0 = nx.c[0];   // candle 0 in either load order (line_offset(0) == 0)
    sEcar[E_FAST] = sEcar[E_SLOW] = sEcar[E_0] = sEcar[E_1] = x0;
    sEcar[E_SIG] = 0.0;
  }

  for (int t0 = 0; t0 < T; t0 += EN_TT) {
    const int tb = t0 + EN_K * tid;
    const int pb = EN_H + EN_K * tid;
    const EnrichArgs& P = sA;
    Tile cu = nx;
    tile_arrived(vin, cu);
    if (t0 + EN_TT < T) load_tile(A, irow, tb + EN_TT, vin, nx);   // prefetch tile n+1

    // ---- phase 1: per-candle quantities into the LDS ring --------------------
    int lcl[EN_K];
    {
      bool miss = false;   // a missing / non-finite input among the lane's candles (enrich_row_missing)
      double pc = cu.pc;
      double tpp = typical_price(cu.ph, cu.pl, cu.pc);
      int run = -1;
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        const int t = tb + k;
        const double c = cu.c[k];
        const double tp = typical_price(cu.h[k], cu.l[k], c);
        const double mf = tp * cu.v[k];
        const double o4 = ohlc4(cu.o[k], cu.h[k], cu.l[k], c);
        miss |= !__builtin_isfinite(o4) | !__builtin_isfinite(mf);   // any of o, h, l, c, v (or an overflow)
        sC[RS1(k)] = c;
        sTR[RS1(k)] = true_range(cu.h[k], cu.l[k], pc);
        sO4[RS1(k)] = o4;
        sMF[RS1(k)] = tp > tpp ? mf : (tp < tpp ? -mf : 0.0);
        if (t == 0 || c != pc) run = t;
        lcl[k] = run;
        pc = c;
        tpp = tp;
      }
      if (__builtin_amdgcn_ballot_w64(miss)) sMiss = 1;   // wave-uniform; read after the walk
    }
    // close prefix (compensated), wave-local
    double Ploc[EN_K];
    {
      dd tot = {0.0, 0.0};
#pragma unroll
      for (int k = 0; k < EN_K; ++k) tot = dd_add1(tot, cu.c[k]);
      const dd inc = wave_scan_dd_dpp(tot, lane);
      if (lane == WAVE - 1) {
        sWh[w] = inc.hi;
        sWl[w] = inc.lo;
      }
      dd acc = {dpp_f64<DPP_WAVE_SHR1>(inc.hi), dpp_f64<DPP_WAVE_SHR1>(inc.lo)};   // lane 0 -> 0
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        acc = dd_add1(acc, cu.c[k]);
        Ploc[k] = dd_round(acc);
        sP[RS1(k)] = Ploc[k];
      }
    }
    // EMA state scan: thread map from the zero state, then wave inclusive scan
    double ex[NE];
    {
      double b[NE] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        const double x = cu.c[k];
        b[E_FAST] = fma(E.la[E_FAST], b[E_FAST], E.lb[E_FAST] * x);
        b[E_SLOW] = fma(E.la[E_SLOW], b[E_SLOW], E.lb[E_SLOW] * x);
        b[E_SIG] = fma(E.la[E_SIG], b[E_SIG], E.lb[E_SIG] * (b[E_FAST] - b[E_SLOW]));
        b[E_0] = fma(E.la[E_0], b[E_0], E.lb[E_0] * x);
        b[E_1] = fma(E.la[E_1], b[E_1], E.lb[E_1] * x);
      }
      // row-internal Hillis-Steele over DPP row_shr 1/2/4/8 (uniform powers)
#define BQ_EMA_STEP(CTRL, J)                                     \
  {                                                              \
    double v[NE], r[NE];                                         \
    _Pragma("unroll") for (int e = 0; e < NE; ++e) v[e] = dpp_f64<CTRL>(b[e]); \
    pow_apply(E.wstep[J], v, r);                                 \
    _Pragma("unroll") for (int e = 0; e < NE; ++e) b[e] += r[e]; \
  }
      BQ_EMA_STEP(DPP_ROW_SHR1, 0)
      BQ_EMA_STEP(DPP_ROW_SHR2, 1)
      BQ_EMA_STEP(DPP_ROW_SHR4, 2)
      BQ_EMA_STEP(DPP_ROW_SHR8, 3)
#undef BQ_EMA_STEP
      // rows 1..3 take the carry of the rows before them: c1 = R0,
      // c2 = A^16 c1 + R1, c3 = A^16 c2 + R2, applied with A^((lane&15)+1)
      {
        double c1[NE], c2[NE], c3[NE], r[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) c1[e] = readlane_f64(b[e], 15);
        pow_apply(E.wstep[4], c1, r);
#pragma unroll
        for (int e = 0; e < NE; ++e) c2[e] = r[e] + readlane_f64(b[e], 31);
        pow_apply(E.wstep[4], c2, r);
#pragma unroll
        for (int e = 0; e < NE; ++e) c3[e] = r[e] + readlane_f64(b[e], 47);
        const int row = lane >> 4;
        if (row > 0) {
          double c[NE];
#pragma unroll
          for (int e = 0; e < NE; ++e) c[e] = row == 1 ? c1[e] : (row == 2 ? c2[e] : c3[e]);
          pow_apply(E.lane[(lane & 15) + 1], c, r);
#pragma unroll
          for (int e = 0; e < NE; ++e) b[e] += r[e];
        }
      }
      if (lane == WAVE - 1) {
#pragma unroll
        for (int e = 0; e < NE; ++e) sWe[w][e] = b[e];
      }
#pragma unroll
      for (int e = 0; e < NE; ++e) ex[e] = dpp_f64<DPP_WAVE_SHR1>(b[e]);   // lane 0 -> 0
    }
    int lpre;
    {   // last-change index + 1 (>= 0, so DPP's zero fill is the identity)
      const int inc = wave_scan_max_dpp(lcl[EN_K - 1] + 1, lane);
      if (lane == WAVE - 1) sWlc[w] = inc - 1;
      lpre = dpp_i32<DPP_WAVE_SHR1>(inc) - 1;   // lane 0 -> -1
    }
    __syncthreads();   // B1: ring, wave totals, carries visible

    // ---- phase 2: carries --------------------------------------------------------
    double wb[EN_NW];   // close-prefix base of each wave's tile slice
    {
      dd acc = {0.0, 0.0};
#pragma unroll
      for (int u = 0; u < EN_NW; ++u) {
        wb[u] = dd_round(acc);
        acc = dd_add(acc, dd{sWh[u], sWl[u]});
      }
    }
    {
      int carry = max(sLcar, lpre);
      for (int u = 0; u < w; ++u) carry = max(carry, sWlc[u]);
#pragma unroll
      for (int k = 0; k < EN_K; ++k) lcl[k] = max(lcl[k], carry);
    }
    double y[NE];
    {
      double C[NE];
#pragma unroll
      for (int e = 0; e < NE; ++e) C[e] = sEcar[e];
      for (int u = 0; u < w; ++u) {
        double r[NE];
        pow_apply(E.wave[1], C, r);
#pragma unroll
        for (int e = 0; e < NE; ++e) C[e] = r[e] + sWe[u][e];
      }
      double r[NE];
      pow_apply(E.lane[lane], C, r);
#pragma unroll
      for (int e = 0; e < NE; ++e) y[e] = ex[e] + r[e];
    }

    // ---- EMA family: exact pandas replay ---------------------------------------
    {
      double mfast[EN_K], msig[EN_K], e0[EN_K], e1[EN_K];
#pragma unroll
      for (int k = 0; k < EN_K; ++k) {
        const double x = cu.c[k];
        y[E_FAST] = ema_step<DIV>(y[E_FAST], x, E, E_FAST);
        y[E_SLOW] = ema_step<DIV>(y[E_SLOW], x, E, E_SLOW);
        y[E_SIG] = ema_step<DIV>(y[E_SIG], y[E_FAST] - y[E_SLOW], E, E_SIG);
        y[E_0] = ema_step<DIV>(y[E_0], x, E, E_0);
        y[E_1] = ema_step<DIV>(y[E_1], x, E, E_1);
        mfast[k] = y[E_FAST] - y[E_SLOW];
        msig[k] = y[E_SIG];
        e0[k] = y[E_0];
        e1[k] = y[E_1];
      }
      const bool whole = t0 + EN_TT <= T;
      if (P.out[BQ_MACD]) store4(P.out[BQ_MACD] + orow, tb, T, vout, mfast, whole);
      if (P.out[BQ_MACD_SIGNAL]) store4(P.out[BQ_MACD_SIGNAL] + orow, tb, T, vout, msig, whole);
      if (P.out[BQ_EMA_FAST]) store4(P.out[BQ_EMA_FAST] + orow, tb, T, vout, e0, whole);
      if (P.out[BQ_EMA_SLOW]) store4(P.out[BQ_EMA_SLOW] + orow, tb, T, vout, e1, whole);
    }

    // ---- rolling windows -------------------------------------------------------
    // Window start positions are at most BQ_MAX_WINDOW < 128 candles back, i.e.
    // in this wave's slice, the previous wave's slice, or (wave 0) the halo,
    // whose prefix is already based at 0.
    double wbw = wb[0], wbp = 0.0;
#pragma unroll
    for (int u = 1; u < EN_NW; ++u) {
      if (w == u) {
        wbw = wb[u];
        wbp = wb[u - 1];
      }
    }
    const int wstart = EN_H + EN_K * WAVE * w;   // first ring position of this wave's slice
    // FULL: every output of the tile has a complete window (t0 >= H > max
    // window) and the tile is complete with vector stores; drops the per-
    // element warm-up masks and the partial-tile paths.
    const bool full = t0 >= EN_H && t0 + EN_TT <= T && vout;
    auto windows = [&](auto fullc) {
      constexpr bool FULL = decltype(fullc)::value;
      const int gstart = EN_H - t0;   // ring position of candle 0 (tile 0 only)
      const int lb = pb / EN_K;
      (void)lb;
      auto warm = [&](int t, int win) { return !FULL && t < win - 1; };
      auto put = [&](double* col, const double (&x)[EN_K]) {
        if (FULL) store4(col + orow, tb, T, true, x, true);
        else store4(col + orow, tb, T, vout, x);
      };
      // close.rolling(win).mean(): prefix difference / win, or the value
      // itself on a constant window (pandas same-value rule).
      auto cmean = [&](int win, double inv, int k) -> double {
        const int t = tb + k, p = pb + k;
        if (warm(t, win)) return qnan();
        if (lcl[k] <= t - win + 1) return cu.c[k];
        const int q = p - win;
        const double base = q >= wstart ? wbw : wbp;
        return div_exact((Ploc[k] + wbw) - (sP[RS(k - win)] + base), (double)win, inv);
      };
      double res[EN_K];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (P.out[BQ_MA_FAST + i]) {
          const int win = win_of<DEF>(i == 0 ? 7 : (i == 1 ? 25 : 100), P.ma[i]);
          const double inv = P.inv_ma[i];
#pragma unroll
          for (int k = 0; k < EN_K; ++k) res[k] = cmean(win, inv, k);
          put(P.out[BQ_MA_FAST + i], res);
        }
      }
      if (P.out[BQ_BB_UPPER] || P.out[BQ_BB_MID] || P.out[BQ_BB_LOWER]) {
        // mean from the prefix; variance from sliding sums of (c - r), (c - r)^2
        // with the lane-local reference r = close at the lane's first candle.
        double up[EN_K], mid[EN_K], lo[EN_K];
        const int win = win_of<DEF>(20, P.bb_w);
        const double bk = P.bb_k, invw = P.inv_bb, invdv = P.inv_bb_dv;
        const bool okdv = win > P.bb_ddof;
        const double r = cu.c[0];
        double s1 = 0.0, s2 = 0.0;
        walk_window<DEF && FULL>(FULL ? 1 - win : max(1 - win, gstart - pb), [&](int x) {
          const double d = sC[RS(x)] - r;
          s1 += d;
          s2 = fma(d, d, s2);
        });
#pragma unroll
        for (int k = 0; k < EN_K; ++k) {
          const int t = tb + k, p = pb + k;
          if (k > 0) {
            const double dn = cu.c[k] - r;
            const double dol = (FULL || p - win >= gstart) ? sC[RS(k - win)] - r : 0.0;
            s1 = (s1 + dn) - dol;
            s2 = fma(-dol, dol, fma(dn, dn, s2));
          }
          const double m = cmean(win, invw, k);
          double sd;
          if (warm(t, win) || !okdv) sd = qnan();
          else if (lcl[k] <= t - win + 1) sd = 0.0;
          else {
            const double var = (s2 - s1 * s1 * invw) * invdv;
            sd = sqrt_nr(var);
          }
          mid[k] = m;
          up[k] = m + bk * sd;
          lo[k] = m - bk * sd;
        }
        if (P.out[BQ_BB_UPPER]) put(P.out[BQ_BB_UPPER], up);
        if (P.out[BQ_BB_MID]) put(P.out[BQ_BB_MID], mid);
        if (P.out[BQ_BB_LOWER]) put(P.out[BQ_BB_LOWER], lo);
      }
      if (P.out[BQ_RSI]) {
        // SMA-RSI = 100 * mean(gain) / (mean(gain) + mean(loss)) with
        // sum(gain) + sum(loss) = A = sum|d| and sum(gain) - sum(loss) = D =
        // c_t - c_{t-w} (telescoping): RSI = 50 (1 + D / A). Counts of up
        // and down moves make the all-gain (100), all-loss (0) and flat (NaN)
        // windows exact. d of candle 0 is NaN -> contributes nothing.
        const int win = win_of<DEF>(14, P.rsi_w);
        double A = 0.0, prev = sC[RS(-win)];
        int nup = 0, ndn = 0;
        walk_window<DEF>(1 - win, [&](int x) {
          const double c = sC[RS(x)], d = c - prev;
          A += fmax(fabs(d), 0.0);   // fmax drops the NaN of candle 0
          nup += d > 0.0;
          ndn += d < 0.0;
          prev = c;
        });
#pragma unroll
        for (int k = 0; k < EN_K; ++k) {
          const int t = tb + k, p = pb + k;
          if (k > 0) {
            const double d = cu.c[k] - cu.c[k - 1];
            const double dold = sC[RS(k - win)] - sC[RS(k - win - 1)];
            A = (A + fabs(d)) - fmax(fabs(dold), 0.0);
            nup += (d > 0.0) - (dold > 0.0);
            ndn += (d < 0.0) - (dold < 0.0);
          }
          if (warm(t, win)) {
            res[k] = qnan();
            continue;
          }
          const double D = cu.c[k] - sC[FULL ? RS(k - win) : (p - win >= gstart ? RS(k - win) : LX(gstart))];
          double v;
          if (nup == 0 && ndn == 0) v = qnan();
          else if (ndn == 0) v = 100.0;
          else if (nup == 0) v = 0.0;
          else v = 50.0 * (1.0 + D / A);
          res[k] = v;
        }
        put(P.out[BQ_RSI], res);
      }
      // sliding mean of a per-candle ring array with the same-value rule
      auto smean = [&](const double* Q, int defw, int win_, double inv, bool nonneg) {
        const int win = win_of<DEF>(defw, win_);
        const double wd = (double)win;
        double sum = 0.0, pq = qnan();
        int run = 0;
        walk_window<DEF>(1 - win, [&](int x) {
          const double q = Q[RS(x)];
          sum += q;
          run = q == pq ? run + 1 : 1;
          pq = q;
        });
#pragma unroll
        for (int k = 0; k < EN_K; ++k) {
          const int t = tb + k;
          if (k > 0) {
            const double q = Q[RS(k)];
            sum = (sum + q) - Q[RS(k - win)];
            run = q == pq ? run + 1 : 1;
            pq = q;
          }
          if (warm(t, win)) res[k] = qnan();
          else if (run >= win) res[k] = pq;
          else res[k] = div_exact(nonneg && sum < 0.0 ? 0.0 : sum, wd, inv);
        }
      };
      if (P.out[BQ_ATR]) {
        smean(sTR, 14, P.atr_w, P.inv_atr, true);
        put(P.out[BQ_ATR], res);
      }
      if (P.out[BQ_TWAP]) {
        smean(sO4, 12, P.twap_w, P.inv_twap, false);
        put(P.out[BQ_TWAP], res);
      }
      if (P.out[BQ_MFI]) {
        // MFI = 100 pos / (pos + neg) with pos + neg = B = sum|f| and
        // pos - neg = F = sum f (f = signed flow): MFI = 50 (1 + F / B);
        // counts of up/down flows make the one-sided and empty windows exact.
        const int win = win_of<DEF>(14, P.mfi_w);
        double B = 0.0, F = 0.0;
        int nup = 0, ndn = 0;
        walk_window<DEF>(1 - win, [&](int x) {
          const double f = sMF[RS(x)];
          B += fabs(f);
          F += f;
          nup += f > 0.0;
          ndn += f < 0.0;
        });
#pragma unroll
        for (int k = 0; k < EN_K; ++k) {
          const int t = tb + k;
          if (k > 0) {
            const double f = sMF[RS(k)], fo = sMF[RS(k - win)];
            B = (B + fabs(f)) - fabs(fo);
            F = (F + f) - fo;
            nup += (f > 0.0) - (fo > 0.0);
            ndn += (f < 0.0) - (fo < 0.0);
          }
          double v;
          if (warm(t, win) || (nup == 0 && ndn == 0)) v = qnan();
          else if (ndn == 0) v = 100.0;
          else if (nup == 0) v = 0.0;
          else v = 50.0 * (1.0 + F / B);
          res[k] = v;
        }
        put(P.out[BQ_MFI], res);
      }
    };
    if (full) windows(std::true_type{});
    else windows(std::false_type{});

    if (t0 + EN_TT >= T) break;
    __syncthreads();   // B2: every read of this tile's ring is done

    // ---- halo for the next tile: owners of ring positions [TT, R) copy them --
    {
      const double plast = __shfl(Ploc[EN_K - 1], WAVE - 1, WAVE);   // last wave, lane 63
      if (pb >= EN_TT) {
#pragma unroll
        for (int k = 0; k < EN_K; ++k) {
          sP[RS1(k - EN_TT)] = Ploc[k] - plast;   // re-based: halo prefix ends at 0
          sC[RS1(k - EN_TT)] = sC[RS1(k)];
          sTR[RS1(k - EN_TT)] = sTR[RS1(k)];
          sO4[RS1(k - EN_TT)] = sO4[RS1(k)];
          sMF[RS1(k - EN_TT)] = sMF[RS1(k)];
        }
      }
      if (tid == EN_NT - 1) {
#pragma unroll
        for (int e = 0; e < NE; ++e) sEcar[e] = y[e];
        sLcar = lcl[EN_K - 1];
      }
    }
  }
  __syncthreads();   // sMiss final; orders the walk's stores before a rewrite's
  if (sMiss) enrich_row_missing(sA, E, irow, orow, sC, sP, sTR, sO4, sMF);
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

const char* bq_version(void) { return "binquant_amd 0.2.0 (gfx950)"; }

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
  if (!in || !out || S < 0 || T < 0 || ld_in < T || ld_out < T || T > (int64_t)0x7fffffff - 2 * EN_TT ||
      S > 0x7fffffff)
    return BQ_EINVAL;
  bq_params dp;
  if (!params) {
    bq_default_params(&dp);
    params = &dp;
  }
  const bq_params& P = *params;
  for (int i = 0; i < 3; ++i)
    if (!window_ok(P.ma_periods[i])) return BQ_EINVAL;
  if (!window_ok(P.rsi_window) || !window_ok(P.bb_window) || !window_ok(P.atr_window) ||
      !window_ok(P.twap_window) || !window_ok(P.mfi_window) || P.bb_ddof < 0 || P.macd_fast < 1 ||
      P.macd_slow < 1 || P.macd_signal < 1 || P.ema_spans[0] < 1 || P.ema_spans[1] < 1)
    return BQ_EINVAL;
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
  if (S == 0 || T == 0 || !any_out) return BQ_OK;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.S = S;
  A.swz = 1;
  {   // a prime multiplier coprime to S: b -> (b * swz) % S is a permutation
    auto gcd = [](int64_t a, int64_t b) {
      while (b) {
        const int64_t t = a % b;
        a = b;
        b = t;
      }
      return a;
    };
    const int64_t primes[] = {7919, 7927, 7933, 7937, 7949, 104729};
    for (int64_t p : primes)
      if (S > 1 && gcd(p % S, S) == 1) {
        A.swz = p % S;
        break;
      }
  }
  for (int i = 0; i < 3; ++i) A.ma[i] = P.ma_periods[i];
  A.rsi_w = P.rsi_window;
  A.bb_w = P.bb_window;
  A.bb_ddof = P.bb_ddof;
  A.atr_w = P.atr_window;
  A.twap_w = P.twap_window;
  A.mfi_w = P.mfi_window;
  A.bb_k = P.bb_k;
  for (int i = 0; i < 3; ++i) A.inv_ma[i] = 1.0 / (double)P.ma_periods[i];
  A.inv_rsi = 1.0 / (double)P.rsi_window;
  A.inv_bb = 1.0 / (double)P.bb_window;
  A.inv_bb_dv = P.bb_window > P.bb_ddof ? 1.0 / (double)(P.bb_window - P.bb_ddof) : 0.0;
  A.inv_atr = 1.0 / (double)P.atr_window;
  A.inv_twap = 1.0 / (double)P.twap_window;
  A.span[E_FAST] = P.macd_fast;
  A.span[E_SLOW] = P.macd_slow;
  A.span[E_SIG] = P.macd_signal;
  A.span[E_0] = P.ema_spans[0];
  A.span[E_1] = P.ema_spans[1];
  A.ema = ema_consts(A.span);

  // 16-byte vector access needs every row start 16-byte aligned.
  auto aligned = [](const void* p) { return (((uintptr_t)p) & 15u) == 0; };
  int vin = (ld_in % 2) == 0;
  for (int i = 0; i < BQ_NUM_INPUTS; ++i) vin &= aligned(in[i]);
  int vout = (ld_out % 2) == 0;
  for (int i = 0; i < BQ_NUM_ENRICH_COLS; ++i)
    if (out[i]) vout &= aligned(out[i]);

  // does any EMA need the explicit `/ (old_wt + new_wt)` (non-unit sum)?
  bool div = false;
  for (int e = 0; e < NE; ++e) {
    const double com = ((double)A.span[e] - 1.0) / 2.0;
    const double al = 1.0 / (1.0 + com);
    div |= ((1.0 - al) + al) != 1.0;
  }
  const dim3 grid((unsigned)S), block(EN_NT);
  hipStream_t st = (hipStream_t)stream;
  const bool def = P.ma_periods[0] == 7 && P.ma_periods[1] == 25 && P.ma_periods[2] == 100 && P.rsi_window == 14 &&
                   P.bb_window == 20 && P.atr_window == 14 && P.twap_window == 12 && P.mfi_window == 14;
#define BQ_EN_LAUNCH(D, V, F) hipLaunchKernelGGL((enrich_kernel<D, V, F>), grid, block, 0, st, A, vin)
  if (def) {
    if (div && vout) BQ_EN_LAUNCH(true, true, true);
    else if (div) BQ_EN_LAUNCH(true, false, true);
    else if (vout) BQ_EN_LAUNCH(false, true, true);
    else BQ_EN_LAUNCH(false, false, true);
  } else {
    if (div && vout) BQ_EN_LAUNCH(true, true, false);
    else if (div) BQ_EN_LAUNCH(true, false, false);
    else if (vout) BQ_EN_LAUNCH(false, true, false);
    else BQ_EN_LAUNCH(false, false, false);
  }
#undef BQ_EN_LAUNCH
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
