// Rolling-window statistics with pandas semantics, for the strategy feature
// pipelines:
//
//   bq_rolling: x.shift(shift).rolling(window, min_periods).<mode>()
//     mean / sum / var / std (ddof 1 or 0): pandas' own window recurrences
//       REPLAYED over the whole row (pandas/_libs/window/aggregations.pyx,
//       2.3.3): roll_sum / roll_mean keep a Kahan sum with separate add and
//       remove compensations, the signbit count (mean clamps) and the
//       same-value run (result = the value / value * nobs); roll_var a
//       compensated Welford mean + ssqdm with the same-value rule -> 0. Each
//       step removes the leaving value, then adds the entering one. The
//       outputs therefore equal pandas' bit for bit (restatement pinned in
//       tests/test_oracle_golden.py; kernels in tests/test_strategies_gpu.py).
//     quantile(q) (linear interpolation), median (roll_median_c), and
//       max / min (q = 1 / 0): order statistics of the window's non-NaN
//       values — a pure function of the window multiset, so any algorithm
//       that selects the same ranks is exact.
//     Used by ActivityBurstPump.compute_indicators
//     (strategies/activity_burst_pump.py:58-63 median(19), :134-139
//     quantile(0.92, 80), :147-152 max(3)), LiquidationSweepPump.compute_pump_score
//     (strategies/liquidation_sweep_pump.py:218-245: mean(20), max/min(6),
//     quantile(0.80, 48)), FailedSpikeFade (quantile(0.85, 60), rolling
//     mean/std(12, 8, 20, 10), sums(2, 3, 5)).
//
//   bq_ewm: x.ewm(alpha, adjust=False, min_periods).mean() with
//           ignore_na=False NaN gaps (the BTC left-merge of
//           liquidation_sweep_pump.py:255-267 and the Wilder ATR/RSI of
//           :215-217 and mean_reversion_fade.py:88-109) — pandas' exact
//           recursion, bit for bit.
//
// Mappings (both HBM-friendly; no lane walks memory on its own):
//   replay (mean/sum/var/std, ewm): lane = symbol, one wave per 64 symbols.
//     Chunks of RP_CT candles are read coalesced (RP_CT lanes cover one
//     symbol's contiguous bytes), transposed through LDS, and the next chunk
//     is in flight while the current one is replayed; results leave through
//     an LDS tile as coalesced row segments. The staged chunks stay in an
//     LDS ring covering window + shift, so the value leaving the window is
//     an LDS read and every input byte crosses HBM once.
//   rank (quantile/median/max/min), two kernels chosen by window and shape:
//     tile: wave = 64 (w <= 65) or 128 consecutive outputs of one symbol; the
//       union of their windows is sorted once per wave (bitonic, registers +
//       lane shuffles) and each lane walks it counting its window's members
//       up to the ranks it needs. No per-lane state along the row, so no
//       warm-up: S * T / 64 waves at any shape.
//     lane: lane = (symbol, segment of the row). Each lane keeps its window
//       SORTED IN REGISTERS (W slots, +inf padding): a removal / insertion is
//       a branch-free pass of compares and selects over the W slots. A
//       segment first rebuilds its window from the w values before it; cheap
//       for short windows on large panels.
#include "bq_device.h"
#include "bq_panel.h"
#include "binquant_amd.h"

#include <stdlib.h>
#include <type_traits>
#include <string.h>

namespace bq {

constexpr int RW_MAXW = BQ_MAX_ROLLING_WINDOW;
constexpr int RW_MAXSHIFT = 32;

constexpr int RW_MAXJOBS = BQ_MAX_ROLL_JOBS;

// one series of a batch (bq_roll_job); jobs of one launch share [S][T]
struct RollJob {
  const double* x;
  double* out;
  int64_t ld_in, ld_out;
  int win, minp, shift, mode, seg, nseg;
  int lower;   // BQ_ROLL_QLOWER: the quantile's lower order statistic, no interpolation
  double q, alpha;
  int64_t rows;   // this job's rows (<= the batch's S; a benchmark row beside a panel)
  uint8_t* cross;    // slide kernel only (bq_rolling_quantile_cross): NULL, or [S][ld_cross]
  int64_t ld_cross;  // (x[t] >= out[t]) & (x[t-1] < out[t-1])
};

struct RollBatch {
  RollJob j[RW_MAXJOBS];
  int64_t S;
  int T;
};

// ---- replay kernels (lane = symbol) --------------------------------------------------
constexpr int RP_CT = 16;

// pandas roll_sum / roll_mean / roll_var state, updated value by value
struct Moments {
  double sum, c_add, c_rem;     // Kahan sum (separate compensations)
  double vn, mean, ssq, v_add, v_rem;   // Welford (nobs as float64, as pandas)
  double prev;
  int nobs, neg, same;
  __device__ __forceinline__ void init(double first) {
    sum = c_add = c_rem = 0.0;
    vn = mean = ssq = v_add = v_rem = 0.0;
    prev = first;
    nobs = neg = same = 0;
  }
  // Straight-line updates: every candidate value is formed and the state
  // takes it by select where v is observed (a missing v leaves the state as
  // it is, as pandas' `if val == val` does). Branches here split a replay
  // step into a dozen basic blocks with their exec-mask bookkeeping; the
  // values are those of the branchy form bit for bit.
  __device__ __forceinline__ void add(double v, bool welford) {
    const bool ok = win_ok(v);   // NaN and +-inf are missing (pandas' window ops); v is used only under ok
    nobs += ok ? 1 : 0;
    if (welford) {
      const double vn1 = vn + 1.0;
      const double pm = mean - v_add;
      const double y = v - v_add;
      const double t = y - mean;
      const double va = t + mean - y;
      const double m1 = vn1 != 0.0 ? mean + t / vn1 : 0.0;
      const double s1 = ssq + (v - pm) * (v - m1);
      vn = ok ? vn1 : vn;
      v_add = ok ? va : v_add;
      mean = ok ? m1 : mean;
      ssq = ok ? s1 : ssq;
    } else {
      const double y = v - c_add;
      const double t = sum + y;
      const double ca = t - sum - y;
      c_add = ok ? ca : c_add;
      sum = ok ? t : sum;
      neg += (ok && signbit(v)) ? 1 : 0;
    }
    same = ok ? ((v == prev) ? same + 1 : 1) : same;
    prev = ok ? v : prev;
  }
  __device__ __forceinline__ void remove(double v, bool welford) {
    const bool ok = win_ok(v);
    nobs -= ok ? 1 : 0;
    if (welford) {
      const double vn1 = vn - 1.0;
      const bool live = vn1 != 0.0;
      const double pm = mean - v_rem;
      const double y = v - v_rem;
      const double t = y - mean;
      const double vr = t + mean - y;
      const double m1 = mean - t / vn1;
      const double s1 = ssq - (v - pm) * (v - m1);
      vn = ok ? vn1 : vn;
      v_rem = ok && live ? vr : v_rem;
      mean = ok ? (live ? m1 : 0.0) : mean;
      ssq = ok ? (live ? s1 : 0.0) : ssq;
    } else {
      const double y = -v - c_rem;
      const double t = sum + y;
      const double cr = t - sum - y;
      c_rem = ok ? cr : c_rem;
      sum = ok ? t : sum;
      neg -= (ok && signbit(v)) ? 1 : 0;
    }
  }
  // calc_sum / calc_mean / calc_var as select chains (every candidate formed;
  // the class is a compile-time constant at the replays' call sites)
  __device__ __forceinline__ double result(int mode, int minp, bool welford) const {
    if (!welford) {
      const double dn = (double)nobs;
      if (mode == BQ_ROLL_SUM) {   // calc_sum
        double r = same >= nobs ? prev * dn : sum;
        r = nobs < minp ? qnan() : r;
        return (nobs == 0 && minp == 0) ? 0.0 : r;
      }
      // calc_mean
      double r = sum / dn;
      r = (neg == nobs && r > 0.0) ? 0.0 : r;
      r = (neg == 0 && r < 0.0) ? 0.0 : r;
      r = same >= nobs ? prev : r;
      return (nobs < minp || nobs <= 0) ? qnan() : r;
    }
    // calc_var (ddof 1 or 0), std = sqrt
    const double ddof = (mode == BQ_ROLL_VAR || mode == BQ_ROLL_STD) ? 1.0 : 0.0;
    double r = ssq / (vn - ddof);
    r = r < 0.0 ? 0.0 : r;
    r = (vn == 1.0 || (double)same >= vn) ? 0.0 : r;
    r = (vn >= (double)minp && vn > ddof) ? r : qnan();
    return (mode == BQ_ROLL_STD || mode == BQ_ROLL_STD0) ? sqrt(r) : r;
  }
};

__host__ __device__ __forceinline__ int replay_class(int mode) {
  return mode == BQ_ROLL_FFILL ? 3 : mode == BQ_ROLL_EWM ? 0 : mode >= BQ_ROLL_VAR ? 2 : 1;
}

// one lane's replay state: pandas' window recurrences (Moments) or the ewm
// recursion (adjust=False, ignore_na=False), advanced one candle per call
struct ReplayLane {
  Moments m;
  double weighted, old_wt;
  int nobs;
  __device__ __forceinline__ void init() {
    m.init(0.0);
    weighted = qnan();
    old_wt = 1.0;
    nobs = 0;
  }
  // v_in = x[t - shift] (NaN before the row), v_out = x[t - shift - w]
  // steady: t >= window + shift + 1 (no first candle, the leaving value is
  // always inside the row) — lets a caller drop the per-step checks
  __device__ __forceinline__ double step(const RollJob& A, bool EWM, bool welford, int t, double v_in, double v_out,
                                         bool FFILL = false, bool steady = false) {
    if (FFILL) {   // last observation carried forward (weighted holds it; infinities are values)
      if (v_in == v_in) weighted = v_in;
      return weighted;
    }
    // window operations: NaN and +-inf are missing (every use of v_in / v_out
    // below is under its observation flag)
    if (EWM) {   // straight-line, as Moments (selects, the same values)
      const double alpha = A.alpha, om = 1.0 - alpha;
      const bool obs = win_ok(v_in);
      const bool wv = weighted == weighted;
      const double ow = wv ? old_wt * om : old_wt;
      const double nw = (ow * weighted + alpha * v_in) / (ow + alpha);
      double w2 = (wv && obs && weighted != v_in) ? nw : weighted;
      w2 = (!wv && obs) ? v_in : w2;
      const bool first = !steady && t == 0;
      weighted = first ? (obs ? v_in : qnan()) : w2;
      old_wt = first ? old_wt : ((wv && obs) ? 1.0 : ow);
      nobs = first ? (obs ? 1 : 0) : nobs + (obs ? 1 : 0);
      return nobs >= A.minp ? weighted : qnan();
    }
    if (!steady && t == 0) m.init(win_val(v_in));   // pandas: prev_value = first value of the series
    if (steady || (t >= A.win && t - A.shift - A.win >= 0)) m.remove(v_out, welford);
    m.add(v_in, welford);
    return m.result(A.mode, A.minp, welford);
  }
};

// LDS: a ring of the last `ring` input chunks (RL = ring * RP_CT candles per
// lane, lane-interleaved); the ring covers window + shift, so the leaving
// value is an LDS read and every input byte crosses HBM once. Results go
// straight from each lane to its row (consecutive steps fill a cache line
// in L2 before it is written back).
__global__ __launch_bounds__(WAVE) void replay_kernel(const RollBatch B, int ring) {
  const RollJob& A = B.j[blockIdx.y];   // wave-uniform: scalar kernarg loads
  const bool FFILL = A.mode == BQ_ROLL_FFILL;
  const bool EWM = A.mode == BQ_ROLL_EWM || FFILL;   // no leaving value
  extern __shared__ double smem[];
  constexpr int TILE = RP_CT * STG_PITCH;
  const int RL = ring * RP_CT;
  const int lane = threadIdx.x;
  const int64_t sym0 = (int64_t)blockIdx.x * WAVE;
  const int64_t S = A.rows;
  if (sym0 >= S) return;   // the block is one wave: a uniform exit
  const int T = B.T, w = A.win, sh = A.shift;
  const bool welford = A.mode >= BQ_ROLL_VAR;
  const bool live = sym0 + lane < S;
  double* __restrict__ orow = A.out + (live ? sym0 + lane : 0) * A.ld_out;
  // ring positions of the entering (t - sh) and leaving (t - sh - w) values,
  // advanced by one per step (no division in the loop)
  auto wrap = [&](int i) { return ((i % RL) + RL) % RL; };
  int pin = wrap(-sh), pout = wrap(-sh - w);
  double ri[RP_CT];
  stage_load<RP_CT>(A.x, A.ld_in, sym0, S, 0, T, lane, ri);
  ReplayLane st;
  st.init();
  for (int t0 = 0; t0 < T; t0 += RP_CT) {
    stage_put<RP_CT>(smem + ((t0 / RP_CT) % ring) * TILE, lane, ri);
    __syncthreads();
    if (t0 + RP_CT < T)   // next chunk in flight during this one's replay
      stage_load<RP_CT>(A.x, A.ld_in, sym0, S, t0 + RP_CT, T, lane, ri);
    auto step = [&](int j) {
      const int t = t0 + j;
      const double v_in = t - sh < 0 ? qnan() : smem[pin * STG_PITCH + lane];
      const double v_out = EWM ? 0.0 : smem[pout * STG_PITCH + lane];
      pin = pin + 1 == RL ? 0 : pin + 1;
      pout = pout + 1 == RL ? 0 : pout + 1;
      const double res = st.step(A, EWM, welford, t, v_in, v_out, FFILL);
      if (live) orow[t] = res;
    };
    if (t0 + RP_CT <= T) {
      // full chunk: unrolled, so each step's result / LDS traffic overlaps
      // the next step's (short) dependent state update
#pragma unroll
      for (int j = 0; j < RP_CT; ++j) step(j);
    } else {
      for (int j = 0; j < T - t0; ++j) step(j);
    }
    __syncthreads();   // the ring slot of this chunk is reused RL candles later
  }
}

// Same replay with a fixed 2-tile LDS footprint (≈17 KB per wave instead of
// the ring's ceil((w + shift) / 16) + 1 tiles, up to 59 KB at w = 80): the
// leaving values are staged from the input again (chunk t0 - shift - w, an
// L2 / MALL hit: it was read w candles earlier), so up to 9 waves per CU fit
// instead of 2-6. Costs one more read of the input (from cache).
// CLS: 0 = ewm, 1 = Kahan sum / mean, 2 = Welford var / std, 3 = ffill — the
// body is specialised per class (shorter dependent chain per step, and a
// per-class launch keeps the registers to that class's state).
// SPW: symbols per wave (64; 32, 16, 8 for measurement). With SPW < 64 the
// same rows spread over 64/SPW times as many waves (lanes >= SPW only help
// stage; each chunk is RS_V * 64 / SPW candles long). Measured: no faster —
// a 12.5k-symbol replay (196 waves) costs ~600 cycles per step in the wave's
// own ~100-instruction stream (NaN guards, the same-value rule, the IEEE
// divide of the mean), not in a shortage of waves.
// staged values per lane and chunk: 16 for the class kernels, 8 for the
// all-classes kernel (its register footprint then allows 2 waves per SIMD
// instead of 1; measured an A/B harness of rounds 1-2 (tools/pipe_ab.sh, removed in round 3: git history): failed-spike replay 3.6 -> 3.2 ms,
// while the class kernels are faster with 16)
#ifndef BQ_RS_V
#define BQ_RS_V 16
#endif
#ifndef BQ_RS_V_MIXED
#define BQ_RS_V_MIXED 8
#endif
#ifndef BQ_RS_STAGE_OUT
#define BQ_RS_STAGE_OUT 1   // results leave through LDS as coalesced row segments
#endif
#ifndef BQ_RS_WPS
#define BQ_RS_WPS 1   // min waves per SIMD (register cap) of the re-staging replays: 1 wave, no spill (see
                      // launch_restage: ~1 wave per SIMD at panel sizes; 2 spilled 26 VGPRs of the Welford class)
#endif
#ifndef BQ_RS_LPT
#define BQ_RS_LPT 1   // mixed replay batches ordered longest class first
#endif
#ifndef BQ_RS_WPS_MIXED
#define BQ_RS_WPS_MIXED 2   // the all-classes kernel
#endif

template <int SPW, int RS_V>
struct ReplayTile {
  static constexpr int CT = RS_V * WAVE / SPW;   // candles per chunk
  static constexpr int P = SPW + 2;           // LDS pitch (doubles) of one candle's row
  static constexpr int N = CT * P;
  // [SPW symbols][CT candles] of rows sym0.. from column t0, read so that
  // consecutive lanes read consecutive candles of one row
  __device__ __forceinline__ static void load(const double* __restrict__ base, int64_t ld, int64_t sym0, int64_t S,
                                              int t0, int T, int lane, double (&r)[RS_V]) {
// Every lane loads (a clamped, valid address) and selects NaN outside the
  // panel: no branch around a load, so no load forces a full vmcnt drain.
#pragma unroll
    for (int k = 0; k < RS_V; ++k) {
      const int e = lane + WAVE * k;
      const int64_t s = sym0 + e / CT;
      const int t = t0 + e % CT;
      const int64_t sc = s < S ? s : S - 1;
      const int tc = t < 0 ? 0 : t < T ? t : T - 1;
      const double v = base[sc * ld + tc];
      r[k] = (s < S && t >= 0 && t < T) ? v : qnan();
    }
  }
  // interior chunk (rows sym0 .. sym0 + SPW - 1 all < S, candles t .. t + CT - 1
  // all inside the row): buffer loads at a per-lane offset fixed for the whole
  // walk plus a per-k scalar row step — no per-element address arithmetic or
  // range selects (the general form above handles the edges)
  static constexpr bool FAST = CT <= WAVE;
  __device__ __forceinline__ static void load_fast(__amdgpu_buffer_rsrc_t rs, unsigned loff, unsigned rowstep,
                                                   int t, double (&r)[RS_V]) {
    const unsigned v = loff + (unsigned)t * (unsigned)sizeof(double);
#pragma unroll
    for (int k = 0; k < RS_V; ++k)
      r[k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, v, (unsigned)k * rowstep, 0));
  }
  // transposed into LDS: lds[candle * P + symbol]
  __device__ __forceinline__ static void put(double* lds, int lane, const double (&r)[RS_V]) {
#pragma unroll
    for (int k = 0; k < RS_V; ++k) {
      const int e = lane + WAVE * k;
      lds[(e % CT) * P + e / CT] = r[k];
    }
  }
};

// Results leave through one buffer store per step, issued by every lane:
// rows past S and lanes >= SPW get an offset past the descriptor's range,
// which the hardware drops. Unconditional stores keep the loop's waits
// counted (vmcnt(N) for the prefetched chunk) instead of draining every
// outstanding result store at each chunk boundary (gfx950's vmcnt counts
// loads and stores alike). Host guarantees 64 * ld_out * 8 < 2^31 (job_ok).
template <int CLS, int SPW, int RS_V>
__device__ __forceinline__ void replay_restage_body(const RollJob& A, const RollBatch& B, double* s_in,
                                                    double* s_out) {
  using Tl = ReplayTile<SPW, RS_V>;
  constexpr int CT = Tl::CT;
  constexpr bool FFILL = CLS == 3;
  constexpr bool EWM = CLS == 0 || FFILL;   // no leaving value
  constexpr bool welford = CLS == 2;
  const int lane = threadIdx.x;
  const int64_t sym0 = (int64_t)blockIdx.x * SPW;
  const int64_t S = A.rows;
  if (sym0 >= S) return;   // the block is one wave: a uniform exit
  const int T = B.T, w = A.win, sh = A.shift;
  const int64_t rows = S - sym0 < SPW ? S - sym0 : SPW;
  const int nbytes = (int)(rows * A.ld_out * (int64_t)sizeof(double));
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc(A.out + sym0 * A.ld_out, 0, nbytes, 0x00020000);
  const bool live = lane < rows;
  const unsigned obase = live ? (unsigned)(lane * A.ld_out * (int64_t)sizeof(double)) : (unsigned)nbytes;
  const int rl = lane < SPW ? lane : SPW - 1;   // lanes >= SPW replay a copy (stores dropped)
  double ri[RS_V], ro[RS_V];
  Tl::load(A.x, A.ld_in, sym0, S, -sh, T, lane, ri);
  if (!EWM) Tl::load(A.x, A.ld_in, sym0, S, -sh - w, T, lane, ro);
  ReplayLane st;
  st.init();
  auto step = [&](int t, double v_in, double v_out, auto steady) {
    const double res = st.step(A, EWM, welford, t, v_in, v_out, FFILL, decltype(steady)::value);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(bq_u32x2, res), orsrc,
                                          obase + (unsigned)t * (unsigned)sizeof(double), 0, 0);
  };
  // full chunks (CT <= 64): a step's result goes into the LDS slot its input
  // came from (already read by this lane), and the chunk leaves through
  // coalesced row segments after its last step — one store instruction then
  // covers 64 / CT rows x CT candles instead of 64 rows x 1 candle
  constexpr bool OUT_LDS = Tl::FAST && BQ_RS_STAGE_OUT;
  auto step_lds = [&](int t, int j, double v_in, double v_out, auto steady) {
    s_in[j * Tl::P + rl] = st.step(A, EWM, welford, t, v_in, v_out, FFILL, decltype(steady)::value);
  };
  // 16 steps at a time: their LDS operands are read into registers first, so
  // no LDS latency sits between two dependent state updates
  constexpr int G = CT < 16 ? CT : 16;
  auto steps16 = [&](int t0, int g, auto steady) {
    double vi[G], vo[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      vi[k] = s_in[(g + k) * Tl::P + rl];
      vo[k] = EWM ? 0.0 : s_out[(g + k) * Tl::P + rl];
    }
#pragma unroll
    for (int k = 0; k < G; ++k) {
      if (OUT_LDS) step_lds(t0 + g + k, g + k, vi[k], vo[k], steady);
      else step(t0 + g + k, vi[k], vo[k], steady);
    }
  };
  // the chunk's results, transposed back out of LDS: element e = lane + 64k is
  // row e / CT, candle e % CT; rows past S fall outside the descriptor
  const unsigned ooff = (unsigned)(((lane / CT) * A.ld_out + lane % CT) * (int64_t)sizeof(double));
  const unsigned orowstep = (unsigned)((WAVE / CT) * A.ld_out * (int64_t)sizeof(double));
  auto flush = [&](int t0) {
    const unsigned v = ooff + (unsigned)t0 * (unsigned)sizeof(double);
#pragma unroll
    for (int k = 0; k < RS_V; ++k) {
      const int e = lane + WAVE * k;
      const double r = s_in[(e % CT) * Tl::P + e / CT];
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(bq_u32x2, r), orsrc, v, (unsigned)k * orowstep, 0);
    }
  };
  // input rows as one buffer (interior chunks load through it)
  const bool rows_full = rows == SPW && A.ld_in <= BQ_MAX_ROLL_LD;
  const __amdgpu_buffer_rsrc_t irsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(A.x) + sym0 * A.ld_in, 0, rows_full ? (int)(SPW * A.ld_in * (int64_t)sizeof(double)) : 0,
      0x00020000);
  const unsigned loff = (unsigned)(((lane / CT) * A.ld_in + lane % CT) * (int64_t)sizeof(double));
  const unsigned rowstep = (unsigned)((WAVE / CT) * A.ld_in * (int64_t)sizeof(double));
  auto stage = [&](int t, double (&r)[RS_V]) {
    if (Tl::FAST && rows_full && t >= 0 && t + CT <= T) Tl::load_fast(irsrc, loff, rowstep, t, r);
    else Tl::load(A.x, A.ld_in, sym0, S, t, T, lane, r);
  };
  const int tfull = T - T % CT;
  int t0 = 0;
  for (; t0 < tfull; t0 += CT) {
    Tl::put(s_in, lane, ri);
    if (!EWM) Tl::put(s_out, lane, ro);
    __syncthreads();
    // next chunks in flight during this one's replay (past T: NaN, unused)
    stage(t0 + CT - sh, ri);
    if (!EWM) stage(t0 + CT - sh - w, ro);
    if (t0 >= w + sh + 1) {   // every step of the chunk is steady
#pragma unroll 1
      for (int g = 0; g < CT; g += G) steps16(t0, g, std::true_type{});
    } else {
#pragma unroll 1
      for (int g = 0; g < CT; g += G) steps16(t0, g, std::false_type{});
    }
    if (OUT_LDS) {
      __syncthreads();   // the chunk's results are in s_in
      flush(t0);
    }
    __syncthreads();   // both tiles are rewritten by the next chunk
  }
  if (t0 < T) {   // tail chunk
    Tl::put(s_in, lane, ri);
    if (!EWM) Tl::put(s_out, lane, ro);
    __syncthreads();
    for (int j = 0; j < T - t0; ++j)
      step(t0 + j, s_in[j * Tl::P + rl], EWM ? 0.0 : s_out[j * Tl::P + rl], std::false_type{});
  }
}

// every job of the batch is of class CLS
// (the job is copied out of the kernel arguments once: read through a
// reference, its fields are re-loaded from memory at every step)
template <int CLS, int SPW>
__global__ __launch_bounds__(WAVE, BQ_RS_WPS) void replay_restage_kernel(const RollBatch B) {
  __shared__ double s_in[ReplayTile<SPW, BQ_RS_V>::N];
  __shared__ double s_out[ReplayTile<SPW, BQ_RS_V>::N];
  const RollJob A = B.j[blockIdx.y];
  replay_restage_body<CLS, SPW, BQ_RS_V>(A, B, s_in, s_out);
}

// jobs of any class in one launch (wave-uniform switch on the job's class):
// for batches that do not fill the chip, where per-class launches would run
// one latency-bound replay after the other
template <int SPW>
__global__ __launch_bounds__(WAVE, BQ_RS_WPS_MIXED) void replay_mixed_kernel(const RollBatch B) {
  constexpr int V = SPW >= 16 ? BQ_RS_V_MIXED : BQ_RS_V;   // chunks of >= 8 candles for SPW < 16
  __shared__ double s_in[ReplayTile<SPW, V>::N];
  __shared__ double s_out[ReplayTile<SPW, V>::N];
  const RollJob A = B.j[blockIdx.y];
  switch (replay_class(A.mode)) {
    case 0: replay_restage_body<0, SPW, V>(A, B, s_in, s_out); break;
    case 1: replay_restage_body<1, SPW, V>(A, B, s_in, s_out); break;
    case 2: replay_restage_body<2, SPW, V>(A, B, s_in, s_out); break;
    default: replay_restage_body<3, SPW, V>(A, B, s_in, s_out);
  }
}

// ---- forward fill as a scan (x.ffill(): exact copies, any order) -------------------
// One 256-thread block per (row, job) walks tiles of 1024 candles (4 per
// lane): the last valid index before each lane comes from a block max-scan
// (DPP within the wave, wave totals through LDS), its value from the tile in
// LDS or the carry of the previous tiles; each lane then fills its 4 candles.
// A fill only copies values, so the result equals the sequential replay bit
// for bit — at 16 B per candle instead of a 2000-step walk per lane (the
// replay's cost for T = 2000 is ~0.5 ms whatever the row count).
constexpr int FF_NT = 256, FF_K = 4, FF_TT = FF_NT * FF_K;

__global__ __launch_bounds__(FF_NT) void ffill_kernel(const RollBatch B, int vec) {
  __shared__ double sv[FF_TT];
  __shared__ int sW[FF_NT / WAVE];
  __shared__ double sCar;
  const RollJob& A = B.j[blockIdx.y];
  const int64_t sym = blockIdx.x;
  if (sym >= A.rows) return;   // the whole block: no barrier is left waiting
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const double* __restrict__ x = A.x + sym * A.ld_in;
  double* __restrict__ out = A.out + sym * A.ld_out;
  const int T = B.T;
  if (tid == 0) sCar = qnan();   // leading NaNs stay
  for (int t0 = 0; t0 < T; t0 += FF_TT) {
    const int tb = t0 + FF_K * tid;
    double v[FF_K];
#pragma unroll
    for (int k = 0; k < FF_K; ++k) v[k] = tb + k < T ? x[tb + k] : qnan();
    int li = -1;
#pragma unroll
    for (int k = 0; k < FF_K; ++k) {
      if (v[k] == v[k]) li = tb + k;
      sv[FF_K * tid + k] = v[k];
    }
    const int inc = wave_scan_max_dpp(li + 1, lane) - 1;   // indices >= -1
    if (lane == WAVE - 1) sW[w] = inc;
    int p = dpp_i32<DPP_WAVE_SHR1>(inc + 1) - 1;           // lane 0 -> -1
    __syncthreads();   // the tile, the wave totals and the carry are visible
    for (int u = 0; u < w; ++u) p = max(p, sW[u]);
    double cur = p >= t0 ? sv[p - t0] : sCar;
    double o[FF_K];
#pragma unroll
    for (int k = 0; k < FF_K; ++k) {
      cur = v[k] == v[k] ? v[k] : cur;
      o[k] = cur;
    }
    store_lines<FF_K>(out, tb, T, vec != 0, o);
    __syncthreads();   // every read of sv / sW / sCar of this tile is done
    if (tid == FF_NT - 1) sCar = cur;
  }
}

// ---- rank kernels (lane = symbol x segment, sorted window in registers) -----------
template <int W>
struct SortedWin {
  double a[W];
  int n;
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (int i = 0; i < W; ++i) a[i] = __builtin_inf();
    n = 0;
  }
  // number of stored values < v (padding is +inf, never counted for finite v)
  __device__ __forceinline__ int rank(double v) const {
    int p = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) p += a[i] < v ? 1 : 0;
    return p;
  }
  __device__ __forceinline__ void insert(double v) {
    const int p = rank(v);
#pragma unroll
    for (int i = W - 1; i > 0; --i) a[i] = i > p ? a[i - 1] : (i == p ? v : a[i]);
    a[0] = p == 0 ? v : a[0];
    ++n;
  }
  __device__ __forceinline__ void erase(double v) {   // v is stored
    const int p = rank(v);
#pragma unroll
    for (int i = 0; i < W - 1; ++i) a[i] = i >= p ? a[i + 1] : a[i];
    a[W - 1] = __builtin_inf();
    --n;
  }
  // a[k] for a run-time k: a masked OR over the slots (a select chain here is
  // folded by the compiler into one dynamically indexed load, which would
  // push the whole window out of registers into scratch)
  __device__ __forceinline__ double get(int k) const {
    unsigned long long r = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const unsigned long long m = 0ull - (unsigned long long)(i == k);
      r |= m & (unsigned long long)__double_as_longlong(a[i]);
    }
    return __longlong_as_double((long long)r);
  }
};

template <int W>
__global__ __launch_bounds__(256) void rank_kernel(const RollBatch B) {
  const RollJob& A = B.j[blockIdx.y];
  const int64_t item = (int64_t)blockIdx.x * 256 + threadIdx.x;
  // consecutive lanes: consecutive symbols of one segment
  const int64_t sym = item % B.S;
  const int seg = (int)(item / B.S);
  if (seg >= A.nseg) return;
  const double* __restrict__ x = A.x + sym * A.ld_in;
  double* __restrict__ out = A.out + sym * A.ld_out;
  const int T = B.T, w = A.win, sh = A.shift;
  const int t_begin = seg * A.seg, t_end = min(T, t_begin + A.seg);
  auto val = [&](int t) -> double {
    const int i = t - sh;
    return (i >= 0 && i < T) ? win_val(x[i]) : qnan();
  };
  SortedWin<W> win;
  win.clear();
  const int t_start = max(0, t_begin - w + 1);   // rebuild the window of t_begin
  // values leave only once they were inserted by this lane (t - w >= t_start)
  double nx_in = val(t_start), nx_out = qnan();
  for (int t = t_start; t < t_end; ++t) {
    const double vin = nx_in, vout = nx_out;
    nx_in = val(t + 1);   // next step's values, in flight
    nx_out = t + 1 - w >= t_start ? val(t + 1 - w) : qnan();
    if (vout == vout) win.erase(vout);
    if (vin == vin) win.insert(vin);
    if (t < t_begin) continue;
    const int n = win.n;
    double r;
    if (n < A.minp || n == 0) r = qnan();
    else if (A.mode == BQ_ROLL_MEDIAN) {
      const int h = n >> 1;
      if (n & 1) r = win.get(h);
      else {
        r = (win.get(h - 1) + win.get(h)) / 2.0;
      }
    } else if (n == 1) {
      r = win.a[0];
    } else {   // roll_quantile, linear interpolation
      const double idxf = A.q * (double)(n - 1);
      const int idx = (int)idxf;
      if ((double)idx == idxf || A.lower) r = win.get(idx);
      else {
        const double lo = win.get(idx), hi = win.get(idx + 1);
        r = lo + (hi - lo) * (idxf - (double)idx);
      }
    }
    out[t] = r;
  }
}

// ---- slide rank kernel (lane = symbol segment, window sorted in W registers) --------
// The window of a compile-time length W is kept SORTED in W registers, NaNs
// (and the slots not yet filled) as +inf placeholders at the top, with the
// non-NaN count n beside it. One step replaces the leaving value `o` (a
// placeholder while the window fills) by the entering value `v` with no
// search and no index arithmetic: the array with one copy of o removed is
//   b[i] = s[i] < o ? s[i] : s[i+1]        (s[W] = +inf)
// and inserting v into a sorted b is a clamp per slot,
//   s'[i] = max(b[i-1], min(v, b[i]))      (b[-1] = -inf),
// i.e. 1 compare, 2 selects, 1 min, 1 max per slot (5 VALU; ~5 W per output
// against the tile kernel's ~1 100 per 64-output sort for w <= 65). Zeros enter as +0 (x + 0.0), so the
// multiset's values are the exact-mode keys' values; order statistics are a
// pure function of the multiset, so the outputs equal the other kernels' bit
// for bit. The quantile's rank K = int(q (w - 1)) of a full window is a
// template constant (the host has an instantiation per (W, K) where this
// kernel wins and sends any other (w, q) to the tile / stencil kernels), and
// the placeholders are split between -inf at the bottom and +inf at the top
// so that the wanted rank of ANY window count n sits in slot K: every output
// reads two fixed registers.
// Parallelism: lanes = (symbol, segment); a segment first inserts the W - 1
// values before it (the warm-up, insert-only passes).
// Measured at 12.5k x 2k (tools/slide_probe.py, identical outputs, round 4
// box): median(19) 0.20 ms, quantile(0.80, 48) 0.35, quantile(0.85, 60) 0.40,
// quantile(0.92, 80) 0.64, lower quantile(0.80, 96) 0.74 — every strategy
// window runs here (the tile / stencil kernels took 0.28 / 0.61 / 0.60 / 0.73
// / 0.82). The VALU count matches the 5-per-slot model (PMC: 129.5 M wave
// instructions for w = 48). Occupancy is not what binds it: at w = 80 / 96
// the window takes 305 / 412 registers (one wave per SIMD), and round-4
// variants at two waves per SIMD (split placeholders from the start instead
// of the barrel shift below: 291 registers; stepwise loops: 216; 2- or 4-step
// chunks: 224-274) ran 0-40 % slower — each slot is a dependent compare ->
// select -> min -> max chain of fp64 operations.
//
// v_min_f64 / v_max_f64 without the compiler's IEEE-mode canonicalisation of
// operands it cannot prove canonical (a third max per slot on the loop-carried
// registers); no NaN ever reaches them here (placeholders are +inf)
__device__ __forceinline__ double min_f64_nn(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double max_f64_nn(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// 8-byte-aligned pairs of doubles: one 16-byte access (rows are 8-byte aligned)
typedef double dbl2u __attribute__((ext_vector_type(2), aligned(8)));

template <int W, int K, bool MED, bool XC = false>
__global__ __launch_bounds__(256) void slide_rank_kernel(const RollBatch B) {
  // steps per chunk: each lane reads / writes 8 * SL_C contiguous bytes
  // (16 for short windows: 0.27 -> 0.22 ms at w = 19; 8 where registers bind)
  constexpr int SL_C = W <= 24 ? 16 : 8;
  const RollJob& A = B.j[blockIdx.y];
  const int64_t item = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t sym = item % B.S;
  const int seg = (int)(item / B.S);
  if (seg >= A.nseg) return;   // no barriers below
  const double* __restrict__ x = A.x + sym * A.ld_in;
  double* __restrict__ out = A.out + sym * A.ld_out;
  const int T = B.T, sh = A.shift;
  const int t_begin = seg * A.seg, t_end = min(T, t_begin + A.seg);
  // with the crossing flags the window of step t_begin - 1 is built too (its
  // oldest value enters the warm-up and leaves at t_begin): the flag at
  // t_begin needs that step's threshold
  // the flags: an instantiation of its own (their registers); a job of that
  // launch without them skips them (block-uniform)
  const bool xc = XC && A.cross != nullptr;
  const int t_start = max(0, t_begin - W + (xc ? 0 : 1));
  const double inf = __builtin_inf();
  // values of steps ts .. ts + SL_C - 1 (x[t - shift], NaN outside the row):
  // a lane's whole span at once, so every line it touches is used up
  // by this lane's back-to-back accesses (a value per step per lane would
  // keep S * nseg partially read lines live in L2)
  auto load_chunk = [&](int ts, double (&v)[SL_C]) {
    const int i0 = ts - sh;
    if (i0 >= 0 && i0 + SL_C <= T) {
#pragma unroll
      for (int j = 0; j < SL_C; j += 2) {
        const dbl2u p = *reinterpret_cast<const dbl2u*>(x + i0 + j);
        v[j] = p.x;
        v[j + 1] = p.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < SL_C; ++j) v[j] = (i0 + j >= 0 && i0 + j < T) ? x[i0 + j] : qnan();
    }
  };
  // Placeholders split so the wanted rank sits in a FIXED slot: with n
  // numbers in the window, a(n) = int(q (n - 1)) (median: (n - 1) / 2) and
  // B(n) = K - a(n) placeholders at the bottom (-inf), the rest at the top
  // (+inf), the a-th smallest number is s[K] and the next one s[K + 1] for any
  // n (B(n) + n <= W since q < 1). n changes by at most 1 per step and B by
  // at most 1 with it, so a step keeps the split by choosing which kind of
  // placeholder leaves or enters (a NaN leaving or entering is a placeholder
  // leaving or entering). No run-time register index anywhere: partial
  // windows (warm-up, NaN gaps, min_periods < w) cost what full ones do.
  auto a_of = [&](int nn) -> int {
    if constexpr (MED) return (nn - 1) >> 1;
    else return (int)(A.q * (double)(nn - 1));
  };
  auto b_of = [&](int nn) -> int { return nn >= 1 ? K - a_of(nn) : K + 1; };
  // the window before the segment's first output (the W - 1 values of steps
  // t_start .. t_begin - 1; NaNs and steps before the row stay +inf): only
  // insertions while it fills (no value leaves yet), each a clamp pass
  // s'[i] = max(s[i-1], min(v, s[i])) from the top down — 2 VALU per slot
  // instead of a full step's 5; the +inf pad in the top slot is what drops.
  double s[W];
#pragma unroll
  for (int i = 0; i < W; ++i) s[i] = inf;
  int n = 0;
  {
    constexpr int NCH = (W + SL_C - 1) / SL_C;
    const int t0 = t_begin - NCH * SL_C;   // step of chunk slot 0
    for (int c = 0; c < NCH; ++c) {
      if (t0 + (c + 1) * SL_C <= t_start) continue;   // chunk wholly before the window
      double v[SL_C];
      load_chunk(t0 + c * SL_C, v);
#pragma unroll
      for (int j = 0; j < SL_C; ++j) {
        const bool num = t0 + c * SL_C + j >= t_start && win_ok(v[j]);   // +-inf: missing (window op)
        n += num ? 1 : 0;
        const double a = num ? v[j] + 0.0 : inf;
#pragma unroll
        for (int i = W - 1; i > 0; --i) s[i] = max_f64_nn(s[i - 1], min_f64_nn(a, s[i]));
        s[0] = min_f64_nn(a, s[0]);
      }
    }
  }
  // then B(n) of the W - n top placeholders move to the bottom: the array
  // shifted up by B (a log-step barrel shift, -inf filling; the B slots that
  // drop off the top are +inf)
  int nb = b_of(n);
#pragma unroll
  for (int bit = 1; bit < W; bit <<= 1) {
    const bool sh_on = (nb & bit) != 0;
#pragma unroll
    for (int i = W - 1; i >= 0; --i) s[i] = sh_on ? (i >= bit ? s[i - bit] : -inf) : s[i];
  }
  // the order statistic of the window in s holding n numbers
  auto rank_value = [&]() -> double {
    if (!(n >= A.minp && n > 0)) return qnan();
    constexpr int K1 = K + 1 < W ? K + 1 : K;
    const double lo = s[K];
    if constexpr (MED) {
      return (n & 1) ? lo : (lo + s[K1]) / 2.0;
    } else {
      const double idxf = A.q * (double)(n - 1);
      const int idx = (int)idxf;
      return ((double)idx == idxf || A.lower) ? lo : lo + (s[K1] - lo) * (idxf - (double)idx);
    }
  };
  // crossing flags: the previous step's series value and threshold (NaN
  // before the row: pandas' shift(1), and NaN compares false)
  double pthr = qnan(), pps = qnan();
  if (xc && t_begin >= 1) {
    pthr = rank_value();
    pps = x[t_begin - 1];
  }
  for (int tc = t_begin; tc < t_end; tc += SL_C) {
    double vin[SL_C], vout[SL_C], r[SL_C], xs[XC ? SL_C : 1];
    load_chunk(tc, vin);
    if constexpr (XC)
      if (xc) load_chunk(tc + sh, xs);   // x[t] itself
    if (tc + SL_C - 1 - W >= t_start) load_chunk(tc - W, vout);   // else: placeholders below
#pragma unroll
    for (int j = 0; j < SL_C; ++j) {
      const int t = tc + j;
      const bool has_out = t - W >= t_start;   // else a placeholder leaves
      const bool in_num = t < t_end && win_ok(vin[j]);   // NaN and +-inf are missing (window op)
      const bool out_num = t < t_end && has_out && win_ok(vout[j]);
      const int n2 = n + (in_num ? 1 : 0) - (out_num ? 1 : 0);
      const int nb2 = b_of(n2);
      // a leaving placeholder is a bottom one when B drops, an entering one a
      // bottom one when B grows (otherwise top; both top when nothing changes:
      // removing an absent +inf and inserting +inf leaves the array as is)
      const double o = out_num ? vout[j] + 0.0 : (nb2 < nb ? -inf : inf);
      const double v = in_num ? vin[j] + 0.0 : (nb2 > nb ? -inf : inf);
      n = n2;
      nb = nb2;
      double bp = -inf;
#pragma unroll
      for (int i = 0; i < W; ++i) {
        const double nxt = i + 1 < W ? s[i + 1] : inf;
        const double b = s[i] < o ? s[i] : nxt;
        s[i] = max_f64_nn(bp, min_f64_nn(v, b));
        bp = b;
      }
      r[j] = rank_value();
    }
    if (XC && xc) {   // (x[t] >= thr[t]) & (x[t - 1] < thr[t - 1]), one byte per candle
      uint64_t f[SL_C / 8];
#pragma unroll
      for (int m = 0; m < SL_C / 8; ++m) f[m] = 0;
#pragma unroll
      for (int j = 0; j < SL_C; ++j) {
        const bool c = xs[j] >= r[j] && pps < pthr;
        f[j / 8] |= (uint64_t)(c ? 1 : 0) << (8 * (j % 8));
        pps = xs[j];
        pthr = r[j];
      }
      uint8_t* __restrict__ cr = A.cross + sym * A.ld_cross;
      if (tc + SL_C <= t_end && (((uintptr_t)(cr + tc)) & 7u) == 0) {
#pragma unroll
        for (int m = 0; m < SL_C / 8; ++m) *reinterpret_cast<uint64_t*>(cr + tc + 8 * m) = f[m];
      } else {
#pragma unroll
        for (int j = 0; j < SL_C; ++j)
          if (tc + j < t_end) cr[tc + j] = (uint8_t)((f[j / 8] >> (8 * (j % 8))) & 1u);
      }
    }
    if (tc >= t_begin && tc + SL_C <= t_end) {
#pragma unroll
      for (int j = 0; j < SL_C; j += 2) {
        dbl2u p;
        p.x = r[j];
        p.y = r[j + 1];
        *reinterpret_cast<dbl2u*>(out + tc + j) = p;
      }
    } else {
#pragma unroll
      for (int j = 0; j < SL_C; ++j)
        if (tc + j >= t_begin && tc + j < t_end) out[tc + j] = r[j];
    }
  }
}

#ifndef BQ_SG_C
#define BQ_SG_C 8   // steps per chunk of slide_group_kernel (4: 0.64 vs 0.61 ms at w = 80)
#endif

// ---- slide rank kernel, lane groups (w >= 48) -----------------------------------------
// slide_rank_kernel's sorted window split over G = 2 or 4 adjacent lanes:
// lane q of a group holds slots q H .. q H + H - 1 (H = W / G), so a lane
// holds 1/G of the registers and a SIMD two to four waves instead of one at
// w = 80 / 96 — the single-lane step is a dependent compare -> select -> min
// -> max chain per slot that one wave per SIMD cannot hide. The group's lanes
// read the same leaving / entering values (the same addresses: one
// transaction) and keep the same count n and placeholder split B(n). A step
// is the same removal / insertion per slot; the two values that cross a lane
// boundary go by one DPP quad permutation each: the upper neighbour's old
// bottom slot (the successor of this lane's top slot) before the step, the
// lower neighbour's top removal result b[H - 1] (the predecessor of this
// lane's bottom clamp) after the removal pass, so slot 0 is clamped last.
// The placeholders are split from the first step (no barrel shift): a
// warm-up step is a full step. The rank slots K, K + 1 lie in one lane
// (static_assert), which alone stores. Same multiset, same slots, same
// arithmetic: the outputs equal slide_rank_kernel's bit for bit.
template <int G>
__device__ __forceinline__ double from_upper(double x) {   // lane q <- lane q + 1 of the group
  return dpp_f64<G == 2 ? 0xB1 : 0xF9>(x);                  // quad_perm [1,0,3,2] / [1,2,3,3]
}
template <int G>
__device__ __forceinline__ double from_lower(double x) {   // lane q <- lane q - 1 of the group
  return dpp_f64<G == 2 ? 0xB1 : 0x90>(x);                  // quad_perm [1,0,3,2] / [0,0,1,2]
}

template <int W, int K, bool MED, int G>
__global__ __launch_bounds__(256) void slide_group_kernel(const RollBatch B) {
  constexpr int H = W / G;
  constexpr int KL = K / H;   // the lane holding the rank slots
  static_assert((G == 2 || G == 4) && W % G == 0 && (K + 1) / H == KL && K + 1 < W, "group layout");
  constexpr int SL_C = BQ_SG_C;
  const RollJob& A = B.j[blockIdx.y];
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int q = threadIdx.x & (G - 1);
  const int64_t item = gid / G;
  const int64_t sym = item % B.S;
  const int seg = (int)(item / B.S);
  if (seg >= A.nseg) return;   // a group leaves together (no barriers below)
  const double* __restrict__ x = A.x + sym * A.ld_in;
  double* __restrict__ out = A.out + sym * A.ld_out;
  const int T = B.T, sh = A.shift;
  const int t_begin = seg * A.seg, t_end = min(T, t_begin + A.seg);
  const int t_start = max(0, t_begin - W + 1);
  const double inf = __builtin_inf();
  auto load_chunk = [&](int ts, double (&v)[SL_C]) {
    const int i0 = ts - sh;
    if (i0 >= 0 && i0 + SL_C <= T) {
#pragma unroll
      for (int j = 0; j < SL_C; j += 2) {
        const dbl2u p = *reinterpret_cast<const dbl2u*>(x + i0 + j);
        v[j] = p.x;
        v[j + 1] = p.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < SL_C; ++j) v[j] = (i0 + j >= 0 && i0 + j < T) ? x[i0 + j] : qnan();
    }
  };
  auto a_of = [&](int nn) -> int {
    if constexpr (MED) return (nn - 1) >> 1;
    else return (int)(A.q * (double)(nn - 1));
  };
  auto b_of = [&](int nn) -> int { return nn >= 1 ? K - a_of(nn) : K + 1; };
  const bool top = q == G - 1, bottom = q == 0;
  double s[H];
  int n = 0, nb = K + 1;
  int tw;   // the first step of the full-step loop
  if constexpr (G == 2) {
    // pairs: the window before the segment filled insert-only (the
    // single-lane kernel's warm-up, 2 VALU per slot instead of 5: every
    // placeholder +inf on top, the lower lane's old top slot handed up for
    // the upper lane's bottom clamp), then the split made by shifting the
    // pair's combined array up by B(n)
#pragma unroll
    for (int i = 0; i < H; ++i) s[i] = inf;
    constexpr int NCH = (W + SL_C - 1) / SL_C;
    const int t0w = t_begin - NCH * SL_C;   // step of chunk slot 0
    for (int c = 0; c < NCH; ++c) {
      if (t0w + (c + 1) * SL_C <= t_start) continue;   // chunk wholly before the window
      double v[SL_C];
      load_chunk(t0w + c * SL_C, v);
#pragma unroll
      for (int j = 0; j < SL_C; ++j) {
        const bool num = t0w + c * SL_C + j >= t_start && win_ok(v[j]);
        n += num ? 1 : 0;
        const double a = num ? v[j] + 0.0 : inf;
        const double dn = from_lower<G>(s[H - 1]);
#pragma unroll
        for (int i = H - 1; i > 0; --i) s[i] = max_f64_nn(s[i - 1], min_f64_nn(a, s[i]));
        s[0] = max_f64_nn(bottom ? -inf : dn, min_f64_nn(a, s[0]));
      }
    }
    // log-step shift of the combined array [lower | upper] by nb (-inf
    // filling): per step b, the upper lane's slots i < b take the lower
    // lane's slot H + i - b (read by a swap before the step), the lower
    // lane's take -inf
    nb = b_of(n);
#pragma unroll
    for (int b = 1; b < W; b <<= 1) {
      const bool sh_on = (nb & b) != 0;
      double p[H];
#pragma unroll
      for (int i = 0; i < H; ++i) {
        if (i >= b) break;
        const int j = H + i - b;
        p[i] = j >= 0 ? from_upper<G>(s[j >= 0 ? j : 0]) : -inf;   // the partner's slot j
      }
#pragma unroll
      for (int i = H - 1; i >= 0; --i) {
        const double v = i >= b ? s[i >= b ? i - b : 0] : (bottom ? -inf : p[i]);
        s[i] = sh_on ? v : s[i];
      }
    }
    tw = t_begin;
  } else {
    // the empty window: B(0) = K + 1 bottom placeholders, the rest on top;
    // steps from t_start (the W - 1 before the segment fill the window) are
    // full steps, in chunks aligned to t_begin (the single-lane output chunks)
#pragma unroll
    for (int i = 0; i < H; ++i) s[i] = q * H + i < K + 1 ? -inf : inf;
    tw = t_begin - ((t_begin - t_start + SL_C - 1) / SL_C) * SL_C;
  }
  for (int tc = tw; tc < t_end; tc += SL_C) {
    double vin[SL_C], vout[SL_C], r[SL_C];
    load_chunk(tc, vin);
    if (tc + SL_C - 1 - W >= t_start) load_chunk(tc - W, vout);   // else: placeholders leave
#pragma unroll
    for (int j = 0; j < SL_C; ++j) {
      const int t = tc + j;
      const bool live = t >= t_start && t < t_end;   // steps outside: no-ops (+inf out, +inf in)
      const bool has_out = t - W >= t_start;
      const bool in_num = live && win_ok(vin[j]);
      const bool out_num = live && has_out && win_ok(vout[j]);
      const int n2 = n + (in_num ? 1 : 0) - (out_num ? 1 : 0);
      const int nb2 = b_of(n2);
      const double o = out_num ? vout[j] + 0.0 : (nb2 < nb ? -inf : inf);
      const double v = in_num ? vin[j] + 0.0 : (nb2 > nb ? -inf : inf);
      n = n2;
      nb = nb2;
      const double up = from_upper<G>(s[0]);   // the old slot above this lane's top one
      const double b0 = s[0] < o ? s[0] : (H > 1 ? s[1 < H ? 1 : 0] : (top ? inf : up));
      double bp = b0;
#pragma unroll
      for (int i = 1; i < H; ++i) {
        const double nxt = i + 1 < H ? s[i + 1 < H ? i + 1 : i] : (top ? inf : up);
        const double b = s[i] < o ? s[i] : nxt;
        s[i] = max_f64_nn(bp, min_f64_nn(v, b));
        bp = b;
      }
      const double dn = from_lower<G>(bp);     // the removal result below this lane's bottom slot
      s[0] = max_f64_nn(bottom ? -inf : dn, min_f64_nn(v, b0));
      r[j] = qnan();
      if (n >= A.minp && n > 0) {
        constexpr int KS = K - KL * H, KS1 = K + 1 - KL * H;
        const double lo = s[KS];
        if constexpr (MED) {
          r[j] = (n & 1) ? lo : (lo + s[KS1]) / 2.0;
        } else {
          const double idxf = A.q * (double)(n - 1);
          const int idx = (int)idxf;
          r[j] = ((double)idx == idxf || A.lower) ? lo : lo + (s[KS1] - lo) * (idxf - (double)idx);
        }
      }
    }
    if (q != KL || tc < t_begin) continue;
    if (tc + SL_C <= t_end) {
#pragma unroll
      for (int j = 0; j < SL_C; j += 2) {
        dbl2u p;
        p.x = r[j];
        p.y = r[j + 1];
        *reinterpret_cast<dbl2u*>(out + tc + j) = p;
      }
    } else {
#pragma unroll
      for (int j = 0; j < SL_C; ++j)
        if (tc + j < t_end) out[tc + j] = r[j];
    }
  }
}

// (x[t] >= thr[t]) & (x[t-1] < thr[t-1]) where the slide kernel does not run
__global__ __launch_bounds__(256) void cross_kernel(const double* __restrict__ x, const double* __restrict__ thr,
                                                    int64_t S, int T, int64_t ld_in, int64_t ld_out,
                                                    uint8_t* __restrict__ cross, int64_t ld_cross) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= S * (int64_t)T) return;
  const int64_t s = i / T;
  const int t = (int)(i - s * T);
  const double* xr = x + s * ld_in;
  const double* tr = thr + s * ld_out;
  const bool c = xr[t] >= tr[t] && t >= 1 && xr[t - 1] < tr[t - 1];
  cross[s * ld_cross + t] = c ? 1 : 0;
}

// ---- tile rank kernel (wave = 64*OPL consecutive outputs of one symbol) --------------
// The windows of TILE consecutive outputs all lie in one union of
// U = w + TILE - 1 consecutive values. The wave loads the union (coalesced:
// one contiguous row span), sorts it once — a bitonic network over 64*EPL
// order-preserving u64 keys with the union position as payload, element
// i = lane*EPL + e so the two shortest distances stay in registers — and
// then every lane walks the sorted union (LDS broadcast reads) counting the
// members of its own window (position in [m, m+w)) until it has passed the
// ranks it needs. The walk runs from the side nearer the ranks (descending
// for q > 0.5) and stops when every lane is done. No lane carries state
// along the row, so there is no warm-up per segment: parallelism is
// S * ceil(T / TILE) waves whatever the shape (the lane kernel above needs
// w warm-up steps per segment, which dominates at live shapes).
__device__ __forceinline__ unsigned long long okey_nan_last(double x) {
  if (x != x) return ~0ull;
  if (x == 0.0) x = 0.0;   // -0.0 and +0.0 compare equal
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ __forceinline__ double okey_value(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & ~(1ull << 63)) : ~k;
  return __longlong_as_double((long long)b);
}

// value of lane ^ ld (ld a power of two, a compile-time constant once the
// sort's loops are unrolled): DPP quad permutes for 1 and 2, ds_swizzle's
// xor mode for 4..16 (no address operand), ds_bpermute only across halves
__device__ __forceinline__ unsigned lane_xor(unsigned v, int ld) {
  switch (ld) {
    case 1: return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // [1,0,3,2]
    case 2: return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // [2,3,0,1]
    case 4: return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (4 << 10));
    case 8: return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (8 << 10));
    case 16: return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (16 << 10));
    default: return __shfl_xor(v, ld, WAVE);
  }
}

// Inclusive XOR prefix of a u32 over the wave (DPP rows + readlane row
// totals; bound_ctrl's 0 is XOR's identity).
__device__ __forceinline__ unsigned wave_scan_xor(unsigned x, int lane) {
  x ^= (unsigned)dpp_i32<DPP_ROW_SHR1>((int)x);
  x ^= (unsigned)dpp_i32<DPP_ROW_SHR2>((int)x);
  x ^= (unsigned)dpp_i32<DPP_ROW_SHR4>((int)x);
  x ^= (unsigned)dpp_i32<DPP_ROW_SHR8>((int)x);
  const unsigned r0 = (unsigned)__builtin_amdgcn_readlane((int)x, 15);
  const unsigned r1 = r0 ^ (unsigned)__builtin_amdgcn_readlane((int)x, 31);
  const unsigned r2 = r1 ^ (unsigned)__builtin_amdgcn_readlane((int)x, 47);
  const int row = lane >> 4;
  return x ^ (row == 0 ? 0u : (row == 1 ? r0 : (row == 2 ? r1 : r2)));
}

// index of the r-th (0-based) set bit of the NW-word mask M (r < popcount(M)):
// the word by running popcounts, then a 16/8/4/2/1 popcount bisection in it;
// selects only (no divergent branches)
template <int NW>
__device__ __forceinline__ int select_bit(const unsigned (&M)[NW], int r) {
  unsigned word = 0;
  int base = 0;
  bool found = false;
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const int c = __popc(M[q]);
    const bool here = !found && r < c;
    word = here ? M[q] : word;
    base = here ? 32 * q : base;
    r = (!found && !here) ? r - c : r;
    found = found || here;
  }
  int p = 0;
#pragma unroll
  for (int h = 16; h >= 1; h >>= 1) {
    const int c = __popc(word & ((1u << h) - 1u));
    const bool up = r >= c;
    r = up ? r - c : r;
    p = up ? p + h : p;
    word = up ? word >> h : word;
  }
  return base + p;
}

// SEL: instead of walking the sorted union, each lane picks its
// ranks by bit selection. Union slot u gets the one-hot mask of its sorted
// index; the wave's XOR prefix over u gives X(u), and the members of window
// [m, m + w) in sorted order are the bits of X(m + w - 1) ^ X(m - 1) (slots
// hold distinct sorted indices). NaNs sort last, so the r-th member for
// r < n (the window's non-NaN count) is a number. Cost per wave: one scan of
// N/32-word masks and two selections per output, instead of a walk of up to
// N broadcast reads that every lane of the wave waits out. Measured at
// 12.5k x 2k (tools/rank_ab.py, identical digests): 64-output tiles 0.74-0.92
// -> 0.57-0.61 ms for every q; 128-output tiles (256 slots, 8-word masks,
// 43 KB of LDS per block) win for central ranks (median 96: 1.30 -> 0.92 ms)
// and lose where the walk from the nearer end is short (q = 0.92, w = 80:
// 0.73 -> 0.95), so the host picks per job (sel_tile).
#ifndef BQ_RANK_SEL
#define BQ_RANK_SEL 1   // 0: never select (measurement)
#endif

#ifndef BQ_TR_WPB
#define BQ_TR_WPB 1   // waves per block of the tile rank kernel
#endif
// PACK (panel-mode jobs, bq_roll_job.panel = 1): the union slot rides in the
// key's low log2(N) bits instead of a separate payload — one 64-bit key per
// element through the sort (two cross-lane moves and two selects per element
// and stage instead of three), the slot read back from the key, the value
// from an LDS copy of the union. Keys that differ only in those low bits
// (values within 2^-(52 - log2 N) relative of each other) may swap order, so
// a selected order statistic is the exact value of an element within that of
// the true one (N = 128: 2^-45) — within rounding, not bit for bit (exact
// mode keeps the full keys).
template <int EPL, int OPL, bool SEL, bool PACK>
__global__ __launch_bounds__(64 * BQ_TR_WPB) void tile_rank_kernel(const RollBatch B) {
  constexpr int N = WAVE * EPL;          // sorted slots (power of two)
  constexpr unsigned long long PMASK = (unsigned long long)(N - 1);
  constexpr int TILE = WAVE * OPL;       // outputs per wave
  constexpr int NWORD = N / 32;          // words of a union-slot mask
  // one wave per block (BQ_TR_WPB = 1): the waves share no LDS, so a block
  // barrier would only make independent tiles wait for each other
  __shared__ unsigned long long s_key[BQ_TR_WPB][N];
  __shared__ unsigned short s_pos[BQ_TR_WPB][PACK ? 1 : N];
  __shared__ double s_val[BQ_TR_WPB][PACK ? N : 1];   // PACK: the union's values by slot
  __shared__ unsigned short s_cnt[BQ_TR_WPB][N + 1];   // non-NaN values before union slot u
  __shared__ unsigned char s_idx[BQ_TR_WPB][SEL ? N : 1];              // union slot -> sorted index
  __shared__ unsigned s_X[BQ_TR_WPB][SEL ? N : 1][SEL ? NWORD : 1];    // XOR prefix of the one-hot masks
  const RollJob& A = B.j[blockIdx.y];
  const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
  const int T = B.T, w = A.win;
  const int64_t nt = (T + TILE - 1) / TILE;
  const int64_t tile = (int64_t)blockIdx.x * BQ_TR_WPB + wv;
  const bool live = tile < B.S * nt;   // every wave reaches the barriers
  const int64_t sym = live ? tile / nt : 0;
  const int t0 = live ? (int)(tile % nt) * TILE : 0;
  const double* __restrict__ x = A.x + sym * A.ld_in;
  const int ubase = t0 - w + 1 - A.shift;   // x index of union slot 0
  const int U = w + TILE - 1;

  unsigned long long key[EPL];
  unsigned pos[EPL];
  bool num[EPL];
  int c = 0;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int u = lane * EPL + e;
    const int i = ubase + u;
    const double v = (live && u < U && t0 - w + 1 + u >= A.shift && i < T) ? win_val(x[i]) : qnan();
    key[e] = okey_nan_last(v);
    num[e] = v == v;
    if constexpr (PACK) {
      key[e] = (key[e] & ~PMASK) | (unsigned long long)u;   // NaN keys stay above every number
      s_val[wv][u] = v;
    }
    pos[e] = (unsigned)u;
    c += num[e] ? 1 : 0;
  }
  // exclusive prefix of the non-NaN counts in union order
  int incl = c;
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const int y = __shfl_up(incl, d, WAVE);
    if (lane >= d) incl += y;
  }
  {
    int run = incl - c;
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      s_cnt[wv][lane * EPL + e] = (unsigned short)run;
      run += num[e] ? 1 : 0;
    }
    if (lane == WAVE - 1) s_cnt[wv][N] = (unsigned short)run;
  }

  // bitonic sort of (key, pos), ascending
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int d = k >> 1; d > 0; d >>= 1) {
      if (d < EPL) {   // partner in this lane's registers
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          if (e & d) continue;
          const int i = lane * EPL + e;
          const bool up = (i & k) == 0;
          const unsigned long long a = key[e], b = key[e + d];
          const bool swap = (up & (b < a)) | (!up & (a < b));   // selects, not branches
          key[e] = swap ? b : a;
          key[e + d] = swap ? a : b;
          if constexpr (!PACK) {
            const unsigned pa = pos[e], pb = pos[e + d];
            pos[e] = swap ? pb : pa;
            pos[e + d] = swap ? pa : pb;
          }
        }
      } else {
        const int ld = d / EPL;   // partner lane distance
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int i = lane * EPL + e;
          const unsigned lo32 = lane_xor((unsigned)key[e], ld);
          const unsigned hi32 = lane_xor((unsigned)(key[e] >> 32), ld);
          const unsigned long long pk = ((unsigned long long)hi32 << 32) | lo32;
          const bool lower = (i & d) == 0, up = (i & k) == 0;
          // the lower slot of an ascending pair keeps the minimum
          const bool keep_min = lower == up;
          const bool take = (keep_min & (pk < key[e])) | (!keep_min & (key[e] < pk));
          key[e] = take ? pk : key[e];
          if constexpr (!PACK) {
            const unsigned pp = lane_xor(pos[e], ld);
            pos[e] = take ? pp : pos[e];
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    if constexpr (PACK) pos[e] = (unsigned)(key[e] & PMASK);
    s_key[wv][lane * EPL + e] = key[e];
    if constexpr (!PACK) s_pos[wv][lane * EPL + e] = (unsigned short)pos[e];
    if constexpr (SEL) s_idx[wv][pos[e]] = (unsigned char)(lane * EPL + e);
  }
  // value of a sorted key: the key itself, or (PACK) the union slot's value
  auto kval = [&](unsigned long long kk) -> double {
    if constexpr (PACK) return s_val[wv][kk & PMASK];
    else return okey_value(kk);
  };
  __syncthreads();
  if constexpr (SEL) {
    // one-hot masks of this lane's union slots, their XOR prefix in slot order
    unsigned P[EPL][NWORD];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int j = s_idx[wv][lane * EPL + e];
#pragma unroll
      for (int q = 0; q < NWORD; ++q) {
        const unsigned oh = (j >> 5) == q ? (1u << (j & 31)) : 0u;
        P[e][q] = e == 0 ? oh : (P[e - 1][q] ^ oh);
      }
    }
#pragma unroll
    for (int q = 0; q < NWORD; ++q) {
      const unsigned tot = P[EPL - 1][q];
      const unsigned excl = wave_scan_xor(tot, lane) ^ tot;
#pragma unroll
      for (int e = 0; e < EPL; ++e) s_X[wv][lane * EPL + e][q] = excl ^ P[e][q];
    }
    __syncthreads();
    double* __restrict__ out = A.out + sym * A.ld_out;
#pragma unroll
    for (int o = 0; o < OPL; ++o) {
      const int mo = o * WAVE + lane;
      const int t = t0 + mo;
      const int n = (int)s_cnt[wv][mo + w] - (int)s_cnt[wv][mo];
      if (!live || t >= T) continue;
      double r = qnan();
      if (n >= A.minp && n > 0) {
        unsigned M[NWORD];
#pragma unroll
        for (int q = 0; q < NWORD; ++q)
          M[q] = s_X[wv][mo + w - 1][q] ^ (mo > 0 ? s_X[wv][mo - 1][q] : 0u);
        int a;
        bool two;
        double frac = 0.0;
        if (A.mode == BQ_ROLL_MEDIAN) {
          const int h = n >> 1;
          a = (n & 1) ? h : h - 1;
          two = !(n & 1);
        } else {
          const double idxf = A.q * (double)(n - 1);
          a = (int)idxf;
          two = n > 1 && (double)a != idxf && !A.lower;
          frac = idxf - (double)a;
        }
        const double lo = kval(s_key[wv][select_bit<NWORD>(M, a)]);
        if (!two) r = lo;
        else {
          const double hi = kval(s_key[wv][select_bit<NWORD>(M, a + 1)]);
          if (A.mode == BQ_ROLL_MEDIAN) r = (lo + hi) / 2.0;
          else r = lo + (hi - lo) * frac;
        }
      }
      out[t] = r;
    }
    return;
  }

  // per output: window count n, the ranks needed, the walk targets
  const int n_num = s_cnt[wv][N];   // non-NaN values in the union (sorted first)
  const bool desc = A.mode == BQ_ROLL_QUANTILE && A.q > 0.5;
  int m[OPL], cnt[OPL], tlo[OPL], thi[OPL];
  bool need2[OPL], act[OPL];
  double idxf[OPL];
  unsigned long long klo[OPL], khi[OPL];
#pragma unroll
  for (int o = 0; o < OPL; ++o) {
    m[o] = o * WAVE + lane;
    const int n = (int)s_cnt[wv][m[o] + w] - (int)s_cnt[wv][m[o]];
    act[o] = live && t0 + m[o] < T && n >= A.minp && n > 0;
    int a = 0;
    need2[o] = false;
    idxf[o] = 0.0;
    if (A.mode == BQ_ROLL_MEDIAN) {
      const int h = n >> 1;
      a = (n & 1) ? h : h - 1;
      need2[o] = !(n & 1);
    } else {
      idxf[o] = A.q * (double)(n - 1);
      a = (int)idxf[o];
      need2[o] = n > 1 && (double)a != idxf[o] && !A.lower;
    }
    tlo[o] = desc ? n - a : a + 1;
    thi[o] = desc ? n - a - 1 : a + 2;
    cnt[o] = 0;
    klo[o] = khi[o] = 0;
  }
  auto done = [&]() {
    bool d = true;
#pragma unroll
    for (int o = 0; o < OPL; ++o) {
      const int need = need2[o] ? (tlo[o] > thi[o] ? tlo[o] : thi[o]) : tlo[o];
      d = d && (!act[o] || cnt[o] >= need);
    }
    return d;
  };
  for (int s0 = 0; s0 < n_num; s0 += 4) {
    if (__all(done())) break;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = s0 + j;
      if (s >= n_num) break;
      const int si = desc ? n_num - 1 - s : s;
      const unsigned long long kk = s_key[wv][si];
      const int p = PACK ? (int)(kk & PMASK) : (int)s_pos[wv][si];
#pragma unroll
      for (int o = 0; o < OPL; ++o) {
        const bool mem = (unsigned)(p - m[o]) < (unsigned)w;
        cnt[o] += mem ? 1 : 0;
        klo[o] = (mem && cnt[o] == tlo[o]) ? kk : klo[o];
        khi[o] = (mem && cnt[o] == thi[o]) ? kk : khi[o];
      }
    }
  }
  double* __restrict__ out = A.out + sym * A.ld_out;
#pragma unroll
  for (int o = 0; o < OPL; ++o) {
    const int t = t0 + m[o];
    if (!live || t >= T) continue;
    double r = qnan();
    if (act[o]) {
      const double lo = kval(klo[o]);
      if (!need2[o]) r = lo;
      else {
        const double hi = kval(khi[o]);
        if (A.mode == BQ_ROLL_MEDIAN) r = (lo + hi) / 2.0;
        else r = lo + (hi - lo) * (idxf[o] - (double)(int)idxf[o]);
      }
    }
    out[t] = r;
  }
}

// ---- stencil rank kernel (lane = one output, window from an LDS row span) ------------
// For short windows (w <= 32): a block takes 256 consecutive outputs of one
// symbol and stages their values plus the w - 1 before them in LDS with one
// coalesced pass; each lane copies its own window into registers (NaN ->
// +inf, counted out) and sorts it with Batcher's odd-even merge network on N
// slots (N the window bucket; slots >= w hold +inf, comparators beyond N are
// pruned — a +inf partner never moves), then picks its ranks. No state along
// the row (no warm-up, no lane walking its own row through the caches),
// ~1.1 reads and one coalesced write per output; the network is
// O(N log^2 N) min/max pairs per output.
template <int N>
__device__ __forceinline__ void sort_network(double (&v)[N]) {
  constexpr int NP = N <= 4 ? 4 : N <= 8 ? 8 : N <= 16 ? 16 : 32;
#pragma unroll
  for (int p = 1; p < NP; p <<= 1) {
#pragma unroll
    for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
      for (int j = k % p; j + k < NP; j += 2 * k) {
#pragma unroll
        for (int i = 0; i < k; ++i) {
          const int a = i + j, b = i + j + k;
          if (b < N && a / (2 * p) == b / (2 * p)) {
            const double x = v[a], y = v[b];
            v[a] = fmin(x, y);
            v[b] = fmax(x, y);
          }
        }
      }
    }
  }
}

template <int N>
__device__ __forceinline__ double pick(const double (&v)[N], int k) {   // v[k], k run-time
  unsigned long long r = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) r |= (0ull - (unsigned long long)(i == k)) & (unsigned long long)__double_as_longlong(v[i]);
  return __longlong_as_double((long long)r);
}

constexpr int SR_NT = 256;

template <int N>
__global__ __launch_bounds__(SR_NT) void stencil_rank_kernel(const RollBatch B) {
  __shared__ double s[SR_NT + N - 1];
  const RollJob& A = B.j[blockIdx.y];
  const int T = B.T, w = A.win;
  const int nbt = (T + SR_NT - 1) / SR_NT;
  const int64_t sym = blockIdx.x / nbt;
  const int t0 = (int)(blockIdx.x % nbt) * SR_NT;
  const double* __restrict__ x = A.x + sym * A.ld_in;
  // s[i] = the series value of candle t0 - (w - 1) + i, i.e. x[that - shift]
  const int base = t0 - (w - 1) - A.shift;
  for (int i = threadIdx.x; i < SR_NT + w - 1; i += SR_NT) {
    const int xi = base + i;
    s[i] = (xi >= 0 && xi < T) ? win_val(x[xi]) : qnan();
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  if (A.mode == BQ_ROLL_ISUM) {
    // integers: every partial sum is exact, so any order gives pandas' Kahan
    // value; pandas' same-value rule (the run of equal values covers the
    // window: prev * nobs) only decides the sign of a zero sum
    double sum = 0.0, last = qnan();
    int n = 0;
    bool same = true;
    for (int j = w - 1; j >= 0; --j) {   // newest first: `last` is pandas' prev
      const double a = s[threadIdx.x + j];
      if (a == a) {
        if (n == 0) last = a;
        same = same && a == last;
        sum += a;
        ++n;
      }
    }
    double r;
    if (n == 0 && A.minp == 0) r = 0.0;
    else if (n < A.minp || n == 0) r = qnan();
    else r = same ? last * (double)n : sum;
    A.out[sym * A.ld_out + t] = r;
    return;
  }
  if (A.mode == BQ_ROLL_QUANTILE && (A.q == 1.0 || A.q == 0.0)) {
    // rolling max / min (q = 1 / 0: rank n - 1 / 0): the extreme of the
    // window's numbers, which is what the network leaves in that slot (its
    // fmin / fmax order -0 below +0 the same way) — w - 1 comparisons
    // instead of the sort
    const bool hi = A.q == 1.0;
    double e = hi ? -__builtin_inf() : __builtin_inf();
    int n = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double a = s[threadIdx.x + j];
      const bool num = j < w && a == a;
      n += num ? 1 : 0;
      e = num ? (hi ? fmax(e, a) : fmin(e, a)) : e;
    }
    A.out[sym * A.ld_out + t] = (n >= A.minp && n > 0) ? e : qnan();
    return;
  }
  double v[N];
  int n = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double a = s[threadIdx.x + j];   // in bounds for every j < N; slots >= w are pads
    const bool num = j < w && a == a;
    n += num ? 1 : 0;
    v[j] = num ? a : __builtin_inf();
  }
  sort_network<N>(v);
  double r = qnan();
  if (n >= A.minp && n > 0) {
    if (A.mode == BQ_ROLL_MEDIAN) {
      const int h = n >> 1;
      r = (n & 1) ? pick(v, h) : (pick(v, h - 1) + pick(v, h)) / 2.0;
    } else if (n == 1) {
      r = v[0];
    } else {   // roll_quantile, linear interpolation (max / min: q = 1 / 0)
      const double idxf = A.q * (double)(n - 1);
      const int idx = (int)idxf;
      if ((double)idx == idxf || A.lower) r = pick(v, idx);
      else {
        const double lo = pick(v, idx), hi = pick(v, idx + 1);
        r = lo + (hi - lo) * (idxf - (double)idx);
      }
    }
  }
  A.out[sym * A.ld_out + t] = r;
}

}  // namespace bq

namespace {

bool job_ok(const bq_roll_job& j, int64_t S, int64_t T) {
  if (!j.x || !j.out || j.ld_in < T || j.ld_out < T || j.min_periods < 0) return false;
  // replay results leave through 32-bit buffer offsets over 64 rows
  if (j.ld_out > BQ_MAX_ROLL_LD) return false;
  // a job's own row count (a benchmark row beside the panel): the lane-per-row
  // kernels (moments, ewm) and the fill honour it; order statistics and the
  // integer sums walk the batch's S rows
  if (j.rows < 0 || j.rows > S) return false;
  const bool own_rows = j.rows != 0 && j.rows != S;
  if (own_rows && j.mode != BQ_ROLL_EWM && j.mode != BQ_ROLL_FFILL &&
      !(j.mode >= BQ_ROLL_MEAN && j.mode <= BQ_ROLL_STD0))
    return false;
  if (j.mode == BQ_ROLL_EWM) return j.alpha > 0.0 && j.alpha <= 1.0;
  if (j.mode == BQ_ROLL_FFILL) return j.shift == 0;
  return j.window >= 1 && j.window <= bq::RW_MAXW && j.shift >= 0 && j.shift <= bq::RW_MAXSHIFT &&
         ((j.mode >= BQ_ROLL_QUANTILE && j.mode <= BQ_ROLL_STD0) || j.mode == BQ_ROLL_ISUM ||
          j.mode == BQ_ROLL_QLOWER) && j.q >= 0.0 &&
         j.q <= 1.0;
}

int rank_bucket(int w) {
  return w <= 8 ? 0 : w <= 24 ? 1 : w <= 48 ? 2 : w <= 64 ? 3 : w <= 80 ? 4 : 5;
}

template <int W>
void launch_rank(const bq::RollBatch& B, int n, int64_t max_items, hipStream_t st) {
  const unsigned blocks = (unsigned)((max_items + 255) / 256);
  hipLaunchKernelGGL(bq::rank_kernel<W>, dim3(blocks, (unsigned)n), dim3(256), 0, st, B);
}

// slide kernel instantiations: (window, full-window rank K, median) of the
// strategies' defaults — ActivityBurstPump's 19-candle medians and
// quantile(0.92, 80), LiquidationSweepPump's quantile(0.80, 48),
// FailedSpikeFade's quantile(0.85, 60), the leadership's lower quantile
// (0.80, 96). At 12.5k x 2k on NaN-free rows (tools/slide_probe.py):
// 0.20 / 0.70 / 0.34 / 0.41 / 0.78 ms against the stencil / tile kernels'
// 0.28 / 0.73 / 0.60 / 0.60 / 0.82. Other (w, q) go to those kernels.
struct SlideCfg {
  int w, k, med;
};
#ifndef BQ_SLIDE_BIG
#define BQ_SLIDE_BIG 1   // 0: w = 80 / 96 on the tile kernel (measurement)
#endif
#ifndef BQ_SLIDE_PAIR_DEFAULT
#define BQ_SLIDE_PAIR_DEFAULT 80   // smallest window on slide_group_kernel (0: none)
#endif
#ifndef BQ_SLIDE_GROUP_DEFAULT
#define BQ_SLIDE_GROUP_DEFAULT 2   // lanes per window there
#endif
constexpr SlideCfg kSlide[] = {{19, 9, 1}, {48, 37, 0}, {60, 50, 0}
#if BQ_SLIDE_BIG
                               , {80, 72, 0}, {96, 76, 0}
#endif
};
constexpr int kNSlide = (int)(sizeof(kSlide) / sizeof(kSlide[0]));

int slide_variant(int w, int mode, double q) {
  for (int i = 0; i < kNSlide; ++i) {
    if (kSlide[i].w != w) continue;
    if (mode == BQ_ROLL_MEDIAN) {
      if (kSlide[i].med && kSlide[i].k == ((w & 1) ? w / 2 : w / 2 - 1)) return i;
    } else if (mode == BQ_ROLL_QUANTILE && !kSlide[i].med && q > 0.0 && q < 1.0 &&
               kSlide[i].k == (int)(q * (double)(w - 1))) {
      return i;
    }
  }
  return -1;
}

// segment length of a slide job: lanes = (symbol, segment), about
// BQ_SLIDE_WAVES waves per SIMD over 1024 SIMDs (the kernel is VALU-bound and
// every slot update is independent, so a few waves hide its loads); each
// segment replays W - 1 warm-up values, so segments stay >= 2 W
// lanes per window of the slide kernel: 1, or BQ_SLIDE_GROUP (2 / 4) for
// windows >= BQ_SLIDE_PAIR_MIN (0: never) — slide_group_kernel
int slide_pair_min() {
  static const int v = [] {
    const char* e = getenv("BQ_SLIDE_PAIR_MIN");
    return e ? atoi(e) : BQ_SLIDE_PAIR_DEFAULT;
  }();
  return v;
}
int slide_group(int w) {
  static const int g = [] {
    const char* e = getenv("BQ_SLIDE_GROUP");
    const int v = e ? atoi(e) : BQ_SLIDE_GROUP_DEFAULT;
    return v == 4 ? 4 : 2;
  }();
  return slide_pair_min() > 0 && w >= slide_pair_min() && w % g == 0 ? g : 1;
}

// Segments of a slide batch (lanes = (symbol, segment) x G lanes per window):
// enough for one round of the kernel's resident waves over the chip, whose
// occupancy comes from its registers (hipOccupancy..., per instantiation) —
// BQ_SLIDE_WAVES rounds (default 1). A second, partial round costs a whole
// segment's time: at 12.5k x 2k the a17 medians (two w = 19 series, 3 waves
// per SIMD) ran 0.40 ms over 10 segments (two rounds) against 0.34 over 5.
// Each segment replays W - 1 warm-up values, so segments stay >= 2 W.
int device_cus() {
  static const int cus = [] {
    int d = 0, c = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      c = 0;
    return c > 0 ? c : 256;
  }();
  return cus;
}
template <typename F>
int resident_waves(F kern) {   // 256-thread workgroups per CU = waves per SIMD
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, 0) != hipSuccess || nb < 1) nb = 1;
  return nb;
}
// ... and no more items in flight than the L2 holds their two streams
// (the entering chunk and the leaving one, `chunk` values each; a group's
// lanes share theirs): 32 MiB = 8 XCDs x 4 MiB. The w = 19 medians (16-value
// chunks) at 7 segments (175k lanes x 256 B > the L2) ran 0.43 ms, at 5
// (125k lanes) 0.34.
int64_t slide_segments(bq::RollBatch& B, int n, int w, int g, int occ, int chunk) {
  static const int rounds = [] {
    const char* e = getenv("BQ_SLIDE_WAVES");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 1;
  }();
  const int64_t l2_items = ((int64_t)32 << 20) / (2 * chunk * 8);
  int64_t items = (int64_t)device_cus() * 4 * occ * 64 * rounds / g;
  items = items < l2_items * rounds ? items : l2_items * rounds;
  const int64_t per = (B.S > 0 ? B.S : 1) * (int64_t)n;
  const int64_t nseg = items / per > 1 ? items / per : 1;
  const int64_t T = B.T;
  int64_t seg = (T + nseg - 1) / nseg;
  if (seg < 2 * w) seg = 2 * w;
  if (seg > T) seg = T > 0 ? T : 1;
  const int ns = (int)((T + seg - 1) / seg);
  for (int i = 0; i < n; ++i) {
    B.j[i].seg = (int)seg;
    B.j[i].nseg = ns;
  }
  return B.S * (int64_t)ns;
}

template <int W, int K, bool MED>
void launch_slide1(const bq::RollBatch& B0, int n, hipStream_t st, bool single) {
  bq::RollBatch B = B0;
  if (single) {   // the crossing-flag instantiation
    static const int occ = resident_waves(bq::slide_rank_kernel<W, K, MED, true>);
    const int64_t items = slide_segments(B, n, W, 1, occ, W <= 24 ? 16 : 8);
    const unsigned blocks = (unsigned)((items + 255) / 256);
    hipLaunchKernelGGL((bq::slide_rank_kernel<W, K, MED, true>), dim3(blocks, (unsigned)n), dim3(256), 0, st, B);
    return;
  }
  if constexpr (W % 4 == 0 && K / (W / 2) == (K + 1) / (W / 2) && K / (W / 4) == (K + 1) / (W / 4) && K + 1 < W) {
    const int g = slide_group(W);
    if (g == 2) {
      static const int occ = resident_waves(bq::slide_group_kernel<W, K, MED, 2>);
      const int64_t items = slide_segments(B, n, W, 2, occ, BQ_SG_C);
      const unsigned blocks = (unsigned)((2 * items + 255) / 256);
      hipLaunchKernelGGL((bq::slide_group_kernel<W, K, MED, 2>), dim3(blocks, (unsigned)n), dim3(256), 0, st, B);
      return;
    }
    if (g == 4) {
      static const int occ = resident_waves(bq::slide_group_kernel<W, K, MED, 4>);
      const int64_t items = slide_segments(B, n, W, 4, occ, BQ_SG_C);
      const unsigned blocks = (unsigned)((4 * items + 255) / 256);
      hipLaunchKernelGGL((bq::slide_group_kernel<W, K, MED, 4>), dim3(blocks, (unsigned)n), dim3(256), 0, st, B);
      return;
    }
  }
  static const int occ = resident_waves(bq::slide_rank_kernel<W, K, MED>);
  const int64_t items = slide_segments(B, n, W, 1, occ, W <= 24 ? 16 : 8);
  const unsigned blocks = (unsigned)((items + 255) / 256);
  hipLaunchKernelGGL((bq::slide_rank_kernel<W, K, MED>), dim3(blocks, (unsigned)n), dim3(256), 0, st, B);
}

// single: the one-lane kernel with the crossing flags (bq_rolling_quantile_cross)
void launch_slide(int v, const bq::RollBatch& B, int n, hipStream_t st, bool single = false) {
  switch (v) {
    case 0: launch_slide1<19, 9, true>(B, n, st, single); break;
    case 1: launch_slide1<48, 37, false>(B, n, st, single); break;
#if BQ_SLIDE_BIG
    case 3: launch_slide1<80, 72, false>(B, n, st, single); break;
    case 4: launch_slide1<96, 76, false>(B, n, st, single); break;
#endif
    default: launch_slide1<60, 50, false>(B, n, st, single);
  }
}
static_assert(kNSlide == 3 + 2 * BQ_SLIDE_BIG, "launch_slide covers every kSlide entry");

template <int EPL, int OPL, bool SEL, bool PACK>
void launch_tile_rank(const bq::RollBatch& B, int n, hipStream_t st) {
  const int64_t nt = (B.T + bq::WAVE * OPL - 1) / (bq::WAVE * OPL);
  const unsigned blocks = (unsigned)((B.S * nt + BQ_TR_WPB - 1) / BQ_TR_WPB);
  hipLaunchKernelGGL((bq::tile_rank_kernel<EPL, OPL, SEL, PACK>), dim3(blocks, (unsigned)n), dim3(64 * BQ_TR_WPB), 0,
                     st, B);
}

// panel-mode order statistics with packed keys (tile_rank_kernel PACK);
// BQ_RANK_PACK=0 keeps the full keys for them too (measurement)
bool rank_pack() {
  static const bool on = [] {
    const char* e = getenv("BQ_RANK_PACK");
    return !(e && e[0] == '0');
  }();
  return on;
}

// tile group of a job: 0 = 64-output tiles (w <= 65: union fits 128 slots),
// bit selection; 1 / 2 = 128-output tiles with selection for central ranks /
// the walk where the rank is near an end of the window (tile_rank_kernel)
int tile_group(int w, int mode, double q) {
  if (w <= 65) return 0;
  // BQ_TILE_SEL=1|0 forces selection / the walk for 128-output tiles (measurement)
  static const int forced = [] {
    const char* e = getenv("BQ_TILE_SEL");
    return e ? atoi(e) : -1;
  }();
  if (forced >= 0) return forced ? 1 : 2;
  // central ranks select (measured, tools/tile_sel_ab.sh: w 96 q 0.8 2.64 vs 3.27 ms
  // a call; w 80 q 0.92 2.70 vs 2.57 — the walk from the top end is short)
  const bool central = mode == BQ_ROLL_MEDIAN || (q >= 0.2 && q <= 0.8);
  return BQ_RANK_SEL && central ? 1 : 2;
}

// window buckets of the stencil kernel (network slots): a bucket of 20 for
// the strategies' 19-candle medians (103 comparators against 132 at 24)
int stencil_bucket(int w) { return w <= 4 ? 0 : w <= 8 ? 1 : w <= 16 ? 2 : w <= 20 ? 3 : w <= 24 ? 4 : 5; }

void launch_stencil(int b, const bq::RollBatch& B, int n, hipStream_t st) {
  const int64_t nbt = (B.T + bq::SR_NT - 1) / bq::SR_NT;
  const dim3 grid((unsigned)(B.S * nbt), (unsigned)n);
  switch (b) {
    case 0: hipLaunchKernelGGL(bq::stencil_rank_kernel<4>, grid, dim3(bq::SR_NT), 0, st, B); break;
    case 1: hipLaunchKernelGGL(bq::stencil_rank_kernel<8>, grid, dim3(bq::SR_NT), 0, st, B); break;
    case 2: hipLaunchKernelGGL(bq::stencil_rank_kernel<16>, grid, dim3(bq::SR_NT), 0, st, B); break;
    case 3: hipLaunchKernelGGL(bq::stencil_rank_kernel<20>, grid, dim3(bq::SR_NT), 0, st, B); break;
    case 4: hipLaunchKernelGGL(bq::stencil_rank_kernel<24>, grid, dim3(bq::SR_NT), 0, st, B); break;
    default: hipLaunchKernelGGL(bq::stencil_rank_kernel<32>, grid, dim3(bq::SR_NT), 0, st, B);
  }
}

// which replay kernel: 0 = LDS ring over the window (one launch, 64 symbols
// per wave), 1 = re-staged leaving values, one launch per class, 2 = re-staged,
// all classes in one launch. BQ_REPLAY_IMPL=ring|restage|mixed forces one
// (measurement; all give identical outputs).
int replay_impl(int nclasses, int64_t waves64) {
  static const int forced = [] {
    const char* e = getenv("BQ_REPLAY_IMPL");
    return !e ? -1
              : (strcmp(e, "ring") == 0      ? 0
                 : strcmp(e, "restage") == 0 ? 1
                 : strcmp(e, "mixed") == 0   ? 2
                                             : -1);
  }();
  if (forced >= 0) return forced;
  // mixed classes: one launch (measured, an A/B harness of rounds 1-2 (tools/replay_ab.sh, removed in round 3: git history), identical
  // digests: 1000 x 400 batch16 0.18 vs 0.33 ms per class; 12.5k x 2k
  // batch16 2.69 vs 2.87 ms — the classes' replays overlap instead of
  // running one after the other)
  (void)waves64;
  return nclasses > 1 ? 2 : 1;
}

// symbols per wave of the re-staged replays: 64. BQ_REPLAY_SPW=32|16|8
// forces fewer (measurement: spreading the rows over 2-4x as many waves did
// not shorten the replay even for small batches — ADX's 3 series over 12.5k
// symbols (588 waves of 64) took 1.12 ms at 64 and 1.49 ms at 16 symbols per
// wave: the step cost is the wave's own instruction stream, not a shortage of
// waves — an A/B harness of rounds 1-2 (tools/spw_ab.sh, removed in round 3: git history), an A/B harness of rounds 1-2 (tools/replay_ab.sh, removed in round 3: git history)).
int replay_spw(int64_t waves64) {
  static const int forced = [] {
    const char* e = getenv("BQ_REPLAY_SPW");
    const int v = e ? atoi(e) : 0;
    return (v == 32 || v == 16 || v == 8) ? v : 64;
  }();
  (void)waves64;
  return forced;
}

template <int SPW>
void launch_restage(int cls, const bq::RollBatch& B, int n, hipStream_t st) {
  const dim3 grid((unsigned)((B.S + SPW - 1) / SPW), (unsigned)n);
  switch (cls) {
    case 0: hipLaunchKernelGGL((bq::replay_restage_kernel<0, SPW>), grid, dim3(bq::WAVE), 0, st, B); break;
    case 1: hipLaunchKernelGGL((bq::replay_restage_kernel<1, SPW>), grid, dim3(bq::WAVE), 0, st, B); break;
    case 2: hipLaunchKernelGGL((bq::replay_restage_kernel<2, SPW>), grid, dim3(bq::WAVE), 0, st, B); break;
    case 3: hipLaunchKernelGGL((bq::replay_restage_kernel<3, SPW>), grid, dim3(bq::WAVE), 0, st, B); break;
    default: hipLaunchKernelGGL((bq::replay_mixed_kernel<SPW>), grid, dim3(bq::WAVE), 0, st, B);
  }
}

// cls 0-3: one class; 4: mixed
void launch_restage_any(int cls, const bq::RollBatch& B, int n, hipStream_t st) {
  switch (replay_spw((B.S + bq::WAVE - 1) / bq::WAVE * n)) {
    case 64: launch_restage<64>(cls, B, n, st); break;
    case 32: launch_restage<32>(cls, B, n, st); break;
    case 16: launch_restage<16>(cls, B, n, st); break;
    default: launch_restage<8>(cls, B, n, st);
  }
}

// which order-statistic kernel: 0 = lane (sorted window per lane), 1 = tile
// (sorted union per wave), 2 = stencil (sorting network per output, w <= 32).
// BQ_RANK_IMPL=lane|tile|stencil forces one (measurement; stencil falls back
// to tile above w = 32).
// BQ_RANK_SLIDE=0 keeps large panels on the tile kernel (measurement)
bool slide_on() {
  static const bool on = [] {
    const char* e = getenv("BQ_RANK_SLIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}

int rank_impl(int w, int64_t S, int64_t T, bool slide) {
  static const int forced = [] {
    const char* e = getenv("BQ_RANK_IMPL");
    return !e ? -1
              : (strcmp(e, "lane") == 0      ? 0
                 : strcmp(e, "tile") == 0    ? 1
                 : strcmp(e, "stencil") == 0 ? 2
                 : strcmp(e, "slide") == 0   ? 3
                                             : -1);
  }();
  if (forced == 3) return slide ? 3 : (w <= 32 ? 2 : 1);
  if (forced >= 0) return forced == 2 && w > 32 ? 1 : forced;
  // large panels with a slide instantiation: the sorted-register window
  // (5 VALU per slot and step, against the tile kernel's sort per 64
  // outputs); live shapes keep the tile / stencil kernels (no warm-up)
  if (slide && S * T >= (int64_t)(1 << 22) && T >= 4 * (int64_t)w && slide_on()) return 3;
  // short windows: the stencil kernel (coalesced, no warm-up, no per-lane row
  // walk); longer ones: the tile kernel, whose sort is shared by 64 / 128
  // outputs (the lane kernel stays selectable for measurement)
  return w <= 32 ? 2 : 1;
}

}  // namespace

extern "C" {

int bq_rolling_batch(const bq_roll_job* jobs, int32_t n_jobs, int64_t S, int64_t T, void* stream) {
  return bq_rolling_batch_cross(jobs, n_jobs, S, T, nullptr, nullptr, stream);
}

int bq_rolling_batch_cross(const bq_roll_job* jobs, int32_t n_jobs, int64_t S, int64_t T, uint8_t* const* cross,
                           const int64_t* ld_cross, void* stream) {
  using namespace bq;
  if (!jobs || n_jobs < 0 || S < 0 || T < 0 || T > 0x7fffffff) return BQ_EINVAL;
  for (int i = 0; i < n_jobs; ++i) {
    if (!job_ok(jobs[i], S, T)) return BQ_EINVAL;
    if (cross && cross[i] && (jobs[i].mode != BQ_ROLL_QUANTILE || jobs[i].rows > 0 || !ld_cross || ld_cross[i] < T))
      return BQ_EINVAL;
  }
  if (S == 0 || T == 0 || n_jobs == 0) return BQ_OK;
  hipStream_t st = (hipStream_t)stream;
  // crossing flags: the slide variants that carry a flag job launch the
  // flag instantiation (one lane per window); elsewhere a flag pass follows
  bool slide_xc[kNSlide] = {};
  for (int i = 0; i < n_jobs; ++i)
    if (cross && cross[i]) {
      const int sv = slide_variant(jobs[i].window, jobs[i].mode, jobs[i].q);
      if (sv >= 0 && rank_impl(jobs[i].window, S, T, true) == 3) slide_xc[sv] = true;
    }
  int nxp = 0;
  int xpass[BQ_MAX_ROLL_JOBS];
  // replay jobs (moments, ewm): lane = symbol; rank jobs grouped by window size
  RollBatch rep;
  memset(&rep, 0, sizeof(rep));
  rep.S = S;
  rep.T = (int)T;
  int nrep = 0;
  RollBatch rank[6];
  int nrank[6] = {0, 0, 0, 0, 0, 0};
  int64_t rank_items[6] = {0, 0, 0, 0, 0, 0};
  for (int b = 0; b < 6; ++b) {
    memset(&rank[b], 0, sizeof(RollBatch));
    rank[b].S = S;
    rank[b].T = (int)T;
  }
  int max_back = 0;   // window + shift of the replay jobs in the batch
  auto flush_rep = [&]() {
    if (!nrep) return;
    const int ring = (max_back + RP_CT - 1) / RP_CT + 1;
    const size_t lds = (size_t)ring * RP_CT * STG_PITCH * sizeof(double);
    // > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU): set once, before
    // any graph capture can be active (first call of the process)
    static const bool lds_opt_in =
        hipFuncSetAttribute((const void*)replay_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==
        hipSuccess;
    (void)lds_opt_in;
    // re-staging kernels: class-specialised when the batch has one class,
    // the mixed kernel otherwise (the LDS ring kernel only when forced;
    // measured: an A/B harness of rounds 1-2 (tools/replay_ab.sh, removed in round 3: git history), identical outputs)
    int ncls[4] = {0, 0, 0, 0};
    for (int i = 0; i < nrep; ++i) ++ncls[replay_class(rep.j[i].mode)];
    const int nclasses = (ncls[0] > 0) + (ncls[1] > 0) + (ncls[2] > 0) + (ncls[3] > 0);
    const int impl = replay_impl(nclasses, ((S + WAVE - 1) / WAVE) * nrep);
    if (impl == 1) {
      RollBatch cls[4];
      for (int c = 0; c < 4; ++c) {
        memset(&cls[c], 0, sizeof(RollBatch));
        cls[c].S = S;
        cls[c].T = (int)T;
        ncls[c] = 0;
      }
      for (int i = 0; i < nrep; ++i) {
        const int c = replay_class(rep.j[i].mode);
        cls[c].j[ncls[c]++] = rep.j[i];
      }
      for (int c = 0; c < 4; ++c)
        if (ncls[c]) launch_restage_any(c, cls[c], ncls[c], st);
    } else if (impl == 2) {
      // longest first: blocks start in blockIdx order (x, then the job), so
      // the costliest replays (Welford, ~3x a Kahan step) go to the front of
      // the grid instead of starting in its tail (outputs are per job)
      if (BQ_RS_LPT) {
        RollJob sorted[RW_MAXJOBS];
        int n = 0;
        for (int c : {2, 1, 0, 3})
          for (int i = 0; i < nrep; ++i)
            if (replay_class(rep.j[i].mode) == c) sorted[n++] = rep.j[i];
        for (int i = 0; i < nrep; ++i) rep.j[i] = sorted[i];
      }
      launch_restage_any(4, rep, nrep, st);
    } else {
      hipLaunchKernelGGL(replay_kernel, dim3((unsigned)((S + WAVE - 1) / WAVE), (unsigned)nrep), dim3(WAVE), lds, st,
                         rep, ring);
    }
    nrep = 0;
    max_back = 0;
  };
  auto flush_rank = [&](int b) {
    if (!nrank[b]) return;
    switch (b) {
      case 0: launch_rank<8>(rank[b], nrank[b], rank_items[b], st); break;
      case 1: launch_rank<24>(rank[b], nrank[b], rank_items[b], st); break;
      case 2: launch_rank<48>(rank[b], nrank[b], rank_items[b], st); break;
      case 3: launch_rank<64>(rank[b], nrank[b], rank_items[b], st); break;
      case 4: launch_rank<80>(rank[b], nrank[b], rank_items[b], st); break;
      default: launch_rank<96>(rank[b], nrank[b], rank_items[b], st);
    }
    nrank[b] = 0;
    rank_items[b] = 0;
  };
  RollBatch tile[6];   // tile group + 3 for panel-mode (packed-key) jobs
  int ntile[6] = {0, 0, 0, 0, 0, 0};
  for (int g = 0; g < 6; ++g) {
    memset(&tile[g], 0, sizeof(RollBatch));
    tile[g].S = S;
    tile[g].T = (int)T;
  }
  auto flush_tile = [&](int g) {
    if (!ntile[g]) return;
    switch (g) {
      case 0: launch_tile_rank<2, 1, BQ_RANK_SEL != 0, false>(tile[g], ntile[g], st); break;
      case 1: launch_tile_rank<4, 2, true, false>(tile[g], ntile[g], st); break;
      case 2: launch_tile_rank<4, 2, false, false>(tile[g], ntile[g], st); break;
      case 3: launch_tile_rank<2, 1, BQ_RANK_SEL != 0, true>(tile[g], ntile[g], st); break;
      case 4: launch_tile_rank<4, 2, true, true>(tile[g], ntile[g], st); break;
      default: launch_tile_rank<4, 2, false, true>(tile[g], ntile[g], st);
    }
    ntile[g] = 0;
  };
  RollBatch slide[kNSlide];
  int nslide[kNSlide] = {};

  for (int v = 0; v < kNSlide; ++v) {
    memset(&slide[v], 0, sizeof(RollBatch));
    slide[v].S = S;
    slide[v].T = (int)T;
  }
  auto flush_slide = [&](int v) {
    if (!nslide[v]) return;
    launch_slide(v, slide[v], nslide[v], st, slide_xc[v]);   // segments set there
    nslide[v] = 0;
  };
  RollBatch ff;
  memset(&ff, 0, sizeof(ff));
  ff.S = S;
  ff.T = (int)T;
  int nff = 0;
  auto flush_ff = [&]() {
    if (!nff) return;
    int vec = 1;   // 16-byte output rows: whole-line stores
    for (int i = 0; i < nff; ++i)
      vec &= (ff.j[i].ld_out % 2) == 0 && (((uintptr_t)ff.j[i].out) & 15u) == 0;
    hipLaunchKernelGGL(ffill_kernel, dim3((unsigned)S, (unsigned)nff), dim3(FF_NT), 0, st, ff, vec);
    nff = 0;
  };
  RollBatch sten[6];
  int nsten[6] = {0, 0, 0, 0, 0, 0};
  for (int b = 0; b < 6; ++b) {
    memset(&sten[b], 0, sizeof(RollBatch));
    sten[b].S = S;
    sten[b].T = (int)T;
  }
  auto flush_sten = [&](int b) {
    if (!nsten[b]) return;
    launch_stencil(b, sten[b], nsten[b], st);
    nsten[b] = 0;
  };
  PanelBatch pan;
  memset(&pan, 0, sizeof(pan));
  pan.S = S;
  pan.T = (int)T;
  int npan = 0;
  auto flush_pan = [&]() {
    if (!npan) return;
    launch_panel(pan, npan, st);
    npan = 0;
  };
  for (int i = 0; i < n_jobs; ++i) {
    const bq_roll_job& in = jobs[i];
    if (in.panel && panel_supported(in.mode, in.window, in.shift)) {   // time-parallel (bq_panel.hip)
      PanelJob& P = pan.j[npan++];
      P.x = in.x;
      P.out = in.out;
      P.ld_in = in.ld_in;
      P.ld_out = in.ld_out;
      P.rows = in.rows > 0 ? in.rows : S;
      P.win = in.window;
      P.minp = in.min_periods;
      P.shift = in.shift;
      P.mode = in.mode;
      P.alpha = in.alpha;
      P.hi = P.lo = nullptr;
      if (npan == PN_MAXJOBS) flush_pan();
      continue;
    }
    RollJob J;
    memset(&J, 0, sizeof(J));
    const bool want_x = cross && cross[i];
    J.x = in.x;
    J.out = in.out;
    J.ld_in = in.ld_in;
    J.ld_out = in.ld_out;
    J.win = in.window;
    J.minp = in.min_periods;
    J.shift = in.shift;
    J.mode = in.mode;
    J.q = in.q;
    J.alpha = in.alpha;
    J.rows = in.rows > 0 ? in.rows : S;
    if (J.mode == BQ_ROLL_QLOWER) {   // an order statistic like the quantile, no interpolation
      J.mode = BQ_ROLL_QUANTILE;
      J.lower = 1;
    }
    if (J.mode == BQ_ROLL_FFILL) {   // a scan, not a replay (ffill_kernel)
      ff.j[nff++] = J;
      if (nff == RW_MAXJOBS) flush_ff();
      continue;
    }
    if (in.mode == BQ_ROLL_ISUM && (in.window > 32 || S * ((T + SR_NT - 1) / SR_NT) > 0x7fffffff))
      J.mode = BQ_ROLL_SUM;   // long window: the replay (identical values for integer series)
    if (J.mode == BQ_ROLL_ISUM) {   // integer-valued sum: a direct window sum, stencil launch
      const int b = stencil_bucket(in.window);
      sten[b].j[nsten[b]++] = J;
      if (nsten[b] == RW_MAXJOBS) flush_sten(b);
    } else if (J.mode >= BQ_ROLL_MEAN) {   // moments / ewm: exact replay
      const int back = (J.mode == BQ_ROLL_EWM || J.mode == BQ_ROLL_FFILL) ? 0 : in.window + in.shift;
      max_back = back > max_back ? back : max_back;
      rep.j[nrep++] = J;
      if (nrep == RW_MAXJOBS) flush_rep();
    } else if (const int sv = slide_variant(in.window, J.mode, J.q);
               rank_impl(in.window, S, T, sv >= 0) == 3) {
      if (want_x) {
        J.cross = cross[i];
        J.ld_cross = ld_cross[i];
      }
      slide[sv].j[nslide[sv]++] = J;
      if (nslide[sv] == RW_MAXJOBS) flush_slide(sv);
    } else if (rank_impl(in.window, S, T, false) == 2 && S * ((T + SR_NT - 1) / SR_NT) <= 0x7fffffff) {
      const int b = stencil_bucket(in.window);
      sten[b].j[nsten[b]++] = J;
      if (nsten[b] == RW_MAXJOBS) flush_sten(b);
    } else if (rank_impl(in.window, S, T, false) >= 1) {
      const int g = tile_group(in.window, in.mode, in.q) + (in.panel && rank_pack() ? 3 : 0);
      tile[g].j[ntile[g]++] = J;
      if (ntile[g] == RW_MAXJOBS) flush_tile(g);
    } else {
      // segments: lanes = (symbol, segment). Enough lanes to fill the SIMDs to
      // the kernel's occupancy (waves per SIMD set by the window's register
      // footprint), but no more than ~80k-130k: every lane streams its own
      // row lines through L2, and beyond that the lines are evicted before
      // their 16 values are used (measured: tools/segx.py sweep). Each
      // segment re-reads one window of warm-up values.
      static const int occ[6] = {8, 6, 3, 2, 2, 1};   // rank_kernel<8,24,48,64,80,96>
      static const int64_t cap[6] = {80000, 80000, 100000, 131072, 131072, 65536};
      const int b0 = rank_bucket(in.window);
      int64_t lanes = (int64_t)1024 * occ[b0] * WAVE;
      lanes = lanes < cap[b0] ? lanes : cap[b0];
      const int64_t nseg_t = lanes / S > 1 ? lanes / S : 1;
      int seg = (int)((T + nseg_t - 1) / nseg_t);
      seg = seg < in.window ? in.window : seg;
      J.seg = seg;
      J.nseg = (int)((T + seg - 1) / seg);
      const int b = rank_bucket(in.window);
      rank[b].j[nrank[b]++] = J;
      const int64_t items = S * (int64_t)J.nseg;
      rank_items[b] = items > rank_items[b] ? items : rank_items[b];
      if (nrank[b] == RW_MAXJOBS) flush_rank(b);
    }
    if (want_x && !J.cross) xpass[nxp++] = i;   // not on the slide kernel: a flag pass after
  }
  flush_pan();
  flush_rep();
  flush_ff();
  for (int b = 0; b < 6; ++b) flush_rank(b);
  for (int g = 0; g < 6; ++g) flush_tile(g);
  for (int v = 0; v < kNSlide; ++v) flush_slide(v);
  for (int b = 0; b < 6; ++b) flush_sten(b);
  for (int u = 0; u < nxp; ++u) {
    const bq_roll_job& in = jobs[xpass[u]];
    const int64_t n = S * T;
    hipLaunchKernelGGL(cross_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in.x, in.out, S, (int)T,
                       in.ld_in, in.ld_out, cross[xpass[u]], ld_cross[xpass[u]]);
  }
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_rolling(const double* x, int64_t S, int64_t T, int64_t ld_in, int32_t window, int32_t min_periods,
               int32_t shift, int32_t mode, double q, double* out, int64_t ld_out, void* stream) {
  if ((mode < BQ_ROLL_QUANTILE || mode > BQ_ROLL_STD0) && mode != BQ_ROLL_ISUM && mode != BQ_ROLL_QLOWER)
    return BQ_EINVAL;
  bq_roll_job j;
  memset(&j, 0, sizeof(j));
  j.x = x;
  j.out = out;
  j.ld_in = ld_in;
  j.ld_out = ld_out;
  j.window = window;
  j.min_periods = min_periods;
  j.shift = shift;
  j.mode = mode;
  j.q = q;
  return bq_rolling_batch(&j, 1, S, T, stream);
}

int bq_rolling_quantile_cross(const double* x, int64_t S, int64_t T, int64_t ld_in, int32_t window,
                              int32_t min_periods, int32_t shift, double q, double* out, int64_t ld_out,
                              uint8_t* cross, int64_t ld_cross, void* stream) {
  if (!cross) return BQ_EINVAL;
  bq_roll_job j;
  memset(&j, 0, sizeof(j));
  j.x = x;
  j.out = out;
  j.ld_in = ld_in;
  j.ld_out = ld_out;
  j.window = window;
  j.min_periods = min_periods;
  j.shift = shift;
  j.mode = BQ_ROLL_QUANTILE;
  j.q = q;
  return bq_rolling_batch_cross(&j, 1, S, T, &cross, &ld_cross, stream);
}

int bq_ewm(const double* x, int64_t S, int64_t T, int64_t ld_in, double alpha, int32_t min_periods, double* out,
           int64_t ld_out, void* stream) {
  bq_roll_job j;
  memset(&j, 0, sizeof(j));
  j.x = x;
  j.out = out;
  j.ld_in = ld_in;
  j.ld_out = ld_out;
  j.min_periods = min_periods;
  j.mode = BQ_ROLL_EWM;
  j.alpha = alpha;
  return bq_rolling_batch(&j, 1, S, T, stream);
}

}  // extern "C"
