// Sequential per-symbol state machines on a [S][T] panel (lane = symbol).
//
//   bq_supertrend: pybinbot Indicators.set_supertrend(df, multiplier=3.0) as
//   called by Coinrule.supertrend_swing_reversal
//   (strategies/coinrule/coinrule.py:140-160, "period adjusted to 10"), which
//   reads bool(df["supertrend"].iloc[-1]). pybinbot is absent, so
//   the recurrence is the restatement in oracle/indicators_ref.py:supertrend:
//     hl2 = (high + low) / 2; upper = hl2 + m * ATR; lower = hl2 - m * ATR
//     trend[0] = up; for t >= 1:
//       close[t] > upper[t-1] -> up;  close[t] < lower[t-1] -> down;
//       otherwise keep the trend, and hold the band on the trend's side
//       (up: lower[t] = max(lower[t], lower[t-1]); down: upper[t] =
//       min(upper[t], upper[t-1])).
//   ATR = TR.rolling(period).mean(): bq_supertrend takes it as an input column;
//   bq_supertrend_hlc forms it in the same walk, replaying pandas' roll_mean
//   (pandas/_libs/window/aggregations.pyx add_mean / remove_mean / calc_mean,
//   pandas 2.3.3: Kahan sums with separate add / remove compensations, the
//   same-value and sign rules, min_periods = period) on the lane's own TR
//   sequence, so its ATR and bands are pandas' bit for bit. NaN bands in the
//   warm-up compare false, so the trend holds its initial `up` state.
//
// Mapping: one wave = 64 symbols; chunks of ST_CT candles are read coalesced
// and transposed through LDS (bq_device.h stage_*); the next chunk's loads are
// in flight while the current chunk's recurrence runs, and the chunk's steps
// are unrolled so the state-independent work (LDS reads, TR, hl2) of later
// steps overlaps the dependent chain of earlier ones. The TR values still in
// the window sit in an LDS ring (period + 16 slots, lane-contiguous).
#include "bq_device.h"
#include "binquant_amd.h"

#include <stdlib.h>

namespace bq {

#ifndef BQ_ST_CT
#define BQ_ST_CT 8
#endif
// candles per staged chunk (the global loads in flight per wave): 8 measured
// 0.836 ms against 0.880 at 16 and 0.910 at 4 (12.5k x 2k, an A/B harness of rounds 1-2 (tools/st_ab.sh, removed in round 3: git history)) —
// the loading wave's prefetch registers shrink by half and the band wave
// starts a chunk sooner
constexpr int ST_CT = BQ_ST_CT;
#ifndef BQ_ST_SUB
#define BQ_ST_SUB 8
#endif
constexpr int ST_SUB = BQ_ST_SUB;   // candles per register sub-chunk of the sequential part

struct StArgs {
  const double *h, *l, *c, *atr;
  uint8_t* up;
  double *upper, *lower;
  int64_t S, ld_in, ld_out;
  int T, period, ring;   // ring: TR slots per lane (period + ST_SUB)
  int warm;              // panel mode: warm-up candles before a chunk
  double mult, inv_period;
};

// pandas roll_mean state for a fixed window with min_periods = window. The
// NaN skips and the result rules are selects, not branches: the walk runs
// one wave per SIMD, where every exec-mask branch is paid in full each step.
struct AtrMean {
  double sum, comp_add, comp_rem, prev;
  int nobs, neg, same;
  __device__ __forceinline__ void add(double v) {
    const bool ok = v == v;
    const double y = v - comp_add;
    const double t = sum + y;
    const double c = t - sum - y;
    sum = ok ? t : sum;
    comp_add = ok ? c : comp_add;
    nobs += ok;
    neg += ok & (bool)signbit(v);
    same = ok ? ((v == prev) ? same + 1 : 1) : same;
    prev = ok ? v : prev;
  }
  __device__ __forceinline__ void remove(double v) {
    const bool ok = v == v;
    const double y = -v - comp_rem;
    const double t = sum + y;
    const double c = t - sum - y;
    sum = ok ? t : sum;
    comp_rem = ok ? c : comp_rem;
    nobs -= ok;
    neg -= ok & (bool)signbit(v);
  }
  // min_periods = window: a value exists only at nobs == window, so the
  // quotient is always sum / window (div_count: IEEE-exact, 3 fp64 ops)
  __device__ __forceinline__ double value(int minp, double wd, double inv_w) const {
    const double r = div_count(sum, wd, inv_w);
    double o = same >= nobs ? prev : r;
    o = ((same < nobs) & (((neg == 0) & (r < 0.0)) | ((neg == nobs) & (r > 0.0)))) ? 0.0 : o;
    return ((nobs < minp) | (nobs <= 0)) ? qnan() : o;
  }
};

// FATR: the ATR is formed here from high / low / close (bq_supertrend_hlc);
// otherwise it is the fourth input column. Per chunk the lane first pulls its
// symbol's candles out of the staging buffer into registers 16 at a time,
// forms their 16 TRs, appends them to the ring and reads back the 16 leaving
// the window (ring of period + 16 slots, so the appends never overwrite one
// still to leave): the sequential part then runs on registers only, and the Kahan
// chain of step j + 1 overlaps the division and band logic of step j.
template <bool FATR>
__global__ __launch_bounds__(WAVE) void supertrend_kernel(const StArgs A) {
  extern __shared__ double sTR[];               // FATR: TR ring [ring][WAVE]
  __shared__ double sX[4][ST_CT * STG_PITCH];   // h, l, c, atr; then upper, lower, trend
  constexpr int NIN = FATR ? 3 : 4;
  const int lane = threadIdx.x;
  const int64_t sym0 = (int64_t)blockIdx.x * WAVE;
  const int T = A.T;
  const int P = A.period, R = A.ring;
  const double pd = (double)P;
  const double* const in[4] = {A.h, A.l, A.c, A.atr};
  double r[4][ST_CT];
#pragma unroll
  for (int f = 0; f < NIN; ++f) stage_load<ST_CT>(in[f], A.ld_in, sym0, A.S, 0, T, lane, r[f]);
  bool up = true;
  double up_p = qnan(), lo_p = qnan(), pc = qnan();   // NaN bands before candle 0
  AtrMean m{0.0, 0.0, 0.0, 0.0, 0, 0, 0};
  int wslot = 0, rslot = FATR ? R - P : 0;   // ring slots of candle t0 and of candle t0 - P
  for (int t0 = 0; t0 < T; t0 += ST_CT) {
#pragma unroll
    for (int f = 0; f < NIN; ++f) stage_put<ST_CT>(sX[f], lane, r[f]);
    __syncthreads();
    // prefetch the next chunk (unconditional: past T the clamped loads give
    // NaN that is never used; no branch keeps the loop's waits counted)
#pragma unroll
    for (int f = 0; f < NIN; ++f) stage_load<ST_CT>(in[f], A.ld_in, sym0, A.S, t0 + ST_CT, T, lane, r[f]);
#pragma unroll
    for (int j0 = 0; j0 < ST_CT; j0 += ST_SUB) {
      const int u0 = t0 + j0;
      double h[ST_SUB], l[ST_SUB], c[ST_SUB], atr[ST_SUB];
#pragma unroll
      for (int j = 0; j < ST_SUB; ++j) {
        const int i = (j0 + j) * STG_PITCH + lane;
        h[j] = sX[0][i];
        l[j] = sX[1][i];
        c[j] = sX[2][i];
        if (!FATR) atr[j] = sX[3][i];
      }
      if (FATR) {
        double tr[ST_SUB], old[ST_SUB];
#pragma unroll
        for (int j = 0; j < ST_SUB; ++j) {
          tr[j] = true_range(h[j], l[j], j == 0 ? pc : c[j - 1]);
          const int ws = wslot + j >= R ? wslot + j - R : wslot + j;
          sTR[ws * WAVE + lane] = tr[j];
        }
        // (one wave: its LDS reads see its own earlier writes)
#pragma unroll
        for (int j = 0; j < ST_SUB; ++j) {
          const int rs = rslot + j >= R ? rslot + j - R : rslot + j;
          old[j] = u0 + j >= P ? sTR[rs * WAVE + lane] : qnan();   // NaN: nothing leaves
        }
        pc = c[ST_SUB - 1];
        wslot = wslot + ST_SUB >= R ? wslot + ST_SUB - R : wslot + ST_SUB;
        rslot = rslot + ST_SUB >= R ? rslot + ST_SUB - R : rslot + ST_SUB;
#pragma unroll
        for (int j = 0; j < ST_SUB; ++j) {
          if (u0 + j < T) {   // pandas: the removal, then the add, then calc_mean
            m.remove(old[j]);
            m.add(tr[j]);
            atr[j] = m.value(P, pd, A.inv_period);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < ST_SUB; ++j) {
        if (u0 + j < T) {   // wave-uniform: the last chunk may be partial
          const double hl2 = (h[j] + l[j]) / 2.0;
          const double m_atr = A.mult * atr[j];
          double bu = hl2 + m_atr, bl = hl2 - m_atr;
          // (t == 0: the NaN previous bands compare false and hold `up`)
          const bool flip_up = c[j] > up_p, flip_dn = !flip_up & (c[j] < lo_p), hold = !flip_up & !flip_dn;
          up = flip_up | (!flip_dn & up);
          bl = (hold & up & (bl < lo_p)) ? lo_p : bl;
          bu = (hold & !up & (bu > up_p)) ? up_p : bu;
          up_p = bu;
          lo_p = bl;
          const int i = (j0 + j) * STG_PITCH + lane;
          sX[0][i] = bu;
          sX[1][i] = bl;
          sX[2][i] = up ? 1.0 : 0.0;
        }
      }
    }
    __syncthreads();
    stage_store<ST_CT>(sX[0], A.upper, A.ld_out, sym0, A.S, t0, T, lane);   // null: dropped
    stage_store<ST_CT>(sX[1], A.lower, A.ld_out, sym0, A.S, t0, T, lane);
    stage_store<ST_CT>(sX[2], A.up, A.ld_out, sym0, A.S, t0, T, lane);
    __syncthreads();
  }
}

// bq_supertrend_hlc as a two-wave pipeline per 64 symbols: the walk is bound
// per wave (its time is flat from 1 024 to 16 384 symbols; ablation at
// 12.5k x 2k — 1.0 ms whole, 0.60 without the ATR replay, 0.83 without the
// stores), so its per-step work is split over two waves on two SIMDs
// (0.95 -> 0.88 ms: what is left is the latency of each chunk's loads with
// only 196 waves' worth of loads in flight). Wave 0
// stages chunk n (loads, LDS transpose), forms its TRs and replays pandas'
// roll_mean into sAtr; wave 1 runs the band / trend recursion on chunk n - 1
// from the same LDS tiles, writes the results in place and streams them out.
// Three barriers per chunk; both waves pass every one of them.
__global__ __launch_bounds__(2 * WAVE) void supertrend_pipe_kernel(const StArgs A) {
  // dynamic LDS (> 64 KiB at the largest periods): two chunk buffers of
  // h, l, c (wave 1 overwrites them with upper, lower, trend), two ATR
  // tiles, then the TR ring [ring][WAVE] of wave 0
  extern __shared__ double smem[];
  constexpr int TL = ST_CT * STG_PITCH;
  double(*sIn)[3][TL] = reinterpret_cast<double(*)[3][TL]>(smem);
  double(*sAtr)[TL] = reinterpret_cast<double(*)[TL]>(smem + 6 * TL);
  double* sTR = smem + 8 * TL;
  const int wv = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const int64_t sym0 = (int64_t)blockIdx.x * WAVE;
  const int T = A.T;
  const int P = A.period, R = A.ring;
  const double pd = (double)P;
  const double* const in[3] = {A.h, A.l, A.c};
  const int nch = (T + ST_CT - 1) / ST_CT;
  // wave 0 state
  double r[3][ST_CT];
  double pc = qnan();
  AtrMean m{0.0, 0.0, 0.0, 0.0, 0, 0, 0};
  int wslot = 0, rslot = R - P;
  // wave 1 state
  bool up = true;
  double up_p = qnan(), lo_p = qnan();   // NaN bands before candle 0
  if (wv == 0) {
#pragma unroll
    for (int f = 0; f < 3; ++f) stage_load<ST_CT>(in[f], A.ld_in, sym0, A.S, 0, T, lane, r[f]);
  }
  for (int n = 0; n <= nch; ++n) {
    const int b = n & 1, b1 = b ^ 1;
    if (wv == 0 && n < nch) {
#pragma unroll
      for (int f = 0; f < 3; ++f) stage_put<ST_CT>(sIn[b][f], lane, r[f]);
    }
    __syncthreads();
    if (wv == 0) {
      if (n < nch) {
        const int t0 = n * ST_CT;
#pragma unroll
        for (int f = 0; f < 3; ++f) stage_load<ST_CT>(in[f], A.ld_in, sym0, A.S, t0 + ST_CT, T, lane, r[f]);
#pragma unroll
        for (int j0 = 0; j0 < ST_CT; j0 += ST_SUB) {
          double tr[ST_SUB], old[ST_SUB], c[ST_SUB];
#pragma unroll
          for (int j = 0; j < ST_SUB; ++j) {
            const int i = (j0 + j) * STG_PITCH + lane;
            c[j] = sIn[b][2][i];
            tr[j] = true_range(sIn[b][0][i], sIn[b][1][i], j == 0 ? pc : c[j - 1]);
            const int ws = wslot + j >= R ? wslot + j - R : wslot + j;
            sTR[ws * WAVE + lane] = tr[j];
          }
#pragma unroll
          for (int j = 0; j < ST_SUB; ++j) {
            const int rs = rslot + j >= R ? rslot + j - R : rslot + j;
            old[j] = t0 + j0 + j >= P ? sTR[rs * WAVE + lane] : qnan();   // NaN: nothing leaves
          }
          pc = c[ST_SUB - 1];
          wslot = wslot + ST_SUB >= R ? wslot + ST_SUB - R : wslot + ST_SUB;
          rslot = rslot + ST_SUB >= R ? rslot + ST_SUB - R : rslot + ST_SUB;
#pragma unroll
          for (int j = 0; j < ST_SUB; ++j) {
            if (t0 + j0 + j < T) {   // pandas: the removal, then the add, then calc_mean
              m.remove(old[j]);
              m.add(tr[j]);
              sAtr[b][(j0 + j) * STG_PITCH + lane] = m.value(P, pd, A.inv_period);
            }
          }
        }
      }
    } else if (n >= 1) {
      const int t0 = (n - 1) * ST_CT;
#pragma unroll
      for (int j = 0; j < ST_CT; ++j) {
        if (t0 + j < T) {
          const int i = j * STG_PITCH + lane;
          const double h = sIn[b1][0][i], l = sIn[b1][1][i], c = sIn[b1][2][i];
          const double hl2 = (h + l) / 2.0;
          const double m_atr = A.mult * sAtr[b1][i];
          double bu = hl2 + m_atr, bl = hl2 - m_atr;
          const bool flip_up = c > up_p, flip_dn = !flip_up & (c < lo_p), hold = !flip_up & !flip_dn;
          up = flip_up | (!flip_dn & up);
          bl = (hold & up & (bl < lo_p)) ? lo_p : bl;
          bu = (hold & !up & (bu > up_p)) ? up_p : bu;
          up_p = bu;
          lo_p = bl;
          sIn[b1][0][i] = bu;
          sIn[b1][1][i] = bl;
          sIn[b1][2][i] = up ? 1.0 : 0.0;
        }
      }
    }
    __syncthreads();
    if (wv == 1 && n >= 1) {
      const int t0 = (n - 1) * ST_CT;
      stage_store<ST_CT>(sIn[b1][0], A.upper, A.ld_out, sym0, A.S, t0, T, lane);   // null: dropped
      stage_store<ST_CT>(sIn[b1][1], A.lower, A.ld_out, sym0, A.S, t0, T, lane);
      stage_store<ST_CT>(sIn[b1][2], A.up, A.ld_out, sym0, A.S, t0, T, lane);
    }
    __syncthreads();
  }
}

// ---- panel mode: a row per workgroup, chunk walks with verified starts ----
// The band / trend recursion only remembers (trend, upper, lower), and two
// walks started from different states meet as soon as both reset their bands
// (a flip, or close beyond the raw band) — in practice within a few dozen
// candles (0.44 % of 96-candle warm-ups end in a different state
// on random-walk panels, 0.07 % at 128). So one 256-thread workgroup takes
// one symbol's row (T <= STP_MAXT, held in LDS) and thread k the chunk
// [kC, kC + C) (C = ceil(T / 256) <= 8): it walks from STP_W candles before
// the chunk, starting from the series-start state (NaN bands, up), keeps the
// state it reaches at the chunk start (its guess), and its chunk's results in
// registers. Chunk k is exact iff its guess equals chunk k - 1's end state
// (chunk 0 starts at the true start, and so does every thread whose warm-up
// reaches candle 0): all threads compare in parallel, every mismatching chunk
// re-walks from its predecessor's end state, and the round repeats until no
// guess differs (each round fixes at least the first wrong chunk; one round
// in practice). The flags and bands therefore equal the sequential recursion
// on the same ATR.
// ATR: per candle, the period's TR values summed directly in time order
// (pandas' min_periods = period and same-value rule) — a pure function of the
// window, equal to pandas' Kahan roll_mean to rounding, not bit for bit (exact
// mode keeps the replay).
// LDS: close and the raw bands (hl2 and TR on the way), one pad slot per 32
// candles so the threads' strided walk positions spread over the banks.
constexpr int STP_NT = 256;
constexpr int STP_W = 96;
constexpr int STP_MAXT = 2048;
constexpr int STP_MAXC = STP_MAXT / STP_NT;   // 8 candles per thread
__host__ __device__ __forceinline__ int stp_slot(int t) { return t + (t >> 5); }
__device__ __forceinline__ bool same_bits(double a, double b) { return a == b || (a != a && b != b); }

__device__ __forceinline__ void st_step(bool& up, double& U, double& L, double c, double bu, double bl) {
  // (the NaN bands of the warm-up compare false and hold `up`)
  const bool flip_up = c > U, flip_dn = !flip_up & (c < L), hold = !flip_up & !flip_dn;
  up = flip_up | (!flip_dn & up);
  bl = (hold & up & (bl < L)) ? L : bl;
  bu = (hold & !up & (bu > U)) ? U : bu;
  U = bu;
  L = bl;
}

// PC: the period as a compile-time constant (the reference's 10), 0 = run time
template <int PC>
__global__ __launch_bounds__(STP_NT) void supertrend_panel_kernel(const StArgs A) {
  extern __shared__ double sm[];
  __shared__ double sBU[STP_NT / WAVE], sBL[STP_NT / WAVE];
  __shared__ int sBup[STP_NT / WAVE];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
  const int64_t sym = blockIdx.x;
  const int T = A.T, P = PC > 0 ? PC : A.period, W = A.warm;
  const double pd = (double)P;
  const int NS = stp_slot(T - 1) + 1;
  double* cA = sm;            // close
  double* uA = sm + NS;       // hl2 -> raw upper band -> final upper
  double* lA = sm + 2 * NS;   // TR -> raw lower band -> final lower
  const double* __restrict__ H = A.h + sym * A.ld_in;
  const double* __restrict__ L = A.l + sym * A.ld_in;
  const double* __restrict__ Cl = A.c + sym * A.ld_in;
  const int nj = (T + STP_NT - 1) / STP_NT;

  // ---- row -> LDS (all loads first), TR from the neighbour's close
  double hv[STP_MAXC], lv[STP_MAXC], cv[STP_MAXC];
#pragma unroll
  for (int j = 0; j < STP_MAXC; ++j) {
    const int t = j * STP_NT + tid;
    const bool in = j < nj && t < T;
    hv[j] = in ? H[t] : qnan();
    lv[j] = in ? L[t] : qnan();
    cv[j] = in ? Cl[t] : qnan();
  }
#pragma unroll
  for (int j = 0; j < STP_MAXC; ++j) {
    const int t = j * STP_NT + tid;
    if (j < nj && t < T) {
      cA[stp_slot(t)] = cv[j];
      uA[stp_slot(t)] = (hv[j] + lv[j]) / 2.0;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < STP_MAXC; ++j) {
    const int t = j * STP_NT + tid;
    if (j < nj && t < T) lA[stp_slot(t)] = true_range(hv[j], lv[j], t > 0 ? cA[stp_slot(t - 1)] : qnan());
  }
  __syncthreads();
  // ---- ATR (rolling(P).mean(), min_periods = P, the window in time order)
  double matr[STP_MAXC];
#pragma unroll
  for (int j = 0; j < STP_MAXC; ++j) {
    const int t = j * STP_NT + tid;
    matr[j] = qnan();
    if (j < nj && t < T && t >= P - 1) {
      const double first = lA[stp_slot(t - P + 1)];
      double s = 0.0;
      int n = 0;
      bool same = true;
      auto add = [&](int u) {
        const double v = lA[stp_slot(u)];
        const bool ok = v == v;
        s += ok ? v : 0.0;
        n += ok;
        same = same && v == first;
      };
      if constexpr (PC > 0) {
#pragma unroll
        for (int i = 0; i < PC; ++i) add(t - PC + 1 + i);
      } else {
        for (int u = t - P + 1; u <= t; ++u) add(u);
      }
      matr[j] = A.mult * (n < P ? qnan() : (same ? first : s / pd));
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < STP_MAXC; ++j) {
    const int t = j * STP_NT + tid;
    if (j < nj && t < T) {
      const double hl2 = uA[stp_slot(t)];
      uA[stp_slot(t)] = hl2 + matr[j];
      lA[stp_slot(t)] = hl2 - matr[j];
    }
  }
  __syncthreads();

  // ---- the threads' walks: warm-up, then the chunk (results in registers)
  const int C = nj;   // ceil(T / 256)
  const int a = tid * C, b = min(a + C, T);
  bool up = true, eup = true;
  double U = qnan(), Lo = qnan(), eU = qnan(), eL = qnan();
  double fU[STP_MAXC], fL[STP_MAXC];
  int fup = 0;
  // rewalk: a re-walk stops where its state meets the recorded one (the rest
  // of the chunk, and its end state, are then unchanged)
  auto walk_chunk = [&](bool rewalk) {
    bool met = false;
#pragma unroll
    for (int j = 0; j < STP_MAXC; ++j) {
      const int t = a + j;
      if (j < C && t < b && !met) {
        const int sl = stp_slot(t);
        st_step(up, U, Lo, cA[sl], uA[sl], lA[sl]);
        met = rewalk && up == (((fup >> j) & 1) != 0) && same_bits(U, fU[j]) && same_bits(Lo, fL[j]);
        fU[j] = U;
        fL[j] = Lo;
        fup = up ? fup | (1 << j) : fup & ~(1 << j);
      }
    }
    if (met) {   // the end state is the recorded chunk's
      const int jl = min(C, b - a) - 1;
#pragma unroll
      for (int j = 0; j < STP_MAXC; ++j)
        if (j == jl) {
          up = ((fup >> j) & 1) != 0;
          U = fU[j];
          Lo = fL[j];
        }
    }
  };
#pragma unroll 4
  for (int t = max(0, a - W); t < min(a, T); ++t) {
    const int sl = stp_slot(t);
    st_step(up, U, Lo, cA[sl], uA[sl], lA[sl]);
  }
  eup = up;
  eU = U;
  eL = Lo;
  walk_chunk(false);

  // ---- verify: chunk k's guess against chunk k - 1's end state, in rounds
  for (;;) {
    if (lane == WAVE - 1) {
      sBup[wv] = up;
      sBU[wv] = U;
      sBL[wv] = Lo;
    }
    __syncthreads();
    bool pup = __shfl_up((int)up, 1, WAVE) != 0;
    double pU = __shfl_up(U, 1, WAVE), pL = __shfl_up(Lo, 1, WAVE);
    if (lane == 0 && wv > 0) {
      pup = sBup[wv - 1] != 0;
      pU = sBU[wv - 1];
      pL = sBL[wv - 1];
    }
    const bool wrong = tid > 0 && a > W && a < T && !(eup == pup && same_bits(eU, pU) && same_bits(eL, pL));
    __syncthreads();   // the boundary states are read before the next round's writes
    if (!__syncthreads_or(wrong)) break;
    if (wrong) {
      up = eup = pup;
      U = eU = pU;
      Lo = eL = pL;
      walk_chunk(true);
    }
  }

  // ---- finals -> LDS (own chunk, in place) -> outputs (coalesced)
#pragma unroll
  for (int j = 0; j < STP_MAXC; ++j) {
    const int t = a + j;
    if (j < C && t < b) {
      const int sl = stp_slot(t);
      uA[sl] = fU[j];
      lA[sl] = fL[j];
      cA[sl] = (fup >> j) & 1 ? 1.0 : 0.0;
    }
  }
  __syncthreads();
  double* __restrict__ ou = A.upper ? A.upper + sym * A.ld_out : nullptr;
  double* __restrict__ ol = A.lower ? A.lower + sym * A.ld_out : nullptr;
  uint8_t* __restrict__ of = A.up + sym * A.ld_out;
#pragma unroll
  for (int j = 0; j < STP_MAXC; ++j) {
    const int t = j * STP_NT + tid;
    if (j < nj && t < T) {
      const int sl = stp_slot(t);
      if (ou) ou[t] = uA[sl];
      if (ol) ol[t] = lA[sl];
      of[t] = cA[sl] != 0.0 ? 1 : 0;
    }
  }
}

}  // namespace bq

namespace {
int launch_supertrend(bool fatr, const double* const* in, int64_t S, int64_t T, int64_t ld_in, int32_t period,
                      double multiplier, uint8_t* up, double* upper, double* lower, int64_t ld_out, void* stream,
                      bool panel = false) {
  using namespace bq;
  if (!in || !up || S < 0 || T < 0 || ld_in < T || ld_out < T || T > 0x7fffffff || !(multiplier == multiplier))
    return BQ_EINVAL;
  if (ld_out > BQ_MAX_ROLL_LD) return BQ_EINVAL;   // 32-bit buffer offsets over a wave's 64 rows
  if (fatr && (period < 1 || period > BQ_MAX_WINDOW)) return BQ_EINVAL;
  for (int i = 0; i < (fatr ? 3 : 4); ++i)
    if (!in[i]) return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  StArgs A;
  A.h = in[0];
  A.l = in[1];
  A.c = in[2];
  A.atr = fatr ? nullptr : in[3];
  A.up = up;
  A.upper = upper;
  A.lower = lower;
  A.S = S;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.T = (int)T;
  A.mult = multiplier;
  const int ring = fatr ? period + ST_SUB : 0;
  A.period = fatr ? period : 0;
  A.inv_period = fatr ? 1.0 / (double)period : 0.0;
  A.ring = ring;
  const unsigned blocks = (unsigned)((S + WAVE - 1) / WAVE);
  if (fatr && panel && T <= STP_MAXT) {   // one workgroup per row, the row in LDS (< 64 KiB)
    // BQ_ST_WARM: warm-up candles (measurement; any value gives the same outputs)
    static const int warm = [] {
      const char* e = getenv("BQ_ST_WARM");
      return e ? atoi(e) : STP_W;
    }();
    A.warm = warm < 0 ? 0 : warm;
    const size_t lds = (size_t)3 * (stp_slot((int)T - 1) + 1) * sizeof(double);
    if (period == 10)
      hipLaunchKernelGGL(supertrend_panel_kernel<10>, dim3((unsigned)S), dim3(STP_NT), lds, (hipStream_t)stream, A);
    else
      hipLaunchKernelGGL(supertrend_panel_kernel<0>, dim3((unsigned)S), dim3(STP_NT), lds, (hipStream_t)stream, A);
    return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
  }
  if (fatr) {
    // > 64 KiB of LDS at the largest periods: opt in once, before any graph
    // capture can be active (first call of the process)
    static const bool lds_opt_in = hipFuncSetAttribute((const void*)supertrend_pipe_kernel,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       160 * 1024) == hipSuccess;
    (void)lds_opt_in;
#ifdef BQ_ST_ONE_WAVE
    hipLaunchKernelGGL(supertrend_kernel<true>, dim3(blocks), dim3(WAVE), (size_t)ring * WAVE * sizeof(double),
                       (hipStream_t)stream, A);
#else
    hipLaunchKernelGGL(supertrend_pipe_kernel, dim3(blocks), dim3(2 * WAVE),
                       (size_t)(8 * ST_CT * STG_PITCH + ring * WAVE) * sizeof(double), (hipStream_t)stream, A);
#endif
  }
  else
    hipLaunchKernelGGL(supertrend_kernel<false>, dim3(blocks), dim3(WAVE), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
}  // namespace

extern "C" int bq_supertrend(const double* const* hlca, int64_t S, int64_t T, int64_t ld_in, double multiplier,
                             uint8_t* up, double* upper, double* lower, int64_t ld_out, void* stream) {
  return launch_supertrend(false, hlca, S, T, ld_in, 0, multiplier, up, upper, lower, ld_out, stream);
}

extern "C" int bq_supertrend_hlc(const double* const* hlc, int64_t S, int64_t T, int64_t ld_in, int32_t period,
                                 double multiplier, uint8_t* up, double* upper, double* lower, int64_t ld_out,
                                 void* stream) {
  return launch_supertrend(true, hlc, S, T, ld_in, period, multiplier, up, upper, lower, ld_out, stream);
}

extern "C" int bq_supertrend_panel(const double* const* hlc, int64_t S, int64_t T, int64_t ld_in, int32_t period,
                                   double multiplier, uint8_t* up, double* upper, double* lower, int64_t ld_out,
                                   void* stream) {
  return launch_supertrend(true, hlc, S, T, ld_in, period, multiplier, up, upper, lower, ld_out, stream, true);
}
