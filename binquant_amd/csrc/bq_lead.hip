// GradualGainerRetest relative-strength leadership at every prefix of a
// [S][T] panel (gfx950): GradualGainerRetest._leadership_allows
// (strategies/gradual_gainer_retest.py:131-196) with _relative_strengths
// (:131-153), column t = the method on the frame df.iloc[:t + 1] against the
// benchmark frame (btc_time ascending; a duplicated time keeps the later
// row, as the reference's dict does).
//
// One pass instead of the staged pipeline (align, two element-wise stages,
// two w = 96 order-statistic jobs, an integer rolling sum: six launches,
// every intermediate through HBM, 2.5 ms at 12.5k x 2k). The method returns
// (leader, rs_2h, rs_6h) — never the 80th-percentile thresholds themselves —
// and "rs >= sorted(h)[a]" holds exactly when at least a + 1 history entries
// are <= rs. So no order statistic is formed: each output counts.
//
// lead_kernel: one workgroup per (symbol, 256-candle tile), a thread per
// candle t.
//   1. the closes and the benchmark closes at each candle's open_time (a
//      guessed lower bound: two loads on a regular grid, a binary search
//      otherwise) of the tile and the 96 + 24 candles before it, in LDS;
//   2. the history entries of the tile and its 95 candles before (times t,
//      t - 8, t - 24 in the benchmark, the six closes > 0: rs_2h / rs_6h,
//      else none), in LDS;
//   3. per candle: the strengths' gate (the last 25 candles present with
//      positive closes, t + 1 >= min_history), rs_2h / rs_6h as the method
//      returns them (0 where the gate is shut), and where the gate is open
//      and both strengths are > 0, one walk over the 96 entries of its
//      window counting n (entries), c2 = #{h2 <= rs_2h}, c6 = #{h6 <= rs_6h}:
//      leader = n >= min_count and c2, c6 >= int(q (n - 1)) + 1. A thread
//      walks two neighbouring candles (one LDS read per step serves both),
//      and the pairs that walk are packed into the tile's first waves (a
//      ballot scan through LDS).
// Inputs cross HBM once (the halo re-reads hit L2); nothing but the outputs
// is written.
#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

#ifndef LD_TILE
#define LD_TILE 2048   // candles per workgroup tile (1 024: 0.52-0.53 ms, 2 048: 0.44-0.45 at 12.5k x 2k)
#endif
constexpr int LD_TT = LD_TILE;
constexpr int LD_NT = LD_TT < 1024 ? LD_TT : 1024;   // threads
constexpr int LD_CPT = LD_TT / LD_NT;                // candles per thread (gate phase)
static_assert(LD_TT % LD_NT == 0 && LD_TT / 2 <= LD_NT, "a thread per walking pair");
constexpr int LD_W = 96;                 // RS_LOOKBACK (compiled)
constexpr int LD_LMAX = 31;              // the long offset's bound (RS 6h: 24)
constexpr int LD_HH = LD_W - 1;          // history halo before the tile
constexpr int LD_CH = LD_HH + LD_LMAX;   // close halo before the tile (history halo + long offset)

struct LeadArgs {
  const int64_t* ts;     // open_time [S][ld_ts]
  const double* close;   // [S][ld_c]
  const int64_t* bts;    // benchmark open_time [nb], ascending
  const double* bclose;  // [nb]
  int64_t S, ld_ts, ld_c, ld_out;
  int T, nb, shrt, lng, min_hist, minc;
  double q;
  double* rs[2];         // outputs [S][ld_out]
  uint8_t* leader;       // output [S][ld_out]
};

__global__ __launch_bounds__(LD_NT) void lead_kernel(const LeadArgs A) {
  __shared__ double sC[LD_CH + LD_TT], sB[LD_CH + LD_TT];
  __shared__ double2 sH[LD_HH + LD_TT];   // (rs_2h, rs_6h) entries: one 16-byte LDS read per walk step
  __shared__ uint64_t sPos[(LD_CH + LD_TT + WAVE - 1) / WAVE];   // bit: close and benchmark close > 0
  __shared__ uint64_t sVal[(LD_HH + LD_TT + WAVE - 1) / WAVE];    // bit: a history entry exists
  const int tid = threadIdx.x;
  const int64_t s = blockIdx.y;
  const int t0 = blockIdx.x * LD_TT;
  const int T = A.T, nb = A.nb, shrt = A.shrt, lng = A.lng;
  const int64_t* __restrict__ ts = A.ts + s * A.ld_ts;
  const double* __restrict__ cl = A.close + s * A.ld_c;
  // 1. closes and benchmark closes of candles t0 - LD_CH .. t0 + LD_TT - 1
  const int64_t bt0 = A.bts[0];
  const int64_t bstep = nb > 1 ? (A.bts[nb - 1] - bt0) / (nb - 1) : 0;
  for (int i = tid; i < LD_CH + LD_TT; i += LD_NT) {
    const int t = t0 - LD_CH + i;
    double c = qnan(), b = qnan();
    if (t >= 0 && t < T) {
      c = cl[t];
      const int64_t key = ts[t];
      // the last benchmark row with this time: on a regular grid the guessed
      // row's time, its successor's and its close are loaded together (one
      // dependent round trip after the candle's time); the search otherwise
      int jg = -1;
      if (bstep > 0 && key >= bt0) {
        const int64_t q = (key - bt0) / bstep;
        jg = q < nb ? (int)q : -1;
      }
      bool hit = false;
      if (jg >= 0) {
        const int64_t tg = A.bts[jg];
        const int64_t tn = jg + 1 < nb ? A.bts[jg + 1] : INT64_MAX;
        const double bg = A.bclose[jg];
        hit = tg == key && tn != key;
        if (hit) b = bg;
      }
      if (!hit) {
        const int j = lower_bound_guess(A.bts, nb, key + 1, bt0, bstep) - 1;
        if (j >= 0 && A.bts[j] == key) b = A.bclose[j];
      }
    }
    sC[i] = c;
    sB[i] = b;
    const uint64_t pm = __ballot(c > 0.0 && b > 0.0);   // slots i - lane .. i - lane + 63 (LD_NT % 64 == 0)
    if ((tid & (WAVE - 1)) == 0) sPos[i / WAVE] = pm;
  }
  __syncthreads();
  // 2. history entries of candles t0 - LD_HH .. t0 + LD_TT - 1 (none outside the row)
  for (int i = tid; i < LD_HH + LD_TT; i += LD_NT) {
    const int k = i + LD_LMAX;   // the candle's slot in sC / sB
    const double c0 = sC[k], c2 = sC[k - shrt], c6 = sC[k - lng];
    const double b0 = sB[k], b2 = sB[k - shrt], b6 = sB[k - lng];
    // a history entry: all three times in the benchmark, min(...) > 0 (:172-180),
    // the reference's float arithmetic c / c[-9] - b / b[-9] (:179-180)
    const bool pos = c0 > 0.0 && c2 > 0.0 && c6 > 0.0 && b0 > 0.0 && b2 > 0.0 && b6 > 0.0;
    sH[i] = make_double2(pos ? c0 / c2 - b0 / b2 : qnan(), pos ? c0 / c6 - b0 / b6 : qnan());
    // the entry exists iff pos (both strengths are then numbers: finite > 0 closes)
    const uint64_t vm = __ballot(pos);   // slots i - lane .. i - lane + 63
    if ((tid & (WAVE - 1)) == 0) sVal[i / WAVE] = vm;
  }
  __syncthreads();
  const int lane = tid & (WAVE - 1), w = tid / WAVE;
  // 3. per candle u of the tile (LD_CPT per thread): _relative_strengths — the
  //    last lng + 1 times present, every close > 0 (:143-149); len(df) >=
  //    MIN_HISTORY (:160)
  constexpr int NP = LD_TT / 2;
  __shared__ unsigned char sAct[LD_TT];
  __shared__ int sList[NP], sWc[LD_NT / WAVE];
#pragma unroll
  for (int q = 0; q < LD_CPT; ++q) {
    const int u = q * LD_NT + tid, t = t0 + u;
    bool act = false;
    if (t < T) {
      const int k = LD_CH + u;
      bool gate = t + 1 >= A.min_hist && t >= lng;
      {   // slots k - lng .. k all positive (lng < 64: at most two mask words)
        const int lo = k - lng, wl = lo / WAVE, wh = k / WAVE;
        const uint64_t hi_mask = ~0ull >> (WAVE - 1 - (k & (WAVE - 1)));   // bits 0 .. k % 64
        const uint64_t lo_mask = ~0ull << (lo & (WAVE - 1));                // bits lo % 64 .. 63
        gate = gate && (wl == wh ? (sPos[wh] & (hi_mask & lo_mask)) == (hi_mask & lo_mask)
                                 : (sPos[wl] & lo_mask) == lo_mask && (sPos[wh] & hi_mask) == hi_mask);
      }
      // (:150-153) c / c[-shrt - 1] - b / b[-shrt - 1]: the gate (every close
      // of the last lng + 1 candles > 0) makes candle t's history entry exist,
      // and the entry is that same expression
      double r2 = 0.0, r6 = 0.0;
      if (gate) {
        const double2 e = sH[LD_HH + u];
        r2 = e.x;
        r6 = e.y;
      }
      const int64_t o = s * A.ld_out + t;
      A.rs[0][o] = gate ? r2 : 0.0;   // (False, 0.0, 0.0) when the strengths are None (:160-161)
      A.rs[1][o] = gate ? r6 : 0.0;
      // otherwise the method's answer is False whatever the thresholds
      act = gate && r2 > 0.0 && r6 > 0.0;
      if (!act) A.leader[o] = 0;
    }
    sAct[u] = act;
  }
  // the window walks, two neighbouring candles per thread (their windows
  // share 95 of 96 entries: one LDS read serves both), the pairs that need
  // one packed into the tile's first waves (the others' waves skip it)
  __syncthreads();
  const bool pa = tid < NP && (sAct[2 * tid] | sAct[2 * tid + 1]);
  const uint64_t m = __ballot(pa);
  if (lane == 0) sWc[w] = __popcll(m);
  __syncthreads();
  int base = 0, total = 0;
  for (int v = 0; v < LD_NT / WAVE; ++v) {
    base += v < w ? sWc[v] : 0;
    total += sWc[v];
  }
  if (pa) sList[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] = tid;
  __syncthreads();
  if (tid >= total) return;
  const int u0 = 2 * sList[tid], u1 = u0 + 1;
  // the strengths are the candles' own history entries (the gate implies
  // they exist; a candle of the pair that does not walk is counted and dropped)
  const double2 q0 = sH[LD_HH + u0], q1 = sH[LD_HH + u1];
  const double r20 = q0.x, r60 = q0.y, r21 = q1.x, r61 = q1.y;
  // the window of the last LD_W positions (:170): how many entries are <=
  // the current strengths (a missing entry is NaN: never <=). Entry h1 - d is
  // candle u1's d-th (d = 0 .. LD_W - 1) and u0's (d - 1)-th: one read per
  // step serves both.
  const int h1 = LD_HH + u1;
  int c20 = 0, c60 = 0, c21, c61;
  {
    const double2 e = sH[h1];
    c21 = e.x <= r21 ? 1 : 0;
    c61 = e.y <= r61 ? 1 : 0;
  }
#pragma unroll 5   // (1 / 10 / 19: equal or slower)
  for (int d = 1; d < LD_W; ++d) {
    const double2 e = sH[h1 - d];
    c21 += e.x <= r21 ? 1 : 0;
    c61 += e.y <= r61 ? 1 : 0;
    c20 += e.x <= r20 ? 1 : 0;
    c60 += e.y <= r60 ? 1 : 0;
  }
  {
    const double2 e = sH[h1 - LD_W];
    c20 += e.x <= r20 ? 1 : 0;
    c60 += e.y <= r60 ? 1 : 0;
  }
  // entry counts from the existence bitmask: slots [h - LD_W + 1, h]
  auto entries = [&](int h) {   // lo >= 0: the halo covers the window
    const int lo = h - (LD_W - 1);
    int n = 0;
    for (int wd = lo / WAVE; wd <= h / WAVE; ++wd) {
      uint64_t m = sVal[wd];
      if (wd == lo / WAVE) m &= ~0ull << (lo & (WAVE - 1));
      if (wd == h / WAVE) m &= ~0ull >> (WAVE - 1 - (h & (WAVE - 1)));
      n += __popcll(m);
    }
    return n;
  };
  const int n0 = entries(h1 - 1), n1 = entries(h1);
  // sorted(h)[int((n - 1) q)] <= rs  <=>  #{h <= rs} >= int((n - 1) q) + 1 (:183-193)
  const int64_t o = s * A.ld_out + t0;
  if (sAct[u0]) {
    const int need = (int)((double)(n0 - 1) * A.q) + 1;
    A.leader[o + u0] = n0 >= A.minc && c20 >= need && c60 >= need ? 1 : 0;
  }
  if (sAct[u1]) {
    const int need = (int)((double)(n1 - 1) * A.q) + 1;
    A.leader[o + u1] = n1 >= A.minc && c21 >= need && c61 >= need ? 1 : 0;
  }
}

}  // namespace bq

extern "C" size_t bq_leadership_workspace_bytes(int64_t S, int64_t T) {
  (void)S;
  (void)T;
  return 0;   // one pass: no intermediate (kept in the ABI for callers that size a workspace)
}

extern "C" int bq_leadership(const int64_t* open_time, int64_t ld_ts, const double* close, int64_t ld_c, int64_t S,
                             int64_t T, const int64_t* bench_ts, const double* bench_close, int64_t nb,
                             double rs_quantile, int32_t lookback, int32_t min_history, int32_t min_count,
                             int32_t short_bars, int32_t long_bars, void* workspace, size_t workspace_bytes,
                             uint8_t* leader, double* rs_2h, double* rs_6h, int64_t ld_out, void* stream) {
  using namespace bq;
  (void)workspace;
  (void)workspace_bytes;
  if (!open_time || !close || !leader || !rs_2h || !rs_6h || S < 0 || T < 0 || ld_ts < T || ld_c < T ||
      ld_out < T || T > 0x7fffffff - 2 * LD_TT || S > 0x7fffffff || nb < 0 || nb > 0x7fffffff)
    return BQ_EINVAL;
  if (lookback != LD_W || !(rs_quantile >= 0.0 && rs_quantile < 1.0) || short_bars < 1 || long_bars < short_bars ||
      long_bars > LD_LMAX || min_count < 1 || min_history < 0)
    return BQ_EINVAL;   // other parameters: the staged pipeline (signals.gradual_gainer_leadership)
  if (S == 0 || T == 0) return BQ_OK;
  hipStream_t st = (hipStream_t)stream;
  if (nb == 0 || !bench_ts || !bench_close) {   // no benchmark: no strengths anywhere
    for (int64_t s = 0; s < S; ++s) {
      if (hipMemsetAsync(leader + s * ld_out, 0, (size_t)T, st) != hipSuccess ||
          hipMemsetAsync(rs_2h + s * ld_out, 0, (size_t)T * sizeof(double), st) != hipSuccess ||
          hipMemsetAsync(rs_6h + s * ld_out, 0, (size_t)T * sizeof(double), st) != hipSuccess)
        return BQ_EHIP;
    }
    return BQ_OK;
  }
  LeadArgs A;
  memset(&A, 0, sizeof(A));
  A.ts = open_time;
  A.close = close;
  A.bts = bench_ts;
  A.bclose = bench_close;
  A.S = S;
  A.T = (int)T;
  A.nb = (int)nb;
  A.ld_ts = ld_ts;
  A.ld_c = ld_c;
  A.ld_out = ld_out;
  A.shrt = short_bars;
  A.lng = long_bars;
  A.min_hist = min_history;
  A.minc = min_count;
  A.q = rs_quantile;
  A.rs[0] = rs_2h;
  A.rs[1] = rs_6h;
  A.leader = leader;
  hipLaunchKernelGGL(lead_kernel, dim3((unsigned)((T + LD_TT - 1) / LD_TT), (unsigned)S), dim3(LD_NT), 0, st, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
