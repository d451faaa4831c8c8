// GradualGainerRetest relative-strength leadership at every prefix of a
// [S][T] panel (gfx950): GradualGainerRetest._leadership_allows
// (strategies/gradual_gainer_retest.py:131-196) with _relative_strengths
// (:131-153), column t = the method on the frame df.iloc[:t + 1] against the
// benchmark frame (btc_time ascending; a duplicated time keeps the later
// row, as the reference's dict does).
//
// Two passes instead of the staged pipeline (align, two element-wise stages,
// two order-statistic jobs, an integer rolling sum: six launches, every
// intermediate through HBM, 2.5 ms at 12.5k x 2k):
//
// pass 1  lead_features_kernel: one workgroup per (symbol, 256-candle tile).
//         The benchmark close at each candle's open_time (a guessed lower
//         bound: two loads on a regular grid, a binary search otherwise),
//         closes and benchmark closes of the tile and its 24-candle halo in
//         LDS; then per candle the history entry (times t, t-8, t-24 present
//         and the six closes > 0: rs_2h / rs_6h, else NaN), the strengths'
//         gate (the last 25 candles present with positive closes, and
//         t + 1 >= min_history) as one byte, and the method's rs_2h / rs_6h
//         outputs (0 where the gate is shut).
// pass 2  lead_rank_kernel: lanes in pairs (rs_2h, rs_6h) of one (symbol,
//         segment). Each lane slides its series' 96-entry history through a
//         sorted-register window (bq_slide.h; the threshold
//         sorted(h)[int((n - 1) q)] is the lower order statistic of rank
//         int(q (n - 1)), NaN below min_count entries), and the pair
//         exchanges its "rs > 0 and rs >= threshold" over DPP: leader =
//         gate and both.
//
// The history is a pure function of (t, t - 8, t - 24) and the entries'
// order does not matter (an order statistic), so the window over pass 1's
// NaN-masked entries equals the reference's list at every t.
#include "bq_slide.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

constexpr int LD_NT = 256;

struct LeadArgs {
  const int64_t* ts;     // open_time [S][ld_ts]
  const double* close;   // [S][ld_c]
  const int64_t* bts;    // benchmark open_time [nb], ascending
  const double* bclose;  // [nb]
  int64_t S, ld_ts, ld_c, ld_w, ld_out;
  int T, nb, shrt, lng, min_hist, minc;
  double q;
  double* h[2];          // workspace [S][ld_w]: history entries rs_2h / rs_6h (NaN: no entry)
  uint8_t* gate;         // workspace [S][ld_w]: strengths present and history long enough
  double* rs[2];         // outputs [S][ld_out]
  uint8_t* leader;       // output [S][ld_out]
  int seg, nseg;         // pass 2 segments
};

__global__ __launch_bounds__(LD_NT) void lead_features_kernel(const LeadArgs A) {
  constexpr int HALO = 32;   // >= the long offset (host: lng <= 31)
  __shared__ double sC[HALO + LD_NT], sB[HALO + LD_NT];
  const int tid = threadIdx.x;
  const int64_t s = blockIdx.y;
  const int t0 = blockIdx.x * LD_NT;
  const int T = A.T, nb = A.nb;
  const int64_t* __restrict__ ts = A.ts + s * A.ld_ts;
  const double* __restrict__ cl = A.close + s * A.ld_c;
  // the benchmark grid for the guessed search
  const int64_t bt0 = A.bts[0];
  const int64_t bstep = nb > 1 ? (A.bts[nb - 1] - bt0) / (nb - 1) : 0;
  for (int i = tid; i < HALO + LD_NT; i += LD_NT) {
    const int t = t0 - HALO + i;
    double c = qnan(), b = qnan();
    if (t >= 0 && t < T) {
      c = cl[t];
      const int64_t key = ts[t];
      const int j = lower_bound_guess(A.bts, nb, key + 1, bt0, bstep) - 1;   // the last row with this time
      if (j >= 0 && A.bts[j] == key) b = A.bclose[j];
    }
    sC[i] = c;
    sB[i] = b;
  }
  __syncthreads();
  const int t = t0 + tid;
  if (t >= T) return;
  const int i = HALO + tid;
  const double c0 = sC[i], c2 = sC[i - A.shrt], c6 = sC[i - A.lng];
  const double b0 = sB[i], b2 = sB[i - A.shrt], b6 = sB[i - A.lng];
  // the reference's float arithmetic: c / c[-9] - b / b[-9] (:151, :179)
  const double r2 = c0 / c2 - b0 / b2;
  const double r6 = c0 / c6 - b0 / b6;
  // a history entry: all three times in the benchmark, min(...) > 0 (:172-180)
  const bool pos = c0 > 0.0 && c2 > 0.0 && c6 > 0.0 && b0 > 0.0 && b2 > 0.0 && b6 > 0.0;
  // _relative_strengths: the last lng + 1 times present, every close > 0
  // (:143-149); len(df) >= MIN_HISTORY (:160)
  bool gate = t + 1 >= A.min_hist && t >= A.lng;
  for (int k = 0; k <= A.lng && gate; ++k) gate = sC[i - k] > 0.0 && sB[i - k] > 0.0;
  const int64_t o = s * A.ld_w + t;
  A.h[0][o] = pos ? r2 : qnan();
  A.h[1][o] = pos ? r6 : qnan();
  A.gate[o] = gate ? 1 : 0;
  const int64_t p = s * A.ld_out + t;
  A.rs[0][p] = gate ? r2 : 0.0;   // (False, 0.0, 0.0) when the strengths are None (:160-161)
  A.rs[1][p] = gate ? r6 : 0.0;
}

// lanes (2k, 2k + 1) = the (rs_2h, rs_6h) series of one (symbol, segment)
template <int W, int K>
__global__ __launch_bounds__(256) void lead_rank_kernel(const LeadArgs A) {
  constexpr int C = 4;   // steps per staged chunk (the window's registers bind: bq_slide.h)
  __shared__ double sv[2][C][256];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int64_t item = (int64_t)blockIdx.x * 256 + tid;
  const int ser = (int)(item & 1);
  const int64_t pair = item >> 1;
  const int64_t sym = pair % A.S;
  const int seg = (int)(pair / A.S);
  if (seg >= A.nseg) return;   // both lanes of a pair leave together; no barriers below
  const double* __restrict__ x = A.h[ser] + sym * A.ld_w;
  const uint8_t* __restrict__ gate = A.gate + sym * A.ld_w;
  uint8_t* __restrict__ lead = A.leader + sym * A.ld_out;
  const int T = A.T;
  const int t_begin = seg * A.seg, t_end = min(T, t_begin + A.seg);
  const int t_start = max(0, t_begin - W + 1);
  auto load_chunk = [&](int ts, double (&v)[C]) {
#pragma unroll
    for (int j = 0; j < C; ++j) v[j] = (ts + j >= 0 && ts + j < T) ? x[ts + j] : qnan();
  };
  double nin[C], nout[C];
  auto fetch = [&](int tc) {
    load_chunk(tc, nin);
    load_chunk(tc - W, nout);
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < C; ++j) {
      sv[0][j][tid] = nin[j];
      sv[1][j][tid] = nout[j];
    }
  };
  SlideRank<W, K, false> R;
  R.init(A.q);
  int tc = t_start;
  if (tc < t_begin) fetch(tc);
  for (; tc < t_begin; tc += C) {   // warm-up: entries t_start .. t_begin - 1, placeholders leave
    stage();
    fetch(tc + C < t_begin ? tc + C : t_begin);
    const int nj = min(C, t_begin - tc);
#pragma unroll 1
    for (int j = 0; j < nj; ++j) R.step(sv[0][j][tid], qnan());
  }
  if (t_start >= t_begin) fetch(t_begin);
  for (tc = t_begin; tc < t_end; tc += C) {
    stage();
    if (tc + C < t_end) fetch(tc + C);
    const int nj = min(C, t_end - tc);
#pragma unroll 1
    for (int j = 0; j < nj; ++j) {
      const int t = tc + j;
      const double v = sv[0][j][tid];
      R.step(v, t - W >= t_start ? sv[1][j][tid] : qnan());
      const double thr = R.value(A.minc, true);
      // rs > 0 and rs >= threshold (a missing threshold: fewer than min_count
      // entries, (False, rs_2h, rs_6h), :181-182); where the gate is open the
      // entry at t exists, so v is the strength itself
      const int ok = (thr == thr && v > 0.0 && v >= thr) ? 1 : 0;
      const int other = __builtin_amdgcn_mov_dpp(ok, 0xB1, 0xF, 0xF, false);   // quad_perm [1, 0, 3, 2]
      if (ser == 0) lead[t] = (gate[t] && ok && other) ? 1 : 0;
    }
  }
  (void)lane;
}

}  // namespace bq

extern "C" size_t bq_leadership_workspace_bytes(int64_t S, int64_t T) {
  if (S <= 0 || T <= 0) return 0;
  const size_t n = (size_t)S * (size_t)T;
  return 2 * n * sizeof(double) + ((n + 255) & ~(size_t)255);
}

extern "C" int bq_leadership(const int64_t* open_time, int64_t ld_ts, const double* close, int64_t ld_c, int64_t S,
                             int64_t T, const int64_t* bench_ts, const double* bench_close, int64_t nb,
                             double rs_quantile, int32_t lookback, int32_t min_history, int32_t min_count,
                             int32_t short_bars, int32_t long_bars, void* workspace, size_t workspace_bytes,
                             uint8_t* leader, double* rs_2h, double* rs_6h, int64_t ld_out, void* stream) {
  using namespace bq;
  constexpr int W = 96, K = 76;   // the strategy's RS_LOOKBACK and int(0.80 * 95)
  if (!open_time || !close || !leader || !rs_2h || !rs_6h || S < 0 || T < 0 || ld_ts < T || ld_c < T ||
      ld_out < T || T > 0x7fffffff - 2 * LD_NT || S > 0x7fffffff || nb < 0 || nb > 0x7fffffff)
    return BQ_EINVAL;
  if (lookback != W || !(rs_quantile >= 0.0 && rs_quantile < 1.0) || (int)(rs_quantile * (double)(W - 1)) != K ||
      short_bars < 1 || long_bars < short_bars || long_bars > 31 || min_count < 1 || min_history < 0)
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
  const size_t need = bq_leadership_workspace_bytes(S, T);
  if (!workspace || workspace_bytes < need || (((uintptr_t)workspace) & 255u)) return BQ_EINVAL;
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
  A.ld_w = T;
  A.ld_out = ld_out;
  A.shrt = short_bars;
  A.lng = long_bars;
  A.min_hist = min_history;
  A.minc = min_count;
  A.q = rs_quantile;
  char* ws = (char*)workspace;
  A.h[0] = (double*)ws;
  A.h[1] = (double*)(ws + (size_t)S * T * sizeof(double));
  A.gate = (uint8_t*)(ws + 2 * (size_t)S * T * sizeof(double));
  A.rs[0] = rs_2h;
  A.rs[1] = rs_6h;
  A.leader = leader;
  // pass 2 segments: ~2 waves per SIMD over 1024 SIMDs (two lanes per
  // (symbol, segment)); each segment replays W - 1 warm-up entries, so
  // segments stay >= 2 W
  const int64_t lanes = (int64_t)1024 * 2 * 64;
  int64_t nseg = lanes / (2 * S);
  nseg = nseg < 1 ? 1 : nseg;
  int64_t seg = (T + nseg - 1) / nseg;
  if (seg < 2 * W) seg = 2 * W;
  A.seg = (int)seg;
  A.nseg = (int)((T + seg - 1) / seg);
  hipLaunchKernelGGL(lead_features_kernel, dim3((unsigned)((T + LD_NT - 1) / LD_NT), (unsigned)S), dim3(LD_NT), 0, st,
                     A);
  const int64_t items = 2 * S * (int64_t)A.nseg;
  hipLaunchKernelGGL((lead_rank_kernel<W, K>), dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}
