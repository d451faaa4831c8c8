// Frame plumbing on the device: time-bucket resampling and timestamp joins of
// ragged [S][ld] kline panels.
//
//   bq_resample_count / bq_resample: Candles.resample(df, interval="1h")
//     (producers/context_evaluator.py:403-407; pybinbot, absent) restated as
//     pandas' df.resample(interval).agg({...}) on the open_time
//     DatetimeIndex: bins [origin + b*I, origin + (b+1)*I) with origin =
//     midnight of the first candle's day (pandas origin="start_day",
//     closed/label left), from the first candle's bin to the last candle's;
//     per field FIRST/LAST (first/last non-NaN), MAX/MIN (NaN skipped), SUM
//     (pandas group_sum: Kahan-compensated, NaN skipped, 0 for an empty bin).
//     Empty bins give NaN (FIRST/LAST/MAX/MIN) and 0 (SUM), as pandas does.
//   bq_align: LiquidationSweepPump's left merge of the benchmark on open_time
//     (strategies/liquidation_sweep_pump.py:255-263: drop_duplicates(keep
//     "last"), merge how="left") -> the benchmark value at each candle's
//     timestamp, NaN where the benchmark has no candle.
//   bq_join_returns: the inner join of ContextEvaluator.dynamic_btc_beta_corr
//     (producers/context_evaluator.py:161-177): log returns of each frame on
//     its own rows, inner-joined on the timestamp and dropna'd, compacted per
//     symbol row (pairs feed bq_beta_corr_pairs).
//
// Timestamps are int64 ms, ascending within a row; lens[s] is the valid
// length of row s (NULL: every row has T candles).
#include "bq_device.h"
#include "binquant_amd.h"

namespace bq {

constexpr int64_t DAY_MS = 86400000;

__device__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) {
  const int64_t q = a / b;
  return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

__device__ __forceinline__ int row_len(const int64_t* lens, int64_t s, int T) {
  if (!lens) return T;
  const int64_t n = lens[s];
  return n < 0 ? 0 : (n > T ? T : (int)n);
}

// origin (pandas start_day) and the first bin index of a row
__device__ __forceinline__ void row_bins(const int64_t* ts, int n, int64_t I, int64_t& origin, int64_t& b0,
                                         int64_t& nb) {
  if (n == 0) {
    origin = b0 = nb = 0;
    return;
  }
  origin = floor_div(ts[0], DAY_MS) * DAY_MS;
  b0 = floor_div(ts[0] - origin, I);
  nb = floor_div(ts[n - 1] - origin, I) - b0 + 1;
}

__global__ void resample_count_kernel(const int64_t* __restrict__ ts, const int64_t* __restrict__ lens, int64_t S,
                                      int T, int64_t ld_in, int64_t I, int64_t* __restrict__ out_lens) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  int64_t origin, b0, nb;
  row_bins(ts + s * ld_in, row_len(lens, s, T), I, origin, b0, nb);
  out_lens[s] = nb;
}

struct ResampleArgs {
  const int64_t* ts;
  const int64_t* lens;
  const double* in[BQ_MAX_RESAMPLE_FIELDS];
  double* out[BQ_MAX_RESAMPLE_FIELDS];
  int32_t agg[BQ_MAX_RESAMPLE_FIELDS];
  int64_t* out_ts;
  int64_t S, ld_in, ld_out, I;
  int T, nf;
  int tail;   // a row with more bins than ld_out keeps its NEWEST ld_out bins
};

constexpr int RS_FULL = 4;   // candles of a full bin on the reference's 15m -> 1h resample

// one thread per (symbol, output bin); consecutive threads take consecutive
// bins of a row, so the candles a wave reads are contiguous
__global__ __launch_bounds__(256) void resample_kernel(const ResampleArgs A) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= A.S * A.ld_out) return;
  const int64_t s = i / A.ld_out;
  const int64_t b = i % A.ld_out;
  const int64_t* __restrict__ ts = A.ts + s * A.ld_in;
  const int n = row_len(A.lens, s, A.T);
  int64_t origin, b0, nb;
  row_bins(ts, n, A.I, origin, b0, nb);
  if (b >= nb) return;
  // tail mode: output bin b is the row's bin b + (nb - ld_out) when the row
  // has more bins than the output holds (a gap widened its span)
  const int64_t skip = A.tail && nb > A.ld_out ? nb - A.ld_out : 0;
  const int64_t key = origin + (b0 + skip + b) * A.I;
  const int64_t t0v = ts[0], span = ts[n - 1] - t0v;   // n >= 1 here (nb > b >= 0)
  const int64_t step = n > 1 && span > 0 && span % (n - 1) == 0 ? span / (n - 1) : 0;
  const int lo = lower_bound_guess(ts, n, key, t0v, step);
  const int hi = lower_bound_guess(ts, n, key + A.I, t0v, step);
  if (A.out_ts) A.out_ts[s * A.ld_out + b] = key;
  if (hi - lo == RS_FULL) {
    // a full bin (every candle of the interval present, the common case): the
    // fields' values are loaded together, then aggregated with selects in the
    // same order and with the same NaN rules as the walks below (one round
    // trip to memory instead of one per field and candle)
    for (int f = 0; f < A.nf; ++f) {
      const double* __restrict__ x = A.in[f] + s * A.ld_in + lo;
      double v[RS_FULL];
#pragma unroll
      for (int j = 0; j < RS_FULL; ++j) v[j] = x[j];
      double r = qnan();
      switch (A.agg[f]) {
        case BQ_AGG_FIRST:
#pragma unroll
          for (int j = RS_FULL - 1; j >= 0; --j) r = v[j] == v[j] ? v[j] : r;
          break;
        case BQ_AGG_LAST:
#pragma unroll
          for (int j = 0; j < RS_FULL; ++j) r = v[j] == v[j] ? v[j] : r;
          break;
        case BQ_AGG_MAX:
#pragma unroll
          for (int j = 0; j < RS_FULL; ++j) r = (v[j] == v[j] && (r != r || v[j] > r)) ? v[j] : r;
          break;
        case BQ_AGG_MIN:
#pragma unroll
          for (int j = 0; j < RS_FULL; ++j) r = (v[j] == v[j] && (r != r || v[j] < r)) ? v[j] : r;
          break;
        default: {   // BQ_AGG_SUM: pandas group_sum (Kahan)
          double sum = 0.0, comp = 0.0;
#pragma unroll
          for (int j = 0; j < RS_FULL; ++j) {
            const bool ok = v[j] == v[j];
            const double y = v[j] - comp;
            const double t = sum + y;
            double c2 = t - sum - y;
            c2 = c2 != c2 ? 0.0 : c2;
            comp = ok ? c2 : comp;
            sum = ok ? t : sum;
          }
          r = sum;
        }
      }
      A.out[f][s * A.ld_out + b] = r;
    }
    return;
  }
  for (int f = 0; f < A.nf; ++f) {
    const double* __restrict__ x = A.in[f] + s * A.ld_in;
    double r;
    switch (A.agg[f]) {
      case BQ_AGG_FIRST: {
        r = qnan();
        for (int j = lo; j < hi; ++j)
          if (x[j] == x[j]) {
            r = x[j];
            break;
          }
        break;
      }
      case BQ_AGG_LAST: {
        r = qnan();
        for (int j = hi - 1; j >= lo; --j)
          if (x[j] == x[j]) {
            r = x[j];
            break;
          }
        break;
      }
      case BQ_AGG_MAX:
      case BQ_AGG_MIN: {
        r = qnan();
        const bool mx = A.agg[f] == BQ_AGG_MAX;
        for (int j = lo; j < hi; ++j) {
          const double v = x[j];
          if (v != v) continue;
          if (r != r || (mx ? v > r : v < r)) r = v;
        }
        break;
      }
      default: {   // BQ_AGG_SUM: pandas group_sum (Kahan)
        double sum = 0.0, comp = 0.0;
        for (int j = lo; j < hi; ++j) {
          const double v = x[j];
          if (v != v) continue;
          const double y = v - comp;
          const double t = sum + y;
          comp = t - sum - y;
          if (comp != comp) comp = 0.0;
          sum = t;
        }
        r = sum;
      }
    }
    A.out[f][s * A.ld_out + b] = r;
  }
}

// last j with bts[j] == key (keep="last"), -1 if none
__device__ __forceinline__ int match_last(const int64_t* __restrict__ bts, int nb, int64_t key) {
  const int j = lower_bound_i64(bts, nb, key + 1) - 1;
  return (j >= 0 && bts[j] == key) ? j : -1;
}

// match_last with a guess: index-aligned frames (the common case: the symbol
// and the benchmark share the 15-minute grid from the same start) hit at the
// guess with two loads instead of a dependent binary search.
__device__ __forceinline__ int match_last_near(const int64_t* __restrict__ bts, int nb, int64_t key, int guess) {
  if (guess >= 0 && guess < nb && bts[guess] == key && (guess + 1 == nb || bts[guess + 1] != key)) return guess;
  return match_last(bts, nb, key);
}

__global__ __launch_bounds__(256) void align_kernel(const int64_t* __restrict__ ts, const int64_t* __restrict__ lens,
                                                    int64_t S, int T, int64_t ld_in, const int64_t* __restrict__ bts,
                                                    const double* __restrict__ bval, int nb, double* __restrict__ out,
                                                    int64_t ld_out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= S * (int64_t)T) return;
  const int64_t s = i / T;
  const int t = (int)(i % T);
  double r = qnan();
  if (t < row_len(lens, s, T)) {
    const int j = match_last(bts, nb, ts[s * ld_in + t]);
    if (j >= 0) r = bval[j];
  }
  out[s * ld_out + t] = r;
}

// The inner join of the two return frames on open_time
// (context_evaluator.py:171-175: df_15m[["returns"]].join(df_btc_15m["returns"],
// how="inner") then dropna): a candle whose time the benchmark holds k times
// joins k rows, in the benchmark's order (pandas' many-to-one join), each
// with its own benchmark return (log of its close over the row before it).
// [jf, jl]: the benchmark rows with this time (jf > jl: none). guess: the
// expected index on an index-aligned grid; a unique hit costs the three
// neighbouring loads the caller made, anything else two binary searches.
__device__ __forceinline__ void jr_range(const int64_t* __restrict__ bts, int nb, int64_t key, int g, int64_t gm,
                                         int64_t g0, int64_t g1, int& jf, int& jl) {
  if (g >= 0 && g < nb && g0 == key && (g == 0 || gm != key) && (g + 1 >= nb || g1 != key)) {
    jf = jl = g;
    return;
  }
  jf = lower_bound_i64(bts, nb, key);
  jl = lower_bound_i64(bts, nb, key + 1) - 1;
}

// inclusive wave sum of an int (shfl ladder)
__device__ __forceinline__ int jr_wave_incl(int v, int lane) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const int u = __shfl_up(v, d, WAVE);
    if (lane >= d) v += u;
  }
  return v;
}

// the joined pairs of one candle, written from position pos (pairs past
// ld_out dropped: the row's count is capped at ld_out by the caller)
__device__ __forceinline__ void jr_write(const double* __restrict__ bclose, double xa, int jf, int jl, int pos,
                                         int64_t ld_out, double* __restrict__ xr, double* __restrict__ yr) {
  for (int j = jf; j <= jl; ++j) {
    const double yb = j > 0 ? log_return(bclose[j], bclose[j - 1]) : qnan();
    if (yb == yb) {
      if (pos < ld_out) {
        xr[pos] = xa;
        yr[pos] = yb;
      }
      ++pos;
    }
  }
}

__device__ __forceinline__ int jr_count(const double* __restrict__ bclose, double xa, int jf, int jl) {
  if (!(xa == xa)) return 0;
  int c = 0;
  for (int j = jf; j <= jl; ++j) c += (j > 0 && log_return(bclose[j], bclose[j - 1]) == log_return(bclose[j], bclose[j - 1])) ? 1 : 0;
  return c;
}

// One workgroup per symbol row, 256-candle tiles: pair count per candle,
// block-wide exclusive scan (wave shfl scans + LDS wave offsets), the pairs
// written in order.
constexpr int JR_NT = 256;
#ifndef JR_SPEC
#define JR_SPEC 1   // whole-row kernel: benchmark closes loaded with the guess
#endif
#ifndef JR_WAVES
#define JR_WAVES 8   // whole-row kernel (512 threads): 8 waves per SIMD, 4 rows per CU in flight
#endif
#ifndef JR_ROW_NT
#define JR_ROW_NT 512   // whole-row kernel block (4 / 8 candles per thread)
#endif

template <int NT>
__device__ __forceinline__ void jr_row_tiled(int64_t s, const int64_t* __restrict__ ts,
                                             const double* __restrict__ close, const int64_t* __restrict__ lens,
                                             int T, int64_t ld_in, const int64_t* __restrict__ bts,
                                             const double* __restrict__ bclose, int nb, double* __restrict__ x,
                                             double* __restrict__ y, int64_t ld_out, int64_t* __restrict__ out_lens) {
  __shared__ int sWave[NT / WAVE];
  __shared__ int sBase;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t* __restrict__ rts = ts + s * ld_in;
  const double* __restrict__ rc = close + s * ld_in;
  double* __restrict__ xr = x + s * ld_out;
  double* __restrict__ yr = y + s * ld_out;
  const int n = row_len(lens, s, T);
  // the row's offset into the benchmark's index, from its first candle
  const int j0 = n > 0 ? lower_bound_i64(bts, nb, rts[0]) : 0;
  const int guess_off = j0 < nb && n > 0 && bts[j0] == rts[0] ? j0 : 0;
  if (tid == 0) sBase = 0;
  __syncthreads();
  for (int t0 = 0; t0 < n; t0 += NT) {
    const int t = t0 + tid;
    double xa = qnan();
    int jf = 0, jl = -1;
    if (t < n && t > 0) {
      xa = log_return(rc[t], rc[t - 1]);   // the frame's own previous row
      const int64_t key = rts[t];
      const int g = t + guess_off;
      jr_range(bts, nb, key, g, g >= 1 && g - 1 < nb ? bts[g - 1] : INT64_MIN, g < nb ? bts[g] : INT64_MIN,
               g + 1 < nb ? bts[g + 1] : INT64_MIN, jf, jl);
    }
    const int c = jr_count(bclose, xa, jf, jl);
    const int inc = jr_wave_incl(c, lane);
    if (lane == WAVE - 1) sWave[w] = inc;
    __syncthreads();
    int off = sBase + inc - c;
    for (int k = 0; k < w; ++k) off += sWave[k];
    if (c) jr_write(bclose, xa, jf, jl, off, ld_out, xr, yr);
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int k = 0; k < NT / WAVE; ++k) tot += sWave[k];
      sBase += tot;
    }
    __syncthreads();
  }
  const int total = sBase < ld_out ? sBase : (int)ld_out;
  // NaN tail so the row reads as a dropna'd series of length out_lens[s]
  for (int64_t t = total + tid; t < ld_out; t += NT) {
    xr[t] = qnan();
    yr[t] = qnan();
  }
  if (tid == 0) out_lens[s] = total;
}


__global__ __launch_bounds__(JR_NT) void join_returns_kernel(const int64_t* __restrict__ ts,
                                                             const double* __restrict__ close,
                                                             const int64_t* __restrict__ lens, int T, int64_t ld_in,
                                                             const int64_t* __restrict__ bts,
                                                             const double* __restrict__ bclose, int nb,
                                                             double* __restrict__ x, double* __restrict__ y,
                                                             int64_t ld_out, int64_t* __restrict__ out_lens) {
  jr_row_tiled<JR_NT>(blockIdx.x, ts, close, lens, T, ld_in, bts, bclose, nb, x, y, ld_out, out_lens);
}

// The rows the whole-row kernel handed back (out_lens[s] == -1: the benchmark
// repeats a time the row joins or looks at), through the tiled join: each
// workgroup reads the flags of 256 rows at once and runs its flagged rows
// (nearly always none).
__global__ __launch_bounds__(JR_NT) void join_returns_fixup_kernel(const int64_t* __restrict__ ts,
                                                                   const double* __restrict__ close,
                                                                   const int64_t* __restrict__ lens, int T,
                                                                   int64_t ld_in, const int64_t* __restrict__ bts,
                                                                   const double* __restrict__ bclose, int nb,
                                                                   double* __restrict__ x, double* __restrict__ y,
                                                                   int64_t ld_out, int64_t* __restrict__ out_lens,
                                                                   int64_t S) {
  __shared__ uint64_t sMask[JR_NT / WAVE];
  const int tid = threadIdx.x;
  const int64_t s0 = (int64_t)blockIdx.x * JR_NT;
  const uint64_t m = __ballot(s0 + tid < S && out_lens[s0 + tid] < 0);
  if ((tid & (WAVE - 1)) == 0) sMask[tid / WAVE] = m;
  __syncthreads();
  for (int u = 0; u < JR_NT / WAVE; ++u)
    for (uint64_t mm = sMask[u]; mm; mm &= mm - 1) {
      jr_row_tiled<JR_NT>(s0 + u * WAVE + __builtin_ctzll(mm), ts, close, lens, T, ld_in, bts, bclose, nb, x, y,
                          ld_out, out_lens);
      __syncthreads();   // sBase is reset by the next row
    }
}

// The same join for rows of up to JR_NT * K candles with the whole row in
// registers (candle t = k * JR_NT + tid: every load instruction of a wave is
// one contiguous 512-byte span): every row's loads go out together — closes
// and times, then the benchmark times around the guessed index, then the
// benchmark closes — three dependent round trips per row instead of three
// per 256-candle tile; the pairs are placed from per-k wave scans of the
// pair counts (one barrier), in the same order and with the same values as
// the tiled kernel.
template <int NT, int K>
__global__ __launch_bounds__(NT, K <= 4 ? JR_WAVES : 4) void join_returns_row_kernel(const int64_t* __restrict__ ts,
                                                                 const double* __restrict__ close,
                                                                 const int64_t* __restrict__ lens, int T, int64_t ld_in,
                                                                 const int64_t* __restrict__ bts,
                                                                 const double* __restrict__ bclose, int nb,
                                                                 double* __restrict__ x, double* __restrict__ y,
                                                                 int64_t ld_out, int64_t* __restrict__ out_lens) {
  constexpr int NW = NT / WAVE;
  __shared__ int sCnt[K][NW];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t s = blockIdx.x;
  const int64_t* __restrict__ rts = ts + s * ld_in;
  const double* __restrict__ rc = close + s * ld_in;
  double* __restrict__ xr = x + s * ld_out;
  double* __restrict__ yr = y + s * ld_out;
  const int n = row_len(lens, s, T);
  double c[K], cp[K];
  int64_t key[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {   // the row's own loads go out first
    const int t = k * NT + tid;
    c[k] = t < n ? rc[t] : qnan();
    cp[k] = t >= 1 && t <= n ? rc[t - 1] : qnan();
    key[k] = t < n ? rts[t] : 0;
  }
  // the row's offset into the benchmark's index: one probe at the benchmark's
  // own step (a regular grid), the binary search where that misses
  int off = 0;
  if (n > 0 && nb > 0) {
    const int64_t k0 = rts[0], bt0 = bts[0], step = nb > 1 ? bts[1] - bt0 : 0;
    const int64_t q = step > 0 && k0 > bt0 ? (k0 - bt0) / step : 0;
    int gg = (int)(q < nb - 1 ? q : nb - 1);
    if (bts[gg] != k0) {
      gg = lower_bound_i64(bts, nb, k0);
      if (gg >= nb || bts[gg] != k0) gg = 0;
    }
    off = gg;
  }
  // the benchmark row at the guessed index (index-aligned frames), the one
  // after it, and (speculatively) the two benchmark closes a hit reads: a
  // guessed hit is the only row with its time unless the benchmark repeats a
  // time inside the block's guessed span, which the same loads show (two
  // equal neighbours); candles the guess misses take the binary search. A
  // block that meets a repeated time hands its row to the fixup pass.
  // (the row after the guess is the next lane's guess: only a wave's last
  // lane loads it)
  int64_t g0[K];
  double b0[K], b1[K];
  bool odd = false;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int g = k * NT + tid + off;
    g0[k] = g < nb ? bts[g] : INT64_MIN;
#if JR_SPEC
    b0[k] = g >= 1 && g < nb ? bclose[g] : qnan();
    b1[k] = g >= 1 && g < nb ? bclose[g - 1] : qnan();
#endif
  }
  int j[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int t = k * NT + tid, g = t + off;
    int64_t g1 = __shfl_down(g0[k], 1, WAVE);
    if (lane == WAVE - 1) g1 = g + 1 < nb ? bts[g + 1] : INT64_MIN;
    // a repeat matters only where a candle of the row joins: lane t checks
    // the pair (g, g + 1) around its own guess, and lane t - 1 covers
    // (g - 1, g); lanes past the row (t >= n) do not send the row to the
    // fixup pass for a repeat it never joins
    odd |= t < n && g + 1 < nb && g0[k] == g1;
    const bool live = t > 0 && t < n;
    const bool hit = g < nb && g0[k] == key[k];   // unique unless odd
    j[k] = !live ? -1 : (hit ? g : -2);
  }
#if !JR_SPEC
#pragma unroll
  for (int k = 0; k < K; ++k) {
    b0[k] = j[k] > 0 ? bclose[j[k]] : qnan();
    b1[k] = j[k] > 0 ? bclose[j[k] - 1] : qnan();
  }
#endif
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (j[k] == -2) {   // off-grid candles (rare)
      const int jf = lower_bound_i64(bts, nb, key[k]);
      const bool found = jf < nb && bts[jf] == key[k];
      odd |= found && jf + 1 < nb && bts[jf + 1] == key[k];   // several rows: the fixup pass
      j[k] = found ? jf : -1;
      b0[k] = j[k] > 0 ? bclose[j[k]] : qnan();
      b1[k] = j[k] > 0 ? bclose[j[k] - 1] : qnan();
    }
  double xa[K], yb[K];
  uint64_t m[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    xa[k] = yb[k] = qnan();
    if (j[k] > 0) {   // t in (0, n) with a benchmark row before it
      xa[k] = log_return(c[k], cp[k]);   // the frame's own previous row
      yb[k] = log_return(b0[k], b1[k]);
    }
    m[k] = __ballot(xa[k] == xa[k] && yb[k] == yb[k]);
    if (lane == 0) sCnt[k][w] = __popcll(m[k]);
  }
  const bool odd_w = __ballot(odd) != 0;
  if (lane == 0 && odd_w) sCnt[0][w] |= 1 << 30;   // rides on the count barrier
  __syncthreads();
  bool odd_b = false;
#pragma unroll
  for (int u = 0; u < NW; ++u) odd_b |= (sCnt[0][u] >> 30) != 0;
  if (odd_b) {   // the speculative pairs are dropped: join_returns_fixup_kernel's row
    if (tid == 0) out_lens[s] = -1;
    return;
  }
  int base = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    int before = base;
    for (int u = 0; u < w; ++u) before += sCnt[k][u];
    for (int u = 0; u < NW; ++u) base += sCnt[k][u];
    if ((m[k] >> lane) & 1ull) {
      const int pos = before + __builtin_amdgcn_mbcnt_hi((uint32_t)(m[k] >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m[k], 0));
      xr[pos] = xa[k];
      yr[pos] = yb[k];
    }
  }
  const int total = base < ld_out ? base : (int)ld_out;
  for (int64_t t = total + tid; t < ld_out; t += NT) {   // NaN tail: a dropna'd series of length out_lens[s]
    xr[t] = qnan();
    yr[t] = qnan();
  }
  if (tid == 0) out_lens[s] = total;
}

}  // namespace bq

extern "C" {

int bq_resample_count(const int64_t* ts, const int64_t* lens, int64_t S, int64_t T, int64_t ld_in,
                      int64_t interval_ms, int64_t* out_lens, void* stream) {
  using namespace bq;
  if (!ts || !out_lens || S < 0 || T < 0 || ld_in < T || interval_ms <= 0 || T > 0x7fffffff) return BQ_EINVAL;
  if (S == 0) return BQ_OK;
  hipLaunchKernelGGL(resample_count_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ts,
                     lens, S, (int)T, ld_in, interval_ms, out_lens);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

static int resample_launch(const int64_t* ts, const double* const* fields, const int32_t* aggs, int32_t nfields,
                           const int64_t* lens, int64_t S, int64_t T, int64_t ld_in, int64_t interval_ms,
                           int64_t* out_ts, double* const* out_fields, int64_t ld_out, int tail, void* stream) {
  using namespace bq;
  if (!ts || S < 0 || T < 0 || ld_in < T || ld_out < 0 || interval_ms <= 0 || nfields < 0 ||
      nfields > BQ_MAX_RESAMPLE_FIELDS || (nfields > 0 && (!fields || !aggs || !out_fields)) || T > 0x7fffffff)
    return BQ_EINVAL;
  ResampleArgs A = {};
  for (int f = 0; f < nfields; ++f) {
    if (!fields[f] || !out_fields[f] || aggs[f] < BQ_AGG_FIRST || aggs[f] > BQ_AGG_SUM) return BQ_EINVAL;
    A.in[f] = fields[f];
    A.out[f] = out_fields[f];
    A.agg[f] = aggs[f];
  }
  if (S == 0 || ld_out == 0) return BQ_OK;
  A.ts = ts;
  A.lens = lens;
  A.out_ts = out_ts;
  A.S = S;
  A.ld_in = ld_in;
  A.ld_out = ld_out;
  A.I = interval_ms;
  A.T = (int)T;
  A.nf = nfields;
  A.tail = tail;
  const int64_t items = S * ld_out;
  hipLaunchKernelGGL(resample_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_resample(const int64_t* ts, const double* const* fields, const int32_t* aggs, int32_t nfields,
                const int64_t* lens, int64_t S, int64_t T, int64_t ld_in, int64_t interval_ms, int64_t* out_ts,
                double* const* out_fields, int64_t ld_out, void* stream) {
  return resample_launch(ts, fields, aggs, nfields, lens, S, T, ld_in, interval_ms, out_ts, out_fields, ld_out, 0,
                         stream);
}

int bq_resample_tail(const int64_t* ts, const double* const* fields, const int32_t* aggs, int32_t nfields,
                     const int64_t* lens, int64_t S, int64_t T, int64_t ld_in, int64_t interval_ms, int64_t* out_ts,
                     double* const* out_fields, int64_t ld_out, void* stream) {
  return resample_launch(ts, fields, aggs, nfields, lens, S, T, ld_in, interval_ms, out_ts, out_fields, ld_out, 1,
                         stream);
}

int bq_align(const int64_t* ts, const int64_t* lens, int64_t S, int64_t T, int64_t ld_in, const int64_t* bench_ts,
             const double* bench_val, int64_t n_bench, double* out, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!ts || !bench_ts || !bench_val || !out || S < 0 || T < 0 || ld_in < T || ld_out < T || n_bench < 0 ||
      T > 0x7fffffff || n_bench > 0x7fffffff)
    return BQ_EINVAL;
  if (S == 0 || T == 0) return BQ_OK;
  const int64_t items = S * T;
  hipLaunchKernelGGL(align_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ts, lens,
                     S, (int)T, ld_in, bench_ts, bench_val, (int)n_bench, out, ld_out);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_join_returns(const int64_t* ts, const double* close, const int64_t* lens, int64_t S, int64_t T, int64_t ld_in,
                    const int64_t* bench_ts, const double* bench_close, int64_t n_bench, double* x, double* y,
                    int64_t ld_out, int64_t* out_lens, void* stream) {
  using namespace bq;
  if (!ts || !close || !bench_ts || !bench_close || !x || !y || !out_lens || S < 0 || T < 0 || ld_in < T ||
      ld_out < T || n_bench < 0 || T > 0x7fffffff || n_bench > 0x7fffffff)
    return BQ_EINVAL;
  if (S == 0) return BQ_OK;
  const hipStream_t st = (hipStream_t)stream;
  if (T <= JR_ROW_NT * 4)
    hipLaunchKernelGGL((join_returns_row_kernel<JR_ROW_NT, 4>), dim3((unsigned)S), dim3(JR_ROW_NT), 0, st, ts, close,
                       lens, (int)T, ld_in, bench_ts, bench_close, (int)n_bench, x, y, ld_out, out_lens);
  else if (T <= JR_ROW_NT * 8)
    hipLaunchKernelGGL((join_returns_row_kernel<JR_ROW_NT, 8>), dim3((unsigned)S), dim3(JR_ROW_NT), 0, st, ts, close,
                       lens, (int)T, ld_in, bench_ts, bench_close, (int)n_bench, x, y, ld_out, out_lens);
  else
    hipLaunchKernelGGL(join_returns_kernel, dim3((unsigned)S), dim3(JR_NT), 0, st, ts, close, lens, (int)T, ld_in,
                       bench_ts, bench_close, (int)n_bench, x, y, ld_out, out_lens);
  if (T <= JR_ROW_NT * 8)
    hipLaunchKernelGGL(join_returns_fixup_kernel, dim3((unsigned)((S + JR_NT - 1) / JR_NT)), dim3(JR_NT), 0, st, ts, close,
                       lens, (int)T, ld_in, bench_ts, bench_close, (int)n_bench, x, y, ld_out, out_lens, S);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
