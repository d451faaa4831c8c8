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
  const int64_t key = origin + (b0 + b) * A.I;
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

// One workgroup per symbol row: keep flag per candle, block-wide exclusive
// scan (wave ballots + LDS wave offsets), scatter the kept pairs in order.
constexpr int JR_NT = 256;

__global__ __launch_bounds__(JR_NT) void join_returns_kernel(const int64_t* __restrict__ ts,
                                                             const double* __restrict__ close,
                                                             const int64_t* __restrict__ lens, int T, int64_t ld_in,
                                                             const int64_t* __restrict__ bts,
                                                             const double* __restrict__ bclose, int nb,
                                                             double* __restrict__ x, double* __restrict__ y,
                                                             int64_t ld_out, int64_t* __restrict__ out_lens) {
  __shared__ int sWave[JR_NT / WAVE];
  __shared__ int sBase;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t s = blockIdx.x;
  const int64_t* __restrict__ rts = ts + s * ld_in;
  const double* __restrict__ rc = close + s * ld_in;
  const int n = row_len(lens, s, T);
  // the row's offset into the benchmark's index, from its first candle
  const int j0 = n > 0 ? match_last(bts, nb, rts[0]) : -1;
  const int guess_off = j0 >= 0 ? j0 : 0;
  if (tid == 0) sBase = 0;
  __syncthreads();
  for (int t0 = 0; t0 < n; t0 += JR_NT) {
    const int t = t0 + tid;
    double xa = qnan(), yb = qnan();
    if (t < n && t > 0) {
      xa = log_return(rc[t], rc[t - 1]);   // the frame's own previous row
      const int j = match_last_near(bts, nb, rts[t], t + guess_off);
      if (j > 0) yb = log_return(bclose[j], bclose[j - 1]);
    }
    const bool keep = xa == xa && yb == yb;
    const uint64_t m = __ballot(keep);
    const int before = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    if (lane == 0) sWave[w] = __popcll(m);
    __syncthreads();
    int off = sBase;
    for (int k = 0; k < w; ++k) off += sWave[k];
    if (keep) {
      x[s * ld_out + off + before] = xa;
      y[s * ld_out + off + before] = yb;
    }
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int k = 0; k < JR_NT / WAVE; ++k) tot += sWave[k];
      sBase += tot;
    }
    __syncthreads();
  }
  // NaN tail so the row reads as a dropna'd series of length out_lens[s]
  for (int t = sBase + tid; t < T; t += JR_NT) {
    x[s * ld_out + t] = qnan();
    y[s * ld_out + t] = qnan();
  }
  if (tid == 0) out_lens[s] = sBase;
}

// The same join for rows of up to JR_NT * K candles with the whole row in
// registers (candle t = k * JR_NT + tid: every load instruction of a wave is
// one contiguous 512-byte span): every row's loads go out together — closes
// and times, then the benchmark times at the guessed index, then the
// benchmark closes — three dependent round trips per row instead of three
// per 256-candle tile; the kept values are placed from the waves' ballots of
// each k (one barrier), in the same order and with the same values as the
// tiled kernel.
template <int K>
__global__ __launch_bounds__(JR_NT) void join_returns_row_kernel(const int64_t* __restrict__ ts,
                                                                 const double* __restrict__ close,
                                                                 const int64_t* __restrict__ lens, int T, int64_t ld_in,
                                                                 const int64_t* __restrict__ bts,
                                                                 const double* __restrict__ bclose, int nb,
                                                                 double* __restrict__ x, double* __restrict__ y,
                                                                 int64_t ld_out, int64_t* __restrict__ out_lens) {
  constexpr int NW = JR_NT / WAVE;
  __shared__ int sCnt[K][NW];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const int64_t s = blockIdx.x;
  const int64_t* __restrict__ rts = ts + s * ld_in;
  const double* __restrict__ rc = close + s * ld_in;
  const int n = row_len(lens, s, T);
  const int j0 = n > 0 ? match_last(bts, nb, rts[0]) : -1;
  const int off = j0 >= 0 ? j0 : 0;
  double c[K], cp[K];
  int64_t key[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int t = k * JR_NT + tid;
    c[k] = t < n ? rc[t] : qnan();
    cp[k] = t >= 1 && t <= n ? rc[t - 1] : qnan();
    key[k] = t < n ? rts[t] : 0;
  }
  // the benchmark row at the guessed index (index-aligned frames), both
  // neighbours for the keep-last check; the binary search only where it misses
  int64_t g0[K], g1[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int g = k * JR_NT + tid + off;
    g0[k] = g < nb ? bts[g] : INT64_MIN;
    g1[k] = g + 1 < nb ? bts[g + 1] : INT64_MIN;
  }
  int j[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int t = k * JR_NT + tid, g = t + off;
    const bool live = t > 0 && t < n;
    const bool hit = g < nb && g0[k] == key[k] && (g + 1 >= nb || g1[k] != key[k]);
    j[k] = !live ? -1 : (hit ? g : -2);
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (j[k] == -2) j[k] = match_last(bts, nb, key[k]);   // off-grid candles (rare)
  double b0[K], b1[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
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
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    int before = base;
    for (int u = 0; u < w; ++u) before += sCnt[k][u];
    for (int u = 0; u < NW; ++u) base += sCnt[k][u];
    if ((m[k] >> lane) & 1ull) {
      const int pos = before + __builtin_amdgcn_mbcnt_hi((uint32_t)(m[k] >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m[k], 0));
      x[s * ld_out + pos] = xa[k];
      y[s * ld_out + pos] = yb[k];
    }
  }
  for (int t = base + tid; t < T; t += JR_NT) {   // NaN tail: a dropna'd series of length out_lens[s]
    x[s * ld_out + t] = qnan();
    y[s * ld_out + t] = qnan();
  }
  if (tid == 0) out_lens[s] = base;
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

int bq_resample(const int64_t* ts, const double* const* fields, const int32_t* aggs, int32_t nfields,
                const int64_t* lens, int64_t S, int64_t T, int64_t ld_in, int64_t interval_ms, int64_t* out_ts,
                double* const* out_fields, int64_t ld_out, void* stream) {
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
  const int64_t items = S * ld_out;
  hipLaunchKernelGGL(resample_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, (hipStream_t)stream, A);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
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
  if (T <= JR_NT * 8)
    hipLaunchKernelGGL(join_returns_row_kernel<8>, dim3((unsigned)S), dim3(JR_NT), 0, st, ts, close, lens, (int)T,
                       ld_in, bench_ts, bench_close, (int)n_bench, x, y, ld_out, out_lens);
  else if (T <= JR_NT * 16)
    hipLaunchKernelGGL(join_returns_row_kernel<16>, dim3((unsigned)S), dim3(JR_NT), 0, st, ts, close, lens, (int)T,
                       ld_in, bench_ts, bench_close, (int)n_bench, x, y, ld_out, out_lens);
  else
    hipLaunchKernelGGL(join_returns_kernel, dim3((unsigned)S), dim3(JR_NT), 0, st, ts, close, lens, (int)T, ld_in,
                       bench_ts, bench_close, (int)n_bench, x, y, ld_out, out_lens);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
