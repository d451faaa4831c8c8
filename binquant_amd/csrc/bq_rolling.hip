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
//   rank (quantile/median/max/min): lane = (symbol, segment of the row).
//     Each lane keeps its window SORTED IN REGISTERS (W slots, +inf padding):
//     a removal / insertion is a branch-free pass of compares and selects over
//     the W slots (no LDS, no serial shift loop), so throughput scales with
//     VALU width instead of LDS latency. A segment first rebuilds its window
//     from the w values before it, so segments are independent.
#include "bq_device.h"
#include "binquant_amd.h"

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
  double q, alpha;
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
  __device__ __forceinline__ void add(double v, bool welford) {
    if (v != v) return;
    ++nobs;
    if (welford) {
      vn += 1.0;
      const double pm = mean - v_add;
      const double y = v - v_add;
      const double t = y - mean;
      v_add = t + mean - y;
      mean = vn != 0.0 ? mean + t / vn : 0.0;
      ssq = ssq + (v - pm) * (v - mean);
    } else {
      const double y = v - c_add;
      const double t = sum + y;
      c_add = t - sum - y;
      sum = t;
      neg += signbit(v) ? 1 : 0;
    }
    same = (v == prev) ? same + 1 : 1;
    prev = v;
  }
  __device__ __forceinline__ void remove(double v, bool welford) {
    if (v != v) return;
    --nobs;
    if (welford) {
      vn -= 1.0;
      if (vn != 0.0) {
        const double pm = mean - v_rem;
        const double y = v - v_rem;
        const double t = y - mean;
        v_rem = t + mean - y;
        mean = mean - t / vn;
        ssq = ssq - (v - pm) * (v - mean);
      } else {
        mean = ssq = 0.0;
      }
    } else {
      const double y = -v - c_rem;
      const double t = sum + y;
      c_rem = t - sum - y;
      sum = t;
      neg -= signbit(v) ? 1 : 0;
    }
  }
  __device__ __forceinline__ double result(int mode, int minp) const {
    switch (mode) {
      case BQ_ROLL_SUM:   // calc_sum
        if (nobs == 0 && minp == 0) return 0.0;
        if (nobs < minp) return qnan();
        return same >= nobs ? prev * (double)nobs : sum;
      case BQ_ROLL_MEAN: {   // calc_mean
        if (nobs < minp || nobs <= 0) return qnan();
        double r = sum / (double)nobs;
        if (same >= nobs) r = prev;
        else if (neg == 0 && r < 0.0) r = 0.0;
        else if (neg == nobs && r > 0.0) r = 0.0;
        return r;
      }
      default: {   // calc_var (ddof 1 or 0), std = sqrt
        const double ddof = (mode == BQ_ROLL_VAR || mode == BQ_ROLL_STD) ? 1.0 : 0.0;
        double r;
        if (vn >= (double)minp && vn > ddof) {
          if (vn == 1.0 || (double)same >= vn) r = 0.0;
          else {
            r = ssq / (vn - ddof);
            r = r < 0.0 ? 0.0 : r;
          }
        } else {
          r = qnan();
        }
        return (mode == BQ_ROLL_STD || mode == BQ_ROLL_STD0) ? sqrt(r) : r;
      }
    }
  }
};

// LDS: a ring of the last `ring` input chunks (RL = ring * RP_CT candles per
// lane, lane-interleaved); the ring covers window + shift, so the leaving
// value is an LDS read and every input byte crosses HBM once. Results go
// straight from each lane to its row (consecutive steps fill a cache line
// in L2 before it is written back), which keeps the LDS per wave small
// enough for several waves per CU.
__global__ __launch_bounds__(WAVE) void replay_kernel(const RollBatch B, int ring) {
  const RollJob& A = B.j[blockIdx.y];   // wave-uniform: scalar kernarg loads
  const bool EWM = A.mode == BQ_ROLL_EWM;
  extern __shared__ double smem[];
  constexpr int TILE = RP_CT * STG_PITCH;
  const int RL = ring * RP_CT;
  const int lane = threadIdx.x;
  const int64_t sym0 = (int64_t)blockIdx.x * WAVE;
  const int64_t S = B.S;
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
  Moments m;
  m.init(0.0);
  // ewm state (pandas ewm, adjust=False, ignore_na=False)
  double weighted = qnan(), old_wt = 1.0;
  int nobs = 0;
  const double alpha = A.alpha, om = 1.0 - alpha;
  for (int t0 = 0; t0 < T; t0 += RP_CT) {
    stage_put<RP_CT>(smem + ((t0 / RP_CT) % ring) * TILE, lane, ri);
    __syncthreads();
    if (t0 + RP_CT < T)   // next chunk in flight during this one's replay
      stage_load<RP_CT>(A.x, A.ld_in, sym0, S, t0 + RP_CT, T, lane, ri);
    auto step = [&](int j) {
      const int t = t0 + j;
      const double v_in = t - sh < 0 ? qnan() : smem[pin * STG_PITCH + lane];
      pin = pin + 1 == RL ? 0 : pin + 1;
      double res;
      if (EWM) {
        if (t == 0) {
          weighted = v_in;
          nobs = v_in == v_in;
        } else {
          const bool obs = v_in == v_in;
          nobs += obs;
          if (weighted == weighted) {
            old_wt *= om;
            if (obs) {
              if (weighted != v_in) {
                weighted = old_wt * weighted + alpha * v_in;
                weighted /= old_wt + alpha;
              }
              old_wt = 1.0;
            }
          } else if (obs) {
            weighted = v_in;
          }
        }
        res = nobs >= A.minp ? weighted : qnan();
      } else {
        if (t == 0) m.init(v_in);   // pandas: prev_value = first value of the series
        if (t >= w && t - sh - w >= 0) m.remove(smem[pout * STG_PITCH + lane], welford);
        pout = pout + 1 == RL ? 0 : pout + 1;
        m.add(v_in, welford);
        res = m.result(A.mode, A.minp);
      }
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
    return (i >= 0 && i < T) ? x[i] : qnan();
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
      if ((double)idx == idxf) r = win.get(idx);
      else {
        const double lo = win.get(idx), hi = win.get(idx + 1);
        r = lo + (hi - lo) * (idxf - (double)idx);
      }
    }
    out[t] = r;
  }
}

}  // namespace bq

namespace {

bool job_ok(const bq_roll_job& j, int64_t T) {
  if (!j.x || !j.out || j.ld_in < T || j.ld_out < T || j.min_periods < 0) return false;
  if (j.mode == BQ_ROLL_EWM) return j.alpha > 0.0 && j.alpha <= 1.0;
  return j.window >= 1 && j.window <= bq::RW_MAXW && j.shift >= 0 && j.shift <= bq::RW_MAXSHIFT &&
         j.mode >= BQ_ROLL_QUANTILE && j.mode <= BQ_ROLL_STD0 && j.q >= 0.0 && j.q <= 1.0;
}

int rank_bucket(int w) {
  return w <= 8 ? 0 : w <= 24 ? 1 : w <= 48 ? 2 : w <= 64 ? 3 : w <= 80 ? 4 : 5;
}

template <int W>
void launch_rank(const bq::RollBatch& B, int n, int64_t max_items, hipStream_t st) {
  const unsigned blocks = (unsigned)((max_items + 255) / 256);
  hipLaunchKernelGGL(bq::rank_kernel<W>, dim3(blocks, (unsigned)n), dim3(256), 0, st, B);
}

}  // namespace

extern "C" {

int bq_rolling_batch(const bq_roll_job* jobs, int32_t n_jobs, int64_t S, int64_t T, void* stream) {
  using namespace bq;
  if (!jobs || n_jobs < 0 || S < 0 || T < 0 || T > 0x7fffffff) return BQ_EINVAL;
  for (int i = 0; i < n_jobs; ++i)
    if (!job_ok(jobs[i], T)) return BQ_EINVAL;
  if (S == 0 || T == 0 || n_jobs == 0) return BQ_OK;
  hipStream_t st = (hipStream_t)stream;
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
    hipLaunchKernelGGL(replay_kernel, dim3((unsigned)((S + WAVE - 1) / WAVE), (unsigned)nrep), dim3(WAVE), lds, st,
                       rep, ring);
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
  for (int i = 0; i < n_jobs; ++i) {
    const bq_roll_job& in = jobs[i];
    RollJob J;
    memset(&J, 0, sizeof(J));
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
    if (in.mode >= BQ_ROLL_MEAN) {   // moments / ewm: exact replay
      const int back = in.mode == BQ_ROLL_EWM ? 0 : in.window + in.shift;
      max_back = back > max_back ? back : max_back;
      rep.j[nrep++] = J;
      if (nrep == RW_MAXJOBS) flush_rep();
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
  }
  flush_rep();
  for (int b = 0; b < 6; ++b) flush_rank(b);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_rolling(const double* x, int64_t S, int64_t T, int64_t ld_in, int32_t window, int32_t min_periods,
               int32_t shift, int32_t mode, double q, double* out, int64_t ld_out, void* stream) {
  if (mode < BQ_ROLL_QUANTILE || mode > BQ_ROLL_STD0) return BQ_EINVAL;
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
