// Device-resident MarketStateStore and the per-message
// features of the live market context (§8a a13/a16).
//
// market_regime/market_state_store.py:19-31 keeps, per symbol, the closed
// candles sorted by timestamp, de-duplicated (keep="last") and capped to the
// last max_bars (tail). Here every symbol owns a ring of max_bars candles in
// HBM (bq_store_view): an update is an in-order append in the common case
// (a new closed candle), and an LDS merge of the incoming sorted run with the
// ring otherwise (a late / corrected candle or a REST history sync,
// klines_provider.py:135-181).
//
// bq_store_features runs LiveMarketContextAccumulator._compute_symbol_features
// (market_regime/live_market_context_accumulator.py:244-297) on the selected
// rings by REPLAYING pandas' own recurrences over the whole history, so the
// values are the pandas values bit for bit:
//   ewm(span, adjust=False, min_periods=1).mean()   (aggregations.pyx ewm)
//   rolling(w, min_periods=1).mean()                (roll_mean: Kahan add /
//       remove with separate compensations, same-value and sign rules)
//   rolling(w, min_periods=1).std(ddof=0)           (roll_var: compensated
//       Welford add / remove, same-value rule), sqrt, fillna(0)
// (restatements pinned bit-exact against pandas 2.3.3 in tests/).
// Lane = symbol; chunks of the rings are read coalesced and transposed
// through LDS; each lane keeps its last 14 true ranges / 20 closes in a
// private LDS ring for the window removals.
#include "bq_device.h"
#include "binquant_amd.h"

#include <string.h>

namespace bq {

struct StoreArgs {
  int64_t* ts;
  double* f[BQ_NUM_INPUTS];
  int32_t* head;
  int32_t* count;
  int64_t* last;
  int64_t cap;
  int M;
};

__device__ __forceinline__ int ring_at(int h, int i, int M) {
  const int p = h + i;
  return p >= M ? p - M : p;
}

// ---- update --------------------------------------------------------------------
constexpr int SU_NT = 64;

struct UpdArgs {
  const int64_t* slot;
  const int64_t* ts;
  const double* f[BQ_NUM_INPUTS];
  const int64_t* seg;
};

// first i in [0, n) with key(i) >= v
template <typename F>
__device__ __forceinline__ int lower_bound_fn(int n, int64_t v, F key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (key(mid) < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(SU_NT) void store_update_kernel(const StoreArgs V, const UpdArgs U) {
  __shared__ int64_t sT[BQ_STORE_MAX_BARS];
  __shared__ double sF[BQ_NUM_INPUTS][BQ_STORE_MAX_BARS];
  __shared__ int sPK[BQ_STORE_MAX_BARS + 1];
  __shared__ int sCnt[SU_NT];
  const int tid = threadIdx.x;
  const int64_t b = U.seg[blockIdx.x], e = U.seg[blockIdx.x + 1];
  const int k = (int)(e - b);
  if (k <= 0) return;
  // a single candle without a close is dropped (market_state_store.py:84);
  // longer runs arrive compacted by the host
  if (k == 1 && !(U.f[BQ_CLOSE][b] == U.f[BQ_CLOSE][b])) return;
  const int64_t s = U.slot[b];
  const int M = V.M;
  const int n = V.count[s], h = V.head[s];
  const int64_t row = s * (int64_t)M;
  const int64_t* __restrict__ its = U.ts + b;

  if (n == 0 || its[0] > V.last[s]) {   // in-order append (the live path)
    const int total = n + k;
    const int keep = min(M, total);
    for (int j = max(0, k - M) + tid; j < k; j += SU_NT) {
      const int p = ring_at(h, (n + j) % M, M);
      V.ts[row + p] = its[j];
#pragma unroll
      for (int c = 0; c < BQ_NUM_INPUTS; ++c) V.f[c][row + p] = U.f[c][b + j];
    }
    if (tid == 0) {
      V.count[s] = keep;
      V.head[s] = (int)((h + (int64_t)(total - keep)) % M);
      V.last[s] = its[k - 1];
    }
    return;
  }

  // general merge: an existing candle is dropped when the run carries its
  // timestamp (keep="last"); sPK[i] = kept existing candles before i
  auto ets = [&](int i) { return V.ts[row + ring_at(h, i, M)]; };
  auto in_run = [&](int64_t v) {
    const int j = lower_bound_fn(k, v, [&](int q) { return its[q]; });
    return j < k && its[j] == v;
  };
  const int chunk = (n + SU_NT - 1) / SU_NT;
  const int i0 = min(n, tid * chunk), i1 = min(n, i0 + chunk);
  int cnt = 0;
  for (int i = i0; i < i1; ++i) cnt += in_run(ets(i)) ? 0 : 1;
  sCnt[tid] = cnt;
  __syncthreads();
  int base = 0;
  for (int q = 0; q < tid; ++q) base += sCnt[q];
  for (int i = i0; i < i1; ++i) {
    sPK[i] = base;
    base += in_run(ets(i)) ? 0 : 1;
  }
  if (tid == SU_NT - 1) sPK[n] = base;
  __syncthreads();
  const int L = sPK[n] + k;
  const int keep = min(M, L), off = L - keep;
  for (int i = tid; i < n; i += SU_NT) {
    if (sPK[i + 1] == sPK[i]) continue;   // dropped
    const int64_t te = ets(i);
    const int pos = sPK[i] + lower_bound_fn(k, te, [&](int q) { return its[q]; });
    if (pos >= off) {
      const int p = ring_at(h, i, M);
      sT[pos - off] = te;
#pragma unroll
      for (int c = 0; c < BQ_NUM_INPUTS; ++c) sF[c][pos - off] = V.f[c][row + p];
    }
  }
  for (int j = tid; j < k; j += SU_NT) {
    const int64_t tj = its[j];
    const int pos = j + sPK[lower_bound_fn(n, tj, ets)];
    if (pos >= off) {
      sT[pos - off] = tj;
#pragma unroll
      for (int c = 0; c < BQ_NUM_INPUTS; ++c) sF[c][pos - off] = U.f[c][b + j];
    }
  }
  __syncthreads();
  for (int q = tid; q < keep; q += SU_NT) {
    V.ts[row + q] = sT[q];
#pragma unroll
    for (int c = 0; c < BQ_NUM_INPUTS; ++c) V.f[c][row + q] = sF[c][q];
  }
  if (tid == 0) {
    V.count[s] = keep;
    V.head[s] = 0;
    V.last[s] = sT[keep - 1];
  }
}

// ---- features of the latest candle -------------------------------------------------
constexpr int SF_CT = 16;
constexpr int SF_ATR = 14;   // live_market_context_accumulator.py:268
constexpr int SF_BB = 20;    // :269-270

// pandas roll_mean state (add_mean / remove_mean / calc_mean)
struct RollMean {
  double sum, comp_add, comp_rem, prev;
  int nobs, neg, same;
  __device__ __forceinline__ void init() {
    sum = comp_add = comp_rem = 0.0;
    nobs = neg = same = 0;
    prev = 0.0;
  }
  __device__ __forceinline__ void add(double v) {
    if (v != v) return;
    ++nobs;
    const double y = v - comp_add;
    const double t = sum + y;
    comp_add = t - sum - y;
    sum = t;
    if (signbit(v)) ++neg;
    same = (v == prev) ? same + 1 : 1;
    prev = v;
  }
  __device__ __forceinline__ void remove(double v) {
    if (v != v) return;
    --nobs;
    const double y = -v - comp_rem;
    const double t = sum + y;
    comp_rem = t - sum - y;
    sum = t;
    if (signbit(v)) --neg;
  }
  __device__ __forceinline__ double value() const {   // min_periods = 1
    if (nobs <= 0) return qnan();
    double r = sum / (double)nobs;
    if (same >= nobs) r = prev;
    else if (neg == 0 && r < 0.0) r = 0.0;
    else if (neg == nobs && r > 0.0) r = 0.0;
    return r;
  }
};

// pandas roll_var state (add_var / remove_var / calc_var), ddof 0
struct RollVar {
  double nobs, mean, ssq, comp_add, comp_rem, prev;
  int same;
  __device__ __forceinline__ void init(double first) {
    nobs = mean = ssq = comp_add = comp_rem = 0.0;
    same = 0;
    prev = first;
  }
  __device__ __forceinline__ void add(double v) {
    if (v != v) return;
    same = (v == prev) ? same + 1 : 1;
    prev = v;
    nobs += 1.0;
    const double pm = mean - comp_add;
    const double y = v - comp_add;
    const double t = y - mean;
    comp_add = t + mean - y;
    mean = nobs != 0.0 ? mean + t / nobs : 0.0;
    ssq = ssq + (v - pm) * (v - mean);
  }
  __device__ __forceinline__ void remove(double v) {
    if (v != v) return;
    nobs -= 1.0;
    if (nobs != 0.0) {
      const double pm = mean - comp_rem;
      const double y = v - comp_rem;
      const double t = y - mean;
      comp_rem = t + mean - y;
      mean = mean - t / nobs;
      ssq = ssq - (v - pm) * (v - mean);
    } else {
      mean = ssq = 0.0;
    }
  }
  __device__ __forceinline__ double var0() const {   // min_periods 1, ddof 0
    if (!(nobs >= 1.0 && nobs > 0.0)) return qnan();
    if (nobs == 1.0 || (double)same >= nobs) return 0.0;
    const double r = ssq / nobs;
    return r < 0.0 ? 0.0 : r;
  }
};

// pandas ewm(adjust=False, min_periods=1) state over a NaN-free close series
// (the step is ewm_step below)
struct Ewm {
  double w, old_wt;
  bool have;
};

struct FeatSel {
  const int64_t* slots;   // selected slots; NULL = slots [0, n) (context mode)
  int64_t n;
  double* feat[BQ_NUM_FEATURES];
  double* close;
  double a20, om20, a50, om50;
  int ema_div;            // om + alpha != 1.0 for a span: keep pandas' divide
  // context mode (bq_store_context_features)
  const int64_t* fresh_ts;   // device scalar: fresh = last == *fresh_ts && count > 0
  double* fresh;             // [n] 1.0 / 0.0 per counted fresh slot
  double* btc_out;           // [8] benchmark features, close, fresh flag
  int64_t btc_slot;
  int btc_counted;
};

// Four waves per 64 symbols, one recurrence chain each (the branch on the
// role is wave-uniform): wave 0 replays the true range and the ATR roll_mean,
// wave 1 both EWMs, wave 2 the 20-bar roll_mean, wave 3 the 20-bar roll_var.
// The chains are independent and each is the same operation sequence as one
// lane doing all of them, so the results are the pandas values bit for bit;
// a symbol's per-step work is spread over four waves (the replay is a
// latency-bound dependent chain per symbol: 10k symbols fill 157 blocks). The
// next chunk of the rings is loaded into registers while the current one is
// replayed from LDS. Waves 1-3 hand their results to wave 0 through LDS.
constexpr int SF_NT = 4 * WAVE;
constexpr int SF_LD = SF_CT * WAVE / SF_NT;   // elements per thread per field and chunk

template <bool EDIV>
__device__ __forceinline__ void ewm_step(Ewm& e, double x, double alpha, double om) {
  if (!e.have) {
    e.w = x;
    e.have = x == x;
    e.old_wt = 1.0;
    return;
  }
  if (x != x) {   // NaN gap: decay only (closes are NaN-free in the store)
    e.old_wt *= om;
    return;
  }
  e.old_wt *= om;
  if (e.w != x) {
    e.w = e.old_wt * e.w + alpha * x;
    // old_wt + alpha == om + alpha == 1.0 exactly for the store's spans
    // (checked on the host, EDIV = false): the divide is the identity
    if (EDIV || e.old_wt != om) e.w /= e.old_wt + alpha;
  }
  e.old_wt = 1.0;
}

template <bool EDIV>
__global__ __launch_bounds__(SF_NT) void store_features_kernel(const StoreArgs V, const FeatSel F) {
  __shared__ double sX[3][SF_CT * STG_PITCH];   // high, low, close chunk (transposed)
  __shared__ double sTR[SF_ATR][WAVE];          // per-symbol ring of true ranges (wave 0)
  __shared__ double sCL[2][SF_BB][WAVE];        // per-symbol rings of closes (waves 2, 3)
  __shared__ double sRes[6][WAVE];              // mean, var, ema20, ema50, last close, previous close
  __shared__ int sH[WAVE], sN[WAVE];
  __shared__ int64_t sRow[WAVE];
  const int lane = threadIdx.x & (WAVE - 1);
  const int role = threadIdx.x / WAVE;   // wave-uniform
  const int64_t i = (int64_t)blockIdx.x * WAVE + lane;
  const int M = V.M;
  int n = 0;
  bool fresh = false;
  if (i < F.n) {
    const int64_t s = F.slots ? F.slots[i] : i;
    n = V.count[s];
    fresh = !F.fresh_ts || (n > 0 && V.last[s] == *F.fresh_ts);
    if (role == 0) {
      sH[lane] = V.head[s];
      sRow[lane] = s * (int64_t)M;
    }
  } else if (role == 0) {
    sH[lane] = 0;
    sRow[lane] = 0;
  }
  // context mode: non-fresh slots are not replayed (except the benchmark,
  // whose features are needed whatever its freshness)
  const bool need = fresh || (F.fresh_ts && i == F.btc_slot);
  if (!need) n = 0;
  if (role == 0) sN[lane] = n;
  int nmax = n;   // equal in every wave: same symbols
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) nmax = max(nmax, __shfl_xor(nmax, d, WAVE));
  __syncthreads();

  Ewm e20 = {0.0, 1.0, false}, e50 = {0.0, 1.0, false};
  RollMean rm;
  RollVar var;
  rm.init();
  double pc = qnan(), c_last = qnan(), c_prev = qnan();
  double rh[SF_LD], rl[SF_LD], rc[SF_LD];
  auto load = [&](int t0) {
#pragma unroll
    for (int q = 0; q < SF_LD; ++q) {
      const int el = threadIdx.x + SF_NT * q;
      const int l = el / SF_CT, t = t0 + el % SF_CT;
      rh[q] = rl[q] = rc[q] = qnan();
      if (t < sN[l]) {
        const int64_t p = sRow[l] + ring_at(sH[l], t, M);
        rh[q] = V.f[BQ_HIGH][p];
        rl[q] = V.f[BQ_LOW][p];
        rc[q] = V.f[BQ_CLOSE][p];
      }
    }
  };
  if (nmax > 0) load(0);
  for (int t0 = 0; t0 < nmax; t0 += SF_CT) {
#pragma unroll
    for (int q = 0; q < SF_LD; ++q) {
      const int el = threadIdx.x + SF_NT * q;
      const int x = (el % SF_CT) * STG_PITCH + el / SF_CT;
      sX[0][x] = rh[q];
      sX[1][x] = rl[q];
      sX[2][x] = rc[q];
    }
    __syncthreads();
    if (t0 + SF_CT < nmax) load(t0 + SF_CT);   // in flight during the replay below
    const int m = min(SF_CT, n - t0);
    if (role == 0) {
      for (int j = 0; j < m; ++j) {
        const int t = t0 + j;
        const int x = j * STG_PITCH + lane;
        const double tr = true_range(sX[0][x], sX[1][x], pc);
        if (t >= SF_ATR) rm.remove(sTR[t % SF_ATR][lane]);
        rm.add(tr);
        sTR[t % SF_ATR][lane] = tr;
        pc = sX[2][x];
      }
    } else if (role == 1) {
      for (int j = 0; j < m; ++j) {
        const double c = sX[2][j * STG_PITCH + lane];
        ewm_step<EDIV>(e20, c, F.a20, F.om20);
        ewm_step<EDIV>(e50, c, F.a50, F.om50);
        c_prev = c_last;
        c_last = c;
      }
    } else if (role == 2) {
      for (int j = 0; j < m; ++j) {
        const int t = t0 + j;
        const double c = sX[2][j * STG_PITCH + lane];
        if (t >= SF_BB) rm.remove(sCL[0][t % SF_BB][lane]);
        rm.add(c);
        sCL[0][t % SF_BB][lane] = c;
      }
    } else {
      for (int j = 0; j < m; ++j) {
        const int t = t0 + j;
        const double c = sX[2][j * STG_PITCH + lane];
        if (t == 0) var.init(c);
        if (t >= SF_BB) var.remove(sCL[1][t % SF_BB][lane]);
        var.add(c);
        sCL[1][t % SF_BB][lane] = c;
      }
    }
    __syncthreads();
  }
  if (role == 1) {
    sRes[2][lane] = e20.w;
    sRes[3][lane] = e50.w;
    sRes[4][lane] = c_last;
    sRes[5][lane] = c_prev;
  } else if (role == 2) {
    sRes[0][lane] = rm.value();
  } else if (role == 3) {
    sRes[1][lane] = var.var0();
  }
  __syncthreads();
  if (role != 0 || i >= F.n) return;
  double ret = qnan(), ema20 = qnan(), ema50 = qnan(), trend = qnan(), atr_pct = qnan(), bbw = qnan();
  const double cl = sRes[4][lane], cp = sRes[5][lane];
  if (n >= 2) {   // _compute_symbol_features returns None below 2 bars (:249-250)
    ema20 = sRes[2][lane];
    ema50 = sRes[3][lane];
    const double a = rm.value();
    const double mu = sRes[0][lane];
    const double v = sRes[1][lane];
    const double sd = v == v ? sqrt(v) : 0.0;   // std(ddof=0).fillna(0)
    const double up = mu + (2.0 * sd), lo = mu - (2.0 * sd);
    ret = safe_pct(cl, cp);
    atr_pct = cl != 0.0 ? a / cl : 0.0;
    bbw = mu != 0.0 ? (up - lo) / fabs(mu) : 0.0;
    trend = ema50 != 0.0 ? (ema20 - ema50) / fabs(ema50) : 0.0;
  }
  const double close = n >= 1 ? cl : qnan();
  if (F.fresh_ts && i == F.btc_slot && F.btc_out) {
    F.btc_out[0] = ret;
    F.btc_out[1] = ema20;
    F.btc_out[2] = ema50;
    F.btc_out[3] = trend;
    F.btc_out[4] = atr_pct;
    F.btc_out[5] = bbw;
    F.btc_out[6] = close;
    F.btc_out[7] = fresh ? 1.0 : 0.0;
  }
  // context mode: a row is a counted fresh symbol or NaN
  const bool row = !F.fresh_ts || (fresh && (i != F.btc_slot || F.btc_counted));
  if (F.fresh) F.fresh[i] = row ? 1.0 : 0.0;
  const double nan = qnan();
  if (F.feat[BQ_F_RETURN]) F.feat[BQ_F_RETURN][i] = row ? ret : nan;
  if (F.feat[BQ_F_EMA20]) F.feat[BQ_F_EMA20][i] = row ? ema20 : nan;
  if (F.feat[BQ_F_EMA50]) F.feat[BQ_F_EMA50][i] = row ? ema50 : nan;
  if (F.feat[BQ_F_TREND]) F.feat[BQ_F_TREND][i] = row ? trend : nan;
  if (F.feat[BQ_F_ATR_PCT]) F.feat[BQ_F_ATR_PCT][i] = row ? atr_pct : nan;
  if (F.feat[BQ_F_BB_WIDTH]) F.feat[BQ_F_BB_WIDTH][i] = row ? bbw : nan;
  if (F.close) F.close[i] = row ? close : nan;
}

// ---- ordered export -------------------------------------------------------------
struct OutTab {
  int64_t* ts;
  double* f[BQ_NUM_INPUTS];
};

__global__ __launch_bounds__(256) void store_gather_kernel(const StoreArgs V, const int64_t* __restrict__ slots,
                                                           int64_t n_sel, const OutTab O, int64_t ld_out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int M = V.M;
  if (i >= n_sel * (int64_t)M) return;
  const int64_t r = i / M;
  const int t = (int)(i % M);
  const int64_t s = slots[r];
  const int n = V.count[s];
  const bool ok = t < n;
  const int64_t p = s * (int64_t)M + ring_at(V.head[s], ok ? t : 0, M);
  if (O.ts) O.ts[r * ld_out + t] = ok ? V.ts[p] : 0;
#pragma unroll
  for (int c = 0; c < BQ_NUM_INPUTS; ++c)
    if (O.f[c]) O.f[c][r * ld_out + t] = ok ? V.f[c][p] : qnan();
}

__host__ bool view_ok(const bq_store_view* v) {
  if (!v || !v->ts || !v->head || !v->count || !v->last || v->capacity < 0 || v->max_bars < 2 ||
      v->max_bars > BQ_STORE_MAX_BARS)
    return false;
  for (int c = 0; c < BQ_NUM_INPUTS; ++c)
    if (!v->field[c]) return false;
  return true;
}

__host__ StoreArgs to_args(const bq_store_view* v) {
  StoreArgs A;
  A.ts = v->ts;
  for (int c = 0; c < BQ_NUM_INPUTS; ++c) A.f[c] = v->field[c];
  A.head = v->head;
  A.count = v->count;
  A.last = v->last;
  A.cap = v->capacity;
  A.M = v->max_bars;
  return A;
}

}  // namespace bq

extern "C" {

int bq_store_update(const bq_store_view* st, const int64_t* slot, const int64_t* ts, const double* const* ohlcv,
                    const int64_t* seg_begin, int64_t n_seg, void* stream) {
  using namespace bq;
  if (!view_ok(st) || !slot || !ts || !ohlcv || !seg_begin || n_seg < 0 || n_seg > 0x7fffffff) return BQ_EINVAL;
  for (int c = 0; c < BQ_NUM_INPUTS; ++c)
    if (!ohlcv[c]) return BQ_EINVAL;
  if (n_seg == 0) return BQ_OK;
  UpdArgs U;
  U.slot = slot;
  U.ts = ts;
  for (int c = 0; c < BQ_NUM_INPUTS; ++c) U.f[c] = ohlcv[c];
  U.seg = seg_begin;
  hipLaunchKernelGGL(store_update_kernel, dim3((unsigned)n_seg), dim3(SU_NT), 0, (hipStream_t)stream, to_args(st), U);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

static int bq_launch_features_impl(const bq_store_view* st, bq::FeatSel& F, void* stream) {
  using namespace bq;
  // pandas: comass = (span - 1) / 2, alpha = 1 / (1 + comass)
  F.a20 = 1.0 / (1.0 + (20.0 - 1.0) / 2.0);
  F.om20 = 1.0 - F.a20;
  F.a50 = 1.0 / (1.0 + (50.0 - 1.0) / 2.0);
  F.om50 = 1.0 - F.a50;
  F.ema_div = (F.om20 + F.a20) != 1.0 || (F.om50 + F.a50) != 1.0;
  const unsigned blocks = (unsigned)((F.n + WAVE - 1) / WAVE);
  if (F.ema_div)
    hipLaunchKernelGGL(store_features_kernel<true>, dim3(blocks), dim3(SF_NT), 0, (hipStream_t)stream, to_args(st), F);
  else
    hipLaunchKernelGGL(store_features_kernel<false>, dim3(blocks), dim3(SF_NT), 0, (hipStream_t)stream, to_args(st), F);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

int bq_store_features(const bq_store_view* st, const int64_t* slots, int64_t n_sel, double* const* feat,
                      double* close_out, void* stream) {
  using namespace bq;
  if (!view_ok(st) || !slots || !feat || n_sel < 0) return BQ_EINVAL;
  if (n_sel == 0) return BQ_OK;
  FeatSel F;
  memset(&F, 0, sizeof F);
  F.slots = slots;
  F.n = n_sel;
  for (int i = 0; i < BQ_NUM_FEATURES; ++i) F.feat[i] = feat[i];
  F.close = close_out;
  F.btc_slot = -1;
  return bq_launch_features_impl(st, F, stream);
}

int bq_store_context_features(const bq_store_view* st, int64_t n, const int64_t* fresh_ts, int64_t btc_slot,
                              int btc_counted, double* const* feat, double* close_out, double* fresh_out,
                              double* btc_out, void* stream) {
  using namespace bq;
  if (!view_ok(st) || !fresh_ts || !feat || n < 0 || n > st->capacity || btc_slot >= n) return BQ_EINVAL;
  if (n == 0) return BQ_OK;
  FeatSel F;
  memset(&F, 0, sizeof F);
  F.slots = nullptr;
  F.n = n;
  for (int i = 0; i < BQ_NUM_FEATURES; ++i) F.feat[i] = feat[i];
  F.close = close_out;
  F.fresh_ts = fresh_ts;
  F.fresh = fresh_out;
  F.btc_out = btc_slot >= 0 ? btc_out : nullptr;
  F.btc_slot = btc_slot;
  F.btc_counted = btc_counted;
  return bq_launch_features_impl(st, F, stream);
}

int bq_store_gather(const bq_store_view* st, const int64_t* slots, int64_t n_sel, int64_t* ts_out,
                    double* const* out, int64_t ld_out, void* stream) {
  using namespace bq;
  if (!view_ok(st) || !slots || !out || n_sel < 0 || ld_out < st->max_bars) return BQ_EINVAL;
  if (n_sel == 0) return BQ_OK;
  OutTab O;
  O.ts = ts_out;
  for (int c = 0; c < BQ_NUM_INPUTS; ++c) O.f[c] = out[c];
  const int64_t items = n_sel * (int64_t)st->max_bars;
  hipLaunchKernelGGL(store_gather_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     to_args(st), slots, n_sel, O, ld_out);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
