// Device-side building blocks shared by the binquant_amd HIP kernels (gfx950).
//
// Numerics contract: every translation unit is compiled with
// -ffp-contract=off so that the element-wise formulas replay pandas' float64
// arithmetic operation-for-operation (pandas' Cython kernels are built without
// FMA contraction). Where a fused multiply-add is wanted (scan carries, which
// are approximations that the exact replay then corrects) it is written out
// explicitly with fma().
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace bq {

constexpr int WAVE = 64;

__device__ __forceinline__ double qnan() { return __builtin_nan(""); }

// pandas' window operations (rolling *, ewm) see +-inf as missing: they run on
// np.where(np.isinf(values), np.nan, values) (BaseWindow._prep_values,
// pandas/core/window/rolling.py). ffill, element-wise ops and np.quantile keep
// infinities. x - x == 0 is false exactly for NaN and +-inf.
__device__ __forceinline__ double win_val(double x) { return x - x == 0.0 ? x : qnan(); }
// the same rule as an observation test (one add + one compare), for loops
// that already select on their observation flag
__device__ __forceinline__ bool win_ok(double x) { return x - x == 0.0; }

// ---- compensated (double-double) accumulation ------------------------------
struct dd {
  double hi, lo;
};

// Knuth TwoSum: s + e == a + b exactly.
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

__device__ __forceinline__ dd dd_add(dd a, dd b) {
  double s, e;
  two_sum(a.hi, b.hi, s, e);
  e += a.lo + b.lo;
  double hi = s + e;
  double lo = e - (hi - s);
  return {hi, lo};
}

__device__ __forceinline__ dd dd_add1(dd a, double b) {
  double s, e;
  two_sum(a.hi, b, s, e);
  e += a.lo;
  double hi = s + e;
  double lo = e - (hi - s);
  return {hi, lo};
}

__device__ __forceinline__ double dd_round(dd a) { return a.hi + a.lo; }

// ---- wavefront (64-lane) scans ---------------------------------------------
// Inclusive prefix of a double-double across the wave (Hillis-Steele over
// __shfl_up; lane i ends with x_0 + ... + x_i).
__device__ __forceinline__ dd wave_incl_scan_dd(dd x, int lane) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    double vh = __shfl_up(x.hi, d, WAVE);
    double vl = __shfl_up(x.lo, d, WAVE);
    if (lane >= d) x = dd_add({vh, vl}, x);
  }
  return x;
}

// Inclusive scan of the affine maps y -> A*y + B_i with a wave-uniform decay A
// per element-group: S_i = B_i + A * S_{i-1}. apow[j] = A^(2^j).
__device__ __forceinline__ double wave_incl_scan_affine(double b, const double* apow, int lane) {
#pragma unroll
  for (int j = 0, d = 1; d < WAVE; d <<= 1, ++j) {
    double v = __shfl_up(b, d, WAVE);
    if (lane >= d) b = fma(apow[j], v, b);
  }
  return b;
}

__device__ __forceinline__ int wave_incl_scan_max(int x, int lane) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    int v = __shfl_up(x, d, WAVE);
    if (lane >= d) x = max(x, v);
  }
  return x;
}

// ---- DPP cross-lane moves (VALU, no LDS traffic) ----------------------------
// row_shr:n shifts within each 16-lane row; wave_shr:1 shifts the whole wave by
// one lane (GFX9 DPP). Lanes without a source read 0 (bound_ctrl), which is the
// identity of every combine used here (sums, affine maps, max of (index+1)).
constexpr int DPP_ROW_SHR1 = 0x111;
constexpr int DPP_ROW_SHR2 = 0x112;
constexpr int DPP_ROW_SHR4 = 0x114;
constexpr int DPP_ROW_SHR8 = 0x118;
constexpr int DPP_WAVE_SHR1 = 0x138;

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true);
}

__device__ __forceinline__ double readlane_f64(double x, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
  return __hiloint2double(hi, lo);
}

// Inclusive wave prefix of a double-double: DPP row scans, then the row totals
// (lanes 15, 31, 47) folded in through readlane.
__device__ __forceinline__ dd wave_scan_dd_dpp(dd x, int lane) {
#define BQ_DD_STEP(CTRL)                                       \
  {                                                            \
    const dd v = {dpp_f64<CTRL>(x.hi), dpp_f64<CTRL>(x.lo)};   \
    x = dd_add(v, x);                                          \
  }
  BQ_DD_STEP(DPP_ROW_SHR1)
  BQ_DD_STEP(DPP_ROW_SHR2)
  BQ_DD_STEP(DPP_ROW_SHR4)
  BQ_DD_STEP(DPP_ROW_SHR8)
#undef BQ_DD_STEP
  const dd r0 = {readlane_f64(x.hi, 15), readlane_f64(x.lo, 15)};
  const dd r1 = {readlane_f64(x.hi, 31), readlane_f64(x.lo, 31)};
  const dd r2 = {readlane_f64(x.hi, 47), readlane_f64(x.lo, 47)};
  const dd c1 = r0, c2 = dd_add(r0, r1), c3 = dd_add(c2, r2);
  const int row = lane >> 4;
  if (row > 0) {
    const dd c = row == 1 ? c1 : (row == 2 ? c2 : c3);
    x = dd_add(c, x);
  }
  return x;
}

// Inclusive wave max of non-negative ints (DPP rows + readlane).
__device__ __forceinline__ int wave_scan_max_dpp(int x, int lane) {
  x = max(x, dpp_i32<DPP_ROW_SHR1>(x));
  x = max(x, dpp_i32<DPP_ROW_SHR2>(x));
  x = max(x, dpp_i32<DPP_ROW_SHR4>(x));
  x = max(x, dpp_i32<DPP_ROW_SHR8>(x));
  const int r0 = __builtin_amdgcn_readlane(x, 15);
  const int r1 = max(r0, __builtin_amdgcn_readlane(x, 31));
  const int r2 = max(r1, __builtin_amdgcn_readlane(x, 47));
  const int row = lane >> 4;
  const int c = row == 0 ? 0 : (row == 1 ? r0 : (row == 2 ? r1 : r2));
  return max(x, c);
}

// A^n for 0 <= n < 2^NB from the table apow[j] = A^(2^j).
template <int NB>
__device__ __forceinline__ double pow_bits(const double* apow, int n) {
  double r = 1.0;
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (n & (1 << j)) r *= apow[j];
  return r;
}

// Inclusive scan of the affine maps b_i + A * S_{i-1} (apow[j] = A^(2^j), a
// wave-uniform decay) on DPP rows + readlane row carries: the shfl ladder's
// result up to rounding (a different association).
__device__ __forceinline__ double wave_scan_affine_dpp(double b, const double* apow, int lane) {
  b = fma(apow[0], dpp_f64<DPP_ROW_SHR1>(b), b);   // out-of-row sources read 0
  b = fma(apow[1], dpp_f64<DPP_ROW_SHR2>(b), b);
  b = fma(apow[2], dpp_f64<DPP_ROW_SHR4>(b), b);
  b = fma(apow[3], dpp_f64<DPP_ROW_SHR8>(b), b);
  const double c1 = readlane_f64(b, 15);
  const double c2 = fma(apow[4], c1, readlane_f64(b, 31));
  const double c3 = fma(apow[4], c2, readlane_f64(b, 47));
  const int row = lane >> 4;
  if (row > 0) {
    const double c = row == 1 ? c1 : (row == 2 ? c2 : c3);
    b = fma(pow_bits<5>(apow, (lane & 15) + 1), c, b);
  }
  return b;
}

// wave_scan_affine_dpp with the lane-constant row-carry factor
// rp = pow_bits<5>(apow, (lane & 15) + 1) computed once by the caller
__device__ __forceinline__ double wave_scan_affine_dpp_rp(double b, const double* apow, double rp, int lane) {
  b = fma(apow[0], dpp_f64<DPP_ROW_SHR1>(b), b);
  b = fma(apow[1], dpp_f64<DPP_ROW_SHR2>(b), b);
  b = fma(apow[2], dpp_f64<DPP_ROW_SHR4>(b), b);
  b = fma(apow[3], dpp_f64<DPP_ROW_SHR8>(b), b);
  const double c1 = readlane_f64(b, 15);
  const double c2 = fma(apow[4], c1, readlane_f64(b, 31));
  const double c3 = fma(apow[4], c2, readlane_f64(b, 47));
  const int row = lane >> 4;
  if (row > 0) {
    const double c = row == 1 ? c1 : (row == 2 ? c2 : c3);
    b = fma(rp, c, b);
  }
  return b;
}

// ---- element-wise restatements of the pandas formulas ----------------------
// delta.where(delta > 0, 0): NaN -> 0   (coinrule/bb_extreme_reversion.py:145)
__device__ __forceinline__ double gain_of(double d) { return d > 0.0 ? d : 0.0; }
// -(delta.where(delta < 0, 0))          (coinrule/bb_extreme_reversion.py:146)
__device__ __forceinline__ double loss_of(double d) { return d < 0.0 ? -d : 0.0; }

// concat([h-l, |h-pc|, |l-pc|], axis=1).max(axis=1) skips NaN, so the first
// row is h-l (market_regime/live_market_context_accumulator.py:256-264).
__device__ __forceinline__ double true_range(double h, double l, double pc) {
  double a = h - l;
  double b = fabs(h - pc);
  double c = fabs(l - pc);
  return fmax(a, fmax(b, c));   // fmax ignores NaN operands, like skipna
}

__device__ __forceinline__ double ohlc4(double o, double h, double l, double c) {
  return (((o + h) + l) + c) / 4.0;
}

__device__ __forceinline__ double typical_price(double h, double l, double c) {
  return ((h + l) + c) / 3.0;
}

// 100 - 100 / (1 + a / b) for a, b >= 0 (RSI / MFI), written with one divide:
// 100 a / (a + b). Same special cases as pandas' form (b = 0 < a -> 100,
// a = b = 0 -> NaN, a = 0 < b -> 0); finite values agree to a few ulps.
__device__ __forceinline__ double oscillator(double a, double b) {
  return (100.0 * a) / (a + b);
}

// x / n for a small integer n via one reciprocal and one FMA correction,
// r = RN(1 / n) computed once on the host. By Markstein's theorem (r within
// half an ulp of 1/n, q = RN(x r) a faithful quotient, e = x - q n exact by
// FMA) RN(q + e r) is the correctly rounded x / n for finite x away from
// underflow: 0 mismatches in 51M random cases over n = 1..256, exponents
// -300..300 (tests/csrc/div_exact_check.c, run by tests/test_div_exact.py).
// 3 instructions against ~10 (one quarter-rate rcp) for the IEEE divide.
__device__ __forceinline__ double div_exact(double x, double n, double r) {
  double q = x * r;
  const double e = fma(-q, n, x);
  return fma(e, r, q);
}

// div_exact where bit-equality with an IEEE divide is contractual (pandas
// replays): zero, infinite and NaN x keep q = x r (±0, ±inf, NaN, as x / n),
// and the rare |x| < 2^-960 takes the IEEE divide (a branch skipped when no
// lane needs it).
__device__ __forceinline__ double div_count(double x, double n, double r) {
  if (__builtin_expect(fabs(x) < 0x1p-960 && x != 0.0, 0)) return x / n;
  const double q = x * r;
  const double c = fma(fma(-q, n, x), r, q);
  return ((x == 0.0) | !(fabs(q) <= __DBL_MAX__)) ? q : c;
}

// 1 / v with the hardware reciprocal and two Newton steps (v > 0)
__device__ __forceinline__ double rcp_nr(double v) {
  double r = __builtin_amdgcn_rcp(v);
  r = fma(r, fma(-v, r, 1.0), r);
  return fma(r, fma(-v, r, 1.0), r);
}

// log(c / p) as pandas forms it (the IEEE quotient, then its log). A 15-minute
// ratio is almost always within 1/8 of 1: there log(m) = 2 atanh(s),
// s = (m - 1) / (m + 1), m - 1 exact, seven odd terms to below half an ulp of
// the sum (|s| <= 1/15, s^16 / 17 < 2^-66): ~20 double ops against ~76 for
// the library log, within 2 ulp of it. Larger moves, zero / negative / NaN
// prices take the library log (a branch, skipped when no lane needs it).
__device__ __forceinline__ double log_return(double c, double p) {
  const double m = c / p;
  const double d = m - 1.0;
  if (__builtin_expect(!(fabs(d) <= 0.125), 0)) return log(m);
  const double s = d * rcp_nr(2.0 + d), z = s * s;
  double r = 1.0 / 15.0;
  r = fma(r, z, 1.0 / 13.0);
  r = fma(r, z, 1.0 / 11.0);
  r = fma(r, z, 1.0 / 9.0);
  r = fma(r, z, 1.0 / 7.0);
  r = fma(r, z, 1.0 / 5.0);
  r = fma(r, z, 1.0 / 3.0);
  return (2.0 * s) * fma(r, z, 1.0);
}

// sqrt for v >= 0 from the hardware reciprocal square root plus one
// Newton/Goldschmidt correction (~2^-46 relative; the IEEE lowering spends
// ~15 instructions on scaling and two iterations). v == 0 -> 0.
__device__ __forceinline__ double sqrt_nr(double v) {
  const double r = __builtin_amdgcn_rsq(v);
  const double s = v * r;
  const double h = 0.5 * r;
  const double e = fma(-s, s, v);
  const double q = fma(h, e, s);
  return v > 0.0 ? q : 0.0;
}

// ---- lane-per-symbol staging (sequential state machines) -------------------
// A wave owns 64 symbols and walks them in chunks of CT candles. A chunk of a
// [S][ld] row-major array is read coalesced (lane i of pass k takes element
// e = i + 64k: symbol e / CT, candle e % CT, so CT consecutive lanes read one
// symbol's contiguous CT * 8 bytes) and transposed through LDS as [CT][PITCH]
// so that lane l then walks symbol l. PITCH = 64 + 2 keeps both the transposed
// writes and the per-lane reads free of bank conflicts for 8-byte elements.
constexpr int STG_PITCH = WAVE + 2;

// 64-bit payload type of __builtin_amdgcn_raw_buffer_store_b64
typedef unsigned int bq_u32x2 __attribute__((__vector_size__(8)));

template <int CT>
__device__ __forceinline__ void stage_load(const double* __restrict__ base, int64_t ld, int64_t sym0, int64_t S,
                                           int t0, int T, int lane, double (&r)[CT]) {
  // every lane loads a clamped, valid address (S, T >= 1) and selects NaN
  // outside the panel: no branch around a load, so the waits for a
  // prefetched chunk stay counted (vmcnt(N)) instead of draining the stores
#pragma unroll
  for (int k = 0; k < CT; ++k) {
    const int e = lane + WAVE * k;
    const int64_t s = sym0 + e / CT;
    const int t = t0 + e % CT;
    const int64_t sc = s < S ? s : S - 1;
    const int tc = t < 0 ? 0 : t < T ? t : T - 1;
    const double v = base[sc * ld + tc];
    r[k] = (s < S && t >= 0 && t < T) ? v : qnan();
  }
}

template <int CT>
__device__ __forceinline__ void stage_put(double* lds, int lane, const double (&r)[CT]) {
#pragma unroll
  for (int k = 0; k < CT; ++k) {
    const int e = lane + WAVE * k;
    lds[(e % CT) * STG_PITCH + e / CT] = r[k];
  }
}

// LDS [CT][PITCH] (written by lane = symbol) -> [S][ld] rows, coalesced.
// Buffer stores issued by every lane through a per-wave descriptor over the
// wave's rows: elements outside the panel (and every element when base is
// null) get an offset past the range, which the hardware drops — no branch
// around a store, so later waits stay counted. Host: 64 * ld * 8 < 2^31.
template <int CT, typename OutT>
__device__ __forceinline__ void stage_store(const double* lds, OutT* __restrict__ base, int64_t ld, int64_t sym0,
                                            int64_t S, int t0, int T, int lane) {
  const int64_t rows = S - sym0 < WAVE ? S - sym0 : WAVE;
  const int nbytes = base ? (int)(rows * ld * (int64_t)sizeof(OutT)) : 0;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base ? base + sym0 * ld : nullptr, 0, nbytes, 0x00020000);
#pragma unroll
  for (int k = 0; k < CT; ++k) {
    const int e = lane + WAVE * k;
    const int r = e / CT;
    const int t = t0 + e % CT;
    const bool ok = r < rows && t < T;
    const unsigned off = ok ? (unsigned)(((int64_t)r * ld + t) * (int64_t)sizeof(OutT)) : (unsigned)nbytes;
    const double v = lds[(e % CT) * STG_PITCH + r];
    if constexpr (sizeof(OutT) == 1)
      __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(OutT)v, rs, off, 0, 0);
    else
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(bq_u32x2, (double)(OutT)v), rs, off, 0, 0);
  }
}

// ---- timestamp search (ascending int64 ms) ---------------------------------
// first index i in [0, n) with ts[i] >= key (n if none)
__device__ __forceinline__ int lower_bound_i64(const int64_t* __restrict__ ts, int n, int64_t key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (ts[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// lower_bound with a guess first: on a regular grid (the kline rows) the
// index of key is (key - ts[0]) / step with step = (ts[n-1] - ts[0]) / (n - 1);
// the guess is taken only when ts[g-1] < key <= ts[g] holds, so the result is
// lower_bound's for any row (a gap or an irregular row falls back to the
// binary search): two loads instead of ~11 dependent ones per search.
__device__ __forceinline__ int lower_bound_guess(const int64_t* __restrict__ ts, int n, int64_t key, int64_t t0v,
                                                 int64_t step) {
  if (step > 0) {
    int64_t g = key <= t0v ? 0 : (key - t0v + step - 1) / step;
    g = g > n ? n : g;
    const bool ok = (g == 0 || ts[g - 1] < key) && (g == n || ts[g] >= key);
    if (ok) return (int)g;
  }
  return lower_bound_i64(ts, n, key);
}

// shared/utils.py:20-23
__device__ __forceinline__ double safe_pct(double cur, double prev) {
  if (prev == 0.0) return 0.0;
  return (cur - prev) / fabs(prev);
}


// ---- line-covering stores ---------------------------------------------------
// A lane holding K consecutive fp64 candles (K/2 16-byte pieces) stores them
// with K/2 instructions, each covering 16 bytes of every 8K bytes: 1/2 (K = 4)
// or 1/4 (K = 8) of each 128-byte line per instruction. At full-chip write
// rates that pattern streams ~20 % below whole-line coverage
// (tools/coalesce_ceiling.hip). line_exchange moves the pieces between lanes
// with v_permlane32_swap / v_permlane16_swap (no LDS) so that register m holds
// candles [128 m, 128 m + 128) of the wave's slice, lane L at candle offset
// line_offset<K>(L) + 128 m: each store instruction writes one contiguous KiB
// (lanes permuted within it). Every lane of the wave must execute it.
// Checked on the GPU by tools/permlane_check.hip.
typedef double dbl2 __attribute__((ext_vector_type(2)));

union DwordsOf2 {
  dbl2 d;
  unsigned u[4];
};

// lanes 32-63 of a <-> lanes 0-31 of b
__device__ __forceinline__ void swap_halves(dbl2& a, dbl2& b) {
  DwordsOf2 x, y;
  x.d = a;
  y.d = b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(x.u[i], y.u[i], false, false);
    x.u[i] = r[0];
    y.u[i] = r[1];
  }
  a = x.d;
  b = y.d;
}

// rows 1 and 3 of a <-> rows 0 and 2 of b (rows of 16 lanes)
__device__ __forceinline__ void swap_rows(dbl2& a, dbl2& b) {
  DwordsOf2 x, y;
  x.d = a;
  y.d = b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(x.u[i], y.u[i], false, false);
    x.u[i] = r[0];
    y.u[i] = r[1];
  }
  a = x.d;
  b = y.d;
}

template <int K>
__device__ __forceinline__ void line_exchange(dbl2 (&p)[K / 2]) {
  static_assert(K == 4 || K == 8, "line_exchange: 4 or 8 candles per lane");
  if constexpr (K == 4) {
    swap_halves(p[0], p[1]);
  } else {   // 4 x 4 transpose of (row, piece): two butterfly stages
    swap_halves(p[0], p[2]);
    swap_halves(p[1], p[3]);
    swap_rows(p[0], p[1]);
    swap_rows(p[2], p[3]);
  }
}

template <int K>
__device__ __forceinline__ int line_offset(int lane) {
  if constexpr (K == 4) return lane < 32 ? 4 * lane : 4 * (lane - 32) + 2;
  else return 8 * (lane & 15) + 2 * (lane >> 4);
}


// Row stores of a lane's K consecutive candles starting at candle tb of `row`
// through line_exchange. vec (16-byte aligned row, wave-uniform) selects the
// exchanged vector path, executed by every lane; full = every candle of the
// wave's slice is < T (drops the range checks). Non-temporal: the outputs
// are streamed, not re-read by the kernel.
template <int K>
__device__ __forceinline__ void store_lines(double* __restrict__ row_, int tb, int T, bool vec, const double (&x)[K],
                                            bool full = false) {
  typedef __attribute__((address_space(1))) double gd;
  typedef __attribute__((address_space(1))) dbl2 gd2;
  gd* row = (gd*)row_;
  if (vec) {
    dbl2 p[K / 2];
#pragma unroll
    for (int j = 0; j < K / 2; ++j) p[j] = dbl2{x[2 * j], x[2 * j + 1]};
    line_exchange<K>(p);
    const int lane = __lane_id();
    const int t = tb - K * lane + line_offset<K>(lane);
#pragma unroll
    for (int m = 0; m < K / 2; ++m) {
      const int u = t + 128 * m;
      if (full || u + 2 <= T) __builtin_nontemporal_store(p[m], reinterpret_cast<gd2*>(row + u));
      else if (u < T) row[u] = p[m].x;
    }
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (tb + k < T) row[tb + k] = x[k];
  }
}


// x = lo .. 0 through f; UNROLL (lo a compile-time constant after inlining)
// unrolls the walk completely, otherwise the compiler's default applies.
template <bool UNROLL, typename F>
__device__ __forceinline__ void walk_window(int lo, F&& f) {
  if constexpr (UNROLL) {
#pragma unroll
    for (int x = lo; x <= 0; ++x) f(x);
  } else {
    for (int x = lo; x <= 0; ++x) f(x);
  }
}


// Inverse of line_exchange (each stage is an involution: apply them in
// reverse order).
template <int K>
__device__ __forceinline__ void line_unexchange(dbl2 (&p)[K / 2]) {
  static_assert(K == 4 || K == 8, "line_unexchange: 4 or 8 candles per lane");
  if constexpr (K == 4) {
    swap_halves(p[0], p[1]);
  } else {
    swap_rows(p[0], p[1]);
    swap_rows(p[2], p[3]);
    swap_halves(p[0], p[2]);
    swap_halves(p[1], p[3]);
  }
}

// Row loads in the line-covering order: issues the lane's K/2 pieces of the
// wave's slice (lane L: candles line_offset<K>(L) + 128 m), each load
// instruction reading one contiguous KiB; candles >= T read as `fill`. The
// pieces land in x (x[2m], x[2m+1]) in exchanged order: line_unexchange_x
// turns them into the lane's K consecutive candles once they have arrived (a
// prefetch issues the loads a tile ahead and exchanges at use). vec
// (16-byte aligned row) is wave-uniform; every lane executes both steps.
template <int K>
__device__ __forceinline__ void load_pieces(const double* __restrict__ row, int tb, int T, double (&x)[K],
                                            double fill) {
  const int lane = __lane_id();
  const int t = tb - K * lane + line_offset<K>(lane);
#pragma unroll
  for (int m = 0; m < K / 2; ++m) {
    const int u = t + 128 * m;
    if (u + 2 <= T) {
      const dbl2 v = *reinterpret_cast<const dbl2*>(row + u);
      x[2 * m] = v.x;
      x[2 * m + 1] = v.y;
    } else {
      x[2 * m] = u < T ? row[u] : fill;
      x[2 * m + 1] = fill;
    }
  }
}

template <int K>
__device__ __forceinline__ void line_unexchange_x(double (&x)[K]) {
  dbl2 p[K / 2];
#pragma unroll
  for (int m = 0; m < K / 2; ++m) p[m] = dbl2{x[2 * m], x[2 * m + 1]};
  line_unexchange<K>(p);
#pragma unroll
  for (int m = 0; m < K / 2; ++m) {
    x[2 * m] = p[m].x;
    x[2 * m + 1] = p[m].y;
  }
}

}  // namespace bq
