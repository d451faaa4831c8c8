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

// A^n for 0 <= n < 2^NB from the table apow[j] = A^(2^j).
template <int NB>
__device__ __forceinline__ double pow_bits(const double* apow, int n) {
  double r = 1.0;
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (n & (1 << j)) r *= apow[j];
  return r;
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

// 100 - 100 / (1 + a / b) with IEEE inf/NaN semantics, as pandas evaluates it.
__device__ __forceinline__ double oscillator(double a, double b) {
  double rs = a / b;
  return 100.0 - (100.0 / (1.0 + rs));
}

// x / n for a small integer n via one reciprocal and one FMA correction:
// the correctly rounded quotient except in rare ties (well inside the 1e-9
// parity tolerance), at a fraction of the cost of an IEEE fp64 divide.
__device__ __forceinline__ double div_exact(double x, double n) {
  const double r = 1.0 / n;   // uniform per window: hoisted by the compiler
  double q = x * r;
  const double e = fma(-q, n, x);
  return fma(e, r, q);
}

// shared/utils.py:20-23
__device__ __forceinline__ double safe_pct(double cur, double prev) {
  if (prev == 0.0) return 0.0;
  return (cur - prev) / fabs(prev);
}

}  // namespace bq
