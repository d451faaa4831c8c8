// Sliding order statistic over a compile-time window, the window kept SORTED
// in W registers (gfx950). Shared by the rolling order statistics
// (bq_rolling.hip slide_rank_kernel) and the fused GradualGainerRetest
// leadership (bq_lead.hip).
//
// NaNs and the slots not holding a number are placeholders: with n numbers
// in the window, a(n) = int(q (n - 1)) (median: (n - 1) / 2) and
// B(n) = K - a(n) placeholders sit at the bottom (-inf), the rest at the top
// (+inf), so the a-th smallest number is s[K] and the next one s[K + 1] for
// any n (B(n) + n <= W since q < 1). One step replaces the leaving value `o`
// by the entering value `v` with no search and no index arithmetic: the
// array with one copy of o removed is
//   b[i] = s[i] < o ? s[i] : s[i+1]        (s[W] = +inf)
// and inserting v into a sorted b is a clamp per slot,
//   s'[i] = max(b[i-1], min(v, b[i]))      (b[-1] = -inf),
// i.e. 1 compare, 2 selects, 1 min, 1 max per slot. n changes by at most 1
// per step and B by at most 1 with it, so a step keeps the split by choosing
// which kind of placeholder leaves or enters (a NaN leaving or entering is a
// placeholder leaving or entering). Zeros enter as +0 (x + 0.0), so the
// multiset's values are the exact keys' values; order statistics are a pure
// function of the multiset, so results equal any other exact kernel's bit for
// bit.
//
// The step is written for a loop that advances ONE step per iteration: a
// chunk of steps unrolled around it makes the compiler hold a second copy of
// the window (and a log-step barrel shift of the split does too), which at
// w = 96 cost 424 registers, one wave per SIMD; stepwise the w = 96 window
// and its update take ~215 (two waves per SIMD).
#pragma once
#include "bq_device.h"

namespace bq {

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

template <int W, int K, bool MED>
struct SlideRank {
  static_assert(K >= 0 && K < W, "rank slot inside the window");
  double s[W];
  int n, nb;
  double q;

  // empty window: B(0) = K + 1 placeholders at the bottom
  __device__ __forceinline__ void init(double q_) {
    const double inf = __builtin_inf();
    q = q_;
    n = 0;
    nb = K + 1;
#pragma unroll
    for (int i = 0; i < W; ++i) s[i] = i <= K ? -inf : inf;
  }

  __device__ __forceinline__ int bottom(int nn) const {
    if (nn < 1) return K + 1;
    if constexpr (MED) return K - ((nn - 1) >> 1);
    else return K - (int)(q * (double)(nn - 1));
  }

  // vin enters, vout leaves (NaN: a placeholder — also for a step whose
  // leaving position was never entered)
  __device__ __forceinline__ void step(double vin, double vout) {
    const double inf = __builtin_inf();
    const bool in_num = vin == vin, out_num = vout == vout;
    const int n2 = n + (in_num ? 1 : 0) - (out_num ? 1 : 0);
    const int nb2 = bottom(n2);
    // a leaving placeholder is a bottom one when B drops, an entering one a
    // bottom one when B grows (otherwise top; both top when nothing changes:
    // removing an absent +inf and inserting +inf leaves the array as is)
    const double o = out_num ? vout + 0.0 : (nb2 < nb ? -inf : inf);
    const double v = in_num ? vin + 0.0 : (nb2 > nb ? -inf : inf);
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
  }

  // quantile(q) with linear interpolation (lower: the lower order statistic,
  // no interpolation) or the median of the window's numbers; NaN below minp
  __device__ __forceinline__ double value(int minp, bool lower) const {
    if (!(n >= minp && n > 0)) return qnan();
    constexpr int K1 = K + 1 < W ? K + 1 : K;
    const double lo = s[K];
    if constexpr (MED) {
      return (n & 1) ? lo : (lo + s[K1]) / 2.0;
    } else {
      const double idxf = q * (double)(n - 1);
      const int idx = (int)idxf;
      return ((double)idx == idxf || lower) ? lo : lo + (s[K1] - lo) * (idxf - (double)idx);
    }
  }
};

}  // namespace bq
