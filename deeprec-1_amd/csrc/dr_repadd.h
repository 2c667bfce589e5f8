// dr_repadd.h -- k in-order fp32 additions of one term, exactly, in O(log)
// steps: rep_add(s, x, k) == fl(...fl(fl(s + x) + x)... + x) (k additions,
// round-to-nearest-even after each), bit for bit.
//
// A long run's serial gradient sum (segment_reduction_ops.cc:391-404: one
// fp32 add per position, ascending) often adds the same term many times in
// a row -- DIN's padding id: every padded history position of a sample
// carries that sample's his_sum gradient, ~50 identical terms per sample.
// Within one binade of the running sum the grid is fixed (ulp u), and while
// the exact sums stay in it every add moves the sum by the same whole number
// of ulps, rint(x / u) -- for a rounding tie (x / u = m + 1/2) only from an
// even sum, which every tie leaves.  So after one plain add, the next n adds
// are s1 + n * rint(x / u) ulps, computed exactly in double, n as far as the
// binade allows; an add that leaves the sum unchanged (x = 0, x below half an
// ulp, NaN, Inf) ends the walk.  The steps near a binade edge or a sign
// change, a tie from an odd sum, zero and subnormal sums are plain adds.
//
// Header-only and host-compilable (tests/test_repadd_host.py checks it
// against the plain loop on the CPU).
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define DR_HD __host__ __device__
#else
#define DR_HD
#endif

namespace dr {

DR_HD inline uint32_t f32_bits(float f) {
  uint32_t b;
  __builtin_memcpy(&b, &f, 4);
  return b;
}

// The common case in integer arithmetic, no branches but the verdict: all k
// adds round on s's own grid (s normal, x normal and at most 2^25 ulps below
// s's, the exact sums inside s's binade, no tie from an odd s).  With a = s
// in ulps (2^23 + mantissa) and x = xu ulps along s's sign, each add moves a
// by D = rint(xu) (ties to even); the exact sum a + j D + xu is checked as
// A' + f with A' = a + (j + 1) D and f = xu - D in [-1/2, 1/2] (only its
// sign matters against the integer bounds).  Returns false to leave it to
// the general walk.
DR_HD inline bool rep_add_grid(float s, float x, int64_t k, float* out) {
  const uint32_t bs = f32_bits(s), bx = f32_bits(x);
  const int es = (int)((bs >> 23) & 0xFF), ex = (int)((bx >> 23) & 0xFF);
  const int sh = es - ex;   // xu = mx / 2^sh
  if (es == 0 || es == 0xFF || ex == 0 || sh < 1 || sh > 25) return false;
  const int64_t mx = (int64_t)((bx & 0x7FFFFFu) | 0x800000u);
  const int64_t ip = mx >> sh, fr = mx & (((int64_t)1 << sh) - 1), half = (int64_t)1 << (sh - 1);
  const bool up = fr > half || (fr == half && (ip & 1));   // |xu| rounded up
  const bool tie = fr == half;
  const int64_t a = (int64_t)(bs & 0x7FFFFFu) | 0x800000;
  if (tie && (a & 1)) return false;
  const int64_t dabs = ip + (up ? 1 : 0);
  const bool grow = ((bs ^ bx) >> 31) == 0;   // x along s's sign
  const int64_t D = grow ? dabs : -dabs;
  // sign of f = xu - D along the magnitude: |xu| - dabs is < 0 when rounded
  // up with a fraction, > 0 when rounded down with one, 0 when exact
  int fs = fr == 0 ? 0 : (up ? -1 : 1);
  if (!grow) fs = -fs;
  const int64_t lo = 0x800000, hi = 0x1000000;
  const int64_t a1 = a + D, ak = a + k * D;   // A' of the first and the last add
  auto in_grid = [&](int64_t ap) {
    const bool below_hi = fs < 0 ? ap <= hi : ap < hi;
    const bool above_lo = fs < 0 ? ap >= lo + 1 : ap >= lo;
    return below_hi && above_lo;
  };
  if (!in_grid(a1) || !in_grid(ak)) return false;
  *out = __builtin_bit_cast(float, (bs & 0x80000000u) + ((uint32_t)es << 23) + (uint32_t)(ak - lo));
  return true;
}

// rep_add_grid in 32-bit integer arithmetic for a short segment (1 < k <
// 128: |k D| <= 2^30, no overflow) -- the form a serial device walk takes
// per segment: ~25 dependent 32-bit ops instead of rep_add's 64-bit and
// double-precision ones.  Same verdict and result as rep_add_grid.
DR_HD inline bool rep_add_grid32(float s, float x, int32_t k, float* out) {
  const uint32_t bs = f32_bits(s), bx = f32_bits(x);
  const int es = (int)((bs >> 23) & 0xFF), ex = (int)((bx >> 23) & 0xFF);
  const int sh = es - ex;
  if (k < 2 || k > 127 || es == 0 || es == 0xFF || ex == 0 || sh < 1 || sh > 25) return false;
  const uint32_t mx = (bx & 0x7FFFFFu) | 0x800000u;
  const uint32_t ip = mx >> sh, fr = mx & ((1u << sh) - 1u), half = 1u << (sh - 1);
  const bool up = fr > half || (fr == half && (ip & 1u));
  const int32_t a = (int32_t)((bs & 0x7FFFFFu) | 0x800000u);
  if (fr == half && (a & 1)) return false;
  const int32_t dabs = (int32_t)ip + (up ? 1 : 0);
  const bool grow = ((bs ^ bx) >> 31) == 0;
  const int32_t D = grow ? dabs : -dabs;
  int fs = fr == 0 ? 0 : (up ? -1 : 1);
  if (!grow) fs = -fs;
  const int32_t lo = 0x800000, hi = 0x1000000;
  const int32_t a1 = a + D, ak = a + k * D;
  const bool ok1 = fs < 0 ? (a1 <= hi && a1 >= lo + 1) : (a1 < hi && a1 >= lo);
  const bool okk = fs < 0 ? (ak <= hi && ak >= lo + 1) : (ak < hi && ak >= lo);
  if (!ok1 || !okk) return false;
  *out = __builtin_bit_cast(float, (bs & 0xFF800000u) + (uint32_t)(ak - lo));
  return true;
}

// k adds of x from s with the first two done by the fp32 adder itself: a1 =
// s + x, a2 = a1 + x.  When s, a1 and a2 share sign and exponent (one grid,
// ulp u), every later add moves the sum by the same D = bits(a2) - bits(a1)
// ulps: the rounding of a_j + x depends only on x's fraction of an ulp --
// and, for a tie, on the sum's parity, which the first add (made on this
// grid) left even and an even D keeps even -- as long as the sums stay
// strictly inside the binade: bits(a2) + (k - 2) D keeps the sign / exponent
// and a nonzero mantissa (one ulp above the lower edge).  Otherwise the
// remaining adds are plain.  A few integer ops after two adds instead of k
// adds; bit-equal to the loop.  (The device walk, grad_rows.hip
// serial_seg_walk, is this with every value wave-uniform;
// tools/repadd_check.cpp checks it here.)
DR_HD inline bool seg_tail_fits(uint32_t b0, uint32_t b1, uint32_t b2, int32_t k, uint32_t* bk) {
  const int32_t D = (int32_t)(b2 - b1);
  const uint32_t e2 = (b2 >> 23) & 0xFF;
  const uint32_t r = b2 + (uint32_t)(k * D);
  *bk = r;
  return k < 128 && ((b0 ^ b2) >> 23) == 0 && ((b1 ^ b2) >> 23) == 0 && ((b2 ^ r) >> 23) == 0 &&
         (r & 0x7FFFFFu) != 0 && e2 != 0 && e2 != 0xFF;
}
DR_HD inline float seg_walk2(float s, float x, int64_t k) {
  if (k <= 0) return s;
  const float a1 = s + x;
  if (--k == 0) return a1;
  const float a2 = a1 + x;
  --k;
  uint32_t bk;
  if (k == 0) return a2;
  if (seg_tail_fits(f32_bits(s), f32_bits(a1), f32_bits(a2), (int32_t)(k < 128 ? k : 128), &bk))
    return __builtin_bit_cast(float, bk);
  s = a2;
  for (int64_t j = 0; j < k; ++j) s = s + x;
  return s;
}

DR_HD inline float rep_add(float s, float x, int64_t k) {
  float r;
  if (k > 1 && rep_add_grid(s, x, k, &r)) return r;
  const double lo = 8388608.0, hi = 16777216.0;   // a binade in ulps: [2^23, 2^24)
  while (k > 0) {
    const float s1 = s + x;   // one plain add, then the rest in closed form if it may
    const uint32_t b1 = f32_bits(s1);
    const bool fixed = b1 == f32_bits(s);   // s + x rounded back to s: so does every later add
    s = s1;
    if (--k == 0 || fixed) break;
    const int ex = (int)((b1 >> 23) & 0xFF);
    if (ex == 0 || ex == 0xFF) continue;   // zero, subnormal, Inf, NaN: plain adds
    // s1's magnitude in ulps of its binade, x along the magnitude in ulps
    // (both exact in double)
    const double inv_u = ldexp(1.0, 150 - ex);
    const double xu = (b1 >> 31) ? -(double)x * inv_u : (double)x * inv_u;
    const double a1 = lo + (double)(b1 & 0x7FFFFFu);
    const double dd = rint(xu);   // the in-grid step: nearest, ties to even
    // a tie (xu = m + 1/2) adds rint(xu) only from an even sum: from an odd
    // one the first add goes to the other neighbour (then all are even)
    if (xu - floor(xu) == 0.5 && (b1 & 1u)) continue;
    // add j (0-based, from a1) rounds on this grid while a1 + j dd + xu is in
    // [lo, hi): monotone in j
    auto in_grid = [&](int64_t j) {
      const double v = a1 + (double)j * dd + xu;
      return v >= lo && v < hi;
    };
    if (dd == 0) {   // s1 + x rounds back to s1: a fixed point
      if (in_grid(0)) break;
      continue;
    }
    int64_t n = k;
    if (!in_grid(n - 1)) {
      const double lim = dd > 0 ? (hi - a1 - xu) / dd : (a1 + xu - lo) / -dd;
      n = lim > 0 ? (lim < (double)k ? (int64_t)lim : k) : 0;
      while (n > 0 && !in_grid(n - 1)) --n;
      while (n < k && in_grid(n)) ++n;
    }
    if (n == 0) continue;
    const double a = (a1 + (double)n * dd) * ldexp(1.0, ex - 150);   // exact (<= the next power of 2)
    s = (float)((b1 >> 31) ? -a : a);
    k -= n;
  }
  return s;
}

// ---- many segments at once ------------------------------------------------
// A chain of segments (term x_j added k_j times, j ascending) taken in
// parallel: while the running sum stays in one binade of one sign (grid
// fixed), segment j moves it by exactly k_j * D_j ulps (rep_add_grid's step),
// so the sum after any prefix of segments is the start plus an integer
// prefix sum -- the sequential dependence is only through the grid, which
// changes rarely (binade edges, sign changes).  A walker takes a window of
// segments: every segment's step on the current grid (seg_grid_term), an
// exclusive prefix of k_j * D_j, a test that each segment's sums stay on the
// grid from its prefix (seg_grid_fits: both ends inside the binade, no tie
// from an odd sum), and takes the segments before the first that fails in
// one step; the failing one is added by rep_add (exact), and the next round
// starts on its new grid.  Bit-equal to the plain loop (tools/repadd_check.cpp
// "rounds" mode checks it against sum-by-sum adds; rows_rounds_seg_kernel
// runs it on the device).

// The grid of a normal nonzero sum s: its sign / exponent bits and its
// magnitude in ulps a in [2^23, 2^24).
struct SegGrid {
  uint32_t se;   // sign | exponent bits of s (mantissa 0)
  int es;        // exponent field
  bool neg;
};
DR_HD inline bool seg_grid_of(float s, SegGrid* g, int64_t* a) {
  const uint32_t bs = f32_bits(s);
  const int es = (int)((bs >> 23) & 0xFF);
  if (es == 0 || es == 0xFF) return false;
  g->se = bs & 0xFF800000u;
  g->es = es;
  g->neg = (bs >> 31) != 0;
  *a = (int64_t)(bs & 0x7FFFFFu) | 0x800000;
  return true;
}
DR_HD inline float seg_grid_value(const SegGrid& g, int64_t a) {   // a in [2^23, 2^24)
  return __builtin_bit_cast(float, g.se + (uint32_t)(a - 0x800000));
}

// One term on a grid: D = its step in ulps along the magnitude, fs the sign
// of (x in ulps - D) along the magnitude (0: exact), tie: x is an odd
// multiple of half an ulp.  ok = false: not expressible as a grid step
// (x within 2 binades of s, a non-finite or subnormal x) -- a plain add.
struct SegTerm {
  int64_t D;
  int fs;
  bool tie, ok;
};
DR_HD inline SegTerm seg_grid_term(const SegGrid& g, float x) {
  SegTerm r{0, 0, false, true};
  const uint32_t bx = f32_bits(x);
  const int ex = (int)((bx >> 23) & 0xFF);
  if ((bx & 0x7FFFFFFFu) == 0) return r;          // +-0: the sum is unchanged
  if (ex == 0 || ex == 0xFF) {
    r.ok = false;
    return r;
  }
  const int sh = g.es - ex;
  if (sh < 1) {
    r.ok = false;
    return r;
  }
  const bool grow = ((bx >> 31) != 0) == g.neg;   // x along s's sign
  if (sh > 25) {   // |x| < 2^-2 ulps: every add rounds back to s (never a tie)
    r.fs = grow ? 1 : -1;
    return r;
  }
  const int64_t mx = (int64_t)((bx & 0x7FFFFFu) | 0x800000u);
  const int64_t ip = mx >> sh, fr = mx & (((int64_t)1 << sh) - 1), half = (int64_t)1 << (sh - 1);
  const bool up = fr > half || (fr == half && (ip & 1));
  r.tie = fr == half;
  const int64_t dabs = ip + (up ? 1 : 0);
  r.D = grow ? dabs : -dabs;
  int fs = fr == 0 ? 0 : (up ? -1 : 1);
  r.fs = grow ? fs : -fs;
  return r;
}

// k adds of the term from a (the running sum in ulps) all round on the grid
DR_HD inline bool seg_grid_fits(int64_t a, int64_t k, const SegTerm& t) {
  if (!t.ok || (t.tie && (a & 1))) return false;
  const int64_t lo = 0x800000, hi = 0x1000000;
  const int64_t a1 = a + t.D, ak = a + k * t.D;
  auto in_grid = [&](int64_t ap) {
    const bool below_hi = t.fs < 0 ? ap <= hi : ap < hi;
    const bool above_lo = t.fs < 0 ? ap >= lo + 1 : ap >= lo;
    return below_hi && above_lo;
  };
  return in_grid(a1) && in_grid(ak);
}

}  // namespace dr
