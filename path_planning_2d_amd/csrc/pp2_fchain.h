// pp2_fchain.h -- exact parallel evaluation of a sequential fp32 sum.
//
// The reference runs every grid-wide sum of its QV-tree on the x86 host as
// one left-to-right fp32 chain, acc = fl(acc + t_x) for x = 0 .. n-1, IEEE
// round-to-nearest-even, no FMA contraction:
//   * std::accumulate of a child belief (search_tree_cuda.cu:225-229),
//   * std::inner_product for the QNode reward (:168-173), evaluateFibCpu
//     (fast_informed_bound_cuda.cu:278-297), evaluatePbviCpu
//     (point_based_value_iteration_cuda.cu:678-699): t_x = fl(b_x * a_x),
//   * the sampling cdf of forwardSampling (search_tree_cuda.cu:176-183).
// A chain of n dependent adds costs n add latencies on any core (~0.25 ms at
// 256^2 on one gfx950 lane).  The result is nevertheless computable in
// parallel, bit for bit, when every term has the same sign (beliefs >= 0;
// rewards and FIB / PBVI values <= 0 -- the sign is checked per chain, mixed
// chains run sequentially):
//
// * Work on |t|; the running sum s is then non-decreasing.  Write s = k * u
//   with u = 2^(E-23) the ulp of its binade [2^E, 2^(E+1)) (E >= -126; the
//   subnormals and [2^-126, 2^-125) share u = 2^-149, so s = 0 is E = -126,
//   k = 0).  While s + t stays below 2^(E+1), fl(s + t) = u * RNE(k + t/u),
//   and t/u = ldexp(t, 23 - E) is exact.  Unless t/u sits exactly halfway
//   between integers (a tie, resolved by the parity of k), that is
//   k + rint(t/u): the increment does not depend on k at all.
// * So a chunk of terms whose sum stays inside binade E and holds no tie
//   advances k by d = sum of rint(t/u) over the chunk -- an integer sum whose
//   order does not matter.  Since k only grows, the chunk stayed inside the
//   binade iff k + d <= 2^24 (k == 2^24 is 2^(E+1), the next binade's first
//   value; a later term that rounds to 0 at ulp u rounds to 0 at 2u too).
// * A driver walks the chunks in x order with the exact state (E, k): a
//   chunk whose table entry was computed for the state's E and holds no tie
//   advances k by d; any other chunk (the binade crossings, a table computed
//   for a neighbouring E, a tie) is added term by term in fp32, exactly as
//   the reference, and the state re-derived from the float.
// The table entry's E comes from an approximate running sum (any value:
// the driver only checks it), so the result equals the sequential chain for
// every input; only the speed depends on how many chunks fall back.
//
// Device code includes this after defining PP2_FC_HD (__host__ __device__);
// the CPU check (tools/fchain_check.cpp) includes it as plain C++.
#pragma once

#include <math.h>
#include <stdint.h>

#ifndef PP2_FC_HD
#define PP2_FC_HD
#endif

namespace pp2 {
namespace fchain {

constexpr int kK24 = 1 << 24;
constexpr int kEMin = -126;
constexpr uint32_t kNoEntry = 0xffffffffu;  // table entry that never applies
constexpr float kQCap = 67108864.0f;        // 2^26: t/u beyond it cannot be valid

PP2_FC_HD inline uint32_t bits_of(float f) { return __builtin_bit_cast(uint32_t, f); }
PP2_FC_HD inline float float_of(uint32_t u) { return __builtin_bit_cast(float, u); }

// Binade domain E of a finite s >= +0 (sign ignored): max(exponent, -126).
PP2_FC_HD inline int domain_of(float s) {
  const int et = (int)((bits_of(s) >> 23) & 0xffu);
  return et <= 1 ? kEMin : et - 127;
}

// (E, k) of a finite s >= +0.  With the float's bits b (sign cleared) and
// exponent field et, E = max(et, 1) - 127 and k = b - ((E + 126) << 23): the
// significand with its hidden bit, or for subnormals the bits themselves --
// branch-free (a walker runs this on the scalar unit, where every branch is
// a pipeline refill).
PP2_FC_HD inline void state_of(float s, int* E, int* k) {
  const uint32_t b = bits_of(s) & 0x7fffffffu;
  const int et = (int)(b >> 23);
  const int e1 = et > 1 ? et : 1;
  *E = e1 - 127;
  *k = (int)(b - ((uint32_t)(e1 - 1) << 23));
}

// k == 2^24 is the next binade's first value.
PP2_FC_HD inline void normalise(int* E, int* k) {
  if (*k == kK24) {
    *E += 1;
    *k = 1 << 23;
  }
}

// The float k * 2^(E-23) (k <= 2^24; E = -126: any k, else k >= 2^23): the
// inverse of state_of, bits ((E + 126) << 23) + k -- k = 2^24 carries into the
// next binade's first value, and past E = 127 into +inf (clamped there: an
// overflowed sum stays +inf whatever it adds).
PP2_FC_HD inline float value_of(int E, int k) {
  const uint32_t b = ((uint32_t)(E + 126) << 23) + (uint32_t)k;
  return float_of(b < 0x7f800000u ? b : 0x7f800000u);
}

// The increment of one term a = |t| (finite) in domain E: rint(a / u) as a
// float (exact integer < 2^26, or 2^26 when larger), and whether it is a tie.
PP2_FC_HD inline float units_of(float a, int E, bool* tie) {
  float q = ldexpf(a, 23 - E);
  q = fminf(q, kQCap);
  const float r = rintf(q);
  *tie = fabsf(q - r) == 0.5f;
  return r;
}

// A tie, t/u = m + 1/2, rounds to the even one of k + m and k + m + 1: its
// increment is m + ((k + m) & 1) -- it depends on k only through k's parity,
// and leaves k even.  (m = q - 1/2, exact: q is a half-integer below 2^26.)
PP2_FC_HD inline int tie_increment(float q, int k) {
  const int m = (int)(q - 0.5f);
  return m + ((k + m) & 1);
}

// One term a = |t| (finite) added to the state exactly: its increment (a
// tie's by the parity of k) when that applies (the sum stays within
// 2^(E+1)), else the fp32 add itself.  (k == 2^24 is left as is: a later
// increment of 0 keeps it, any other goes through the fp32 add from
// value_of, which carries.)  A wave applies this to a chunk's terms in
// parallel: the increments' prefix sum up to the first term that does not
// apply, that term's fp32 add, and again (chunk_exact).
PP2_FC_HD inline void add_exact(int* E, int* k, float a) {
  bool tie;
  const float r = units_of(a, *E, &tie);
  const int inc = tie ? tie_increment(ldexpf(a, 23 - *E), *k) : (int)r;
  if (*k + inc <= kK24) {
    *k += inc;
  } else {
    const float s = value_of(*E, *k) + a;
    state_of(s, E, k);
  }
}

// Table entry of a chunk: d units in domain E, or kNoEntry.
PP2_FC_HD inline uint32_t make_entry(int E, float d, bool tie) {
  if (tie || !(d < (float)kK24)) return kNoEntry;
  return ((uint32_t)(E + 128) << 24) | (uint32_t)d;
}
PP2_FC_HD inline int entry_domain(uint32_t e) { return (int)(e >> 24) - 128; }
PP2_FC_HD inline int entry_units(uint32_t e) { return (int)(e & 0xffffffu); }
// Whether an entry applies in the state's domain E: it was computed for E --
// or it adds nothing (d = 0 with no tie: every |t| / u below 1/2) and was
// computed for a lower domain, where at E each ratio is 2^(E_e - E) times
// smaller, still below 1/2.  (The tail of a concentrated belief: once the
// exact sum sits at 1.0 and the approximate one just below, every later chunk
// was tabled for the binade below.)
PP2_FC_HD inline bool entry_applies(uint32_t e, int E) {
  return e != kNoEntry &&
         (entry_domain(e) == E || (entry_units(e) == 0 && entry_domain(e) < E));
}

}  // namespace fchain
}  // namespace pp2
