// nlp/random.hxx -- the reference's random draws, restated with the engine's
// state exposed (parity at the RNG boundary).
//
// main.cxx:194-195 draws every deletion batch from one std::default_random_engine
// (libstdc++: minstd_rand0, x <- 16807 x mod 2^31 - 1) through
// uniform_real_distribution<double>(0, 1), i.e. generate_canonical<double, 53>:
// two engine calls per double (k = max(1, (53 + 30 - 1) / 30) with
// log2(2^31 - 2) truncated to 30), sum = (g1 - 1) + (g2 - 1) R in double,
// R = 2^31 - 2, divided by double(R^2) (the running product kept as double,
// multiplied in long double), 1 mapped to nextafter(1, 0).  Same arithmetic,
// same values, without libstdc++'s per-call long double logarithms; the engine
// state can be carried from one batch to the next (main.cxx keeps one engine).
#pragma once
#include <cmath>
#include <cstdint>

namespace nlp {

/** std::minstd_rand0 with its state readable: Minstd0(seed) == minstd_rand0(seed). */
struct Minstd0 {
  using result_type = uint32_t;
  uint32_t x;
  explicit Minstd0(uint64_t seed = 1) {
    x = uint32_t(seed % 2147483647u);
    if (x == 0) x = 1;
  }
  static constexpr uint32_t min() { return 1u; }
  static constexpr uint32_t max() { return 2147483646u; }
  uint32_t operator()() {
    x = uint32_t((uint64_t)x * 16807u % 2147483647u);
    return x;
  }
};

/** uniform_real_distribution<double>(0.0, 1.0)(g) for g a minstd_rand0. */
inline double canonical01(Minstd0& g) {
  const long double r = 2147483646.0L;
  double sum = 0.0, tmp = 1.0;
  for (int k = 0; k < 2; ++k) {
    sum += double(g() - 1u) * tmp;
    tmp = double((long double)tmp * r);
  }
  double ret = sum / tmp;
  if (ret >= 1.0) ret = std::nextafter(1.0, 0.0);
  return ret * (1.0 - 0.0) + 0.0;
}

}  // namespace nlp
