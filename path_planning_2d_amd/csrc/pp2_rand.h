// pp2_rand.h -- host random streams the reference draws from (private).
#pragma once
#include <stdint.h>

namespace pp2rt {

// glibc random_r, TYPE_3 (x**31 + x**3 + 1), as srand(seed) / rand().  The
// reference never seeds rand(), so its stream is seed 1; PBVI's belief-set
// expansion and the QV-tree's state samples draw from the same stream.
struct GlibcRand {
  int32_t r[31];
  int f = 3, b = 0;
  uint64_t calls = 0;
  void seed(uint32_t s) {
    int64_t word = (int32_t)(s == 0 ? 1 : s);
    r[0] = (int32_t)word;
    for (int i = 1; i < 31; ++i) {
      const int64_t hi = word / 127773, lo = word % 127773;
      word = 16807 * lo - 2836 * hi;
      if (word < 0) word += 2147483647;
      r[i] = (int32_t)word;
    }
    f = 3;
    b = 0;
    for (int i = 0; i < 310; ++i) (void)next();
    calls = 0;
  }
  int32_t next() {
    const uint32_t val = (uint32_t)r[f] + (uint32_t)r[b];
    r[f] = (int32_t)val;
    if (++f >= 31) {
      f = 0;
      ++b;
    } else if (++b >= 31) {
      b = 0;
    }
    ++calls;
    return (int32_t)(val >> 1);
  }
  // (float)rand() / ((float)RAND_MAX + 1.0f)
  float unit() { return (float)next() / ((float)2147483647 + 1.0f); }
};

}  // namespace pp2rt
