// Host build of csrc/np_sum.h (tests/test_np_sum.py): reads "d" then d*d float64 values (float32
// representable) per case from stdin, prints np_abs_sum32 as a float's bit pattern.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../midagma_amd/csrc/np_sum.h"

int main() {
  long long d;
  while (std::scanf("%lld", &d) == 1) {
    std::vector<double> W((size_t)(d * d));
    for (auto& x : W)
      if (std::scanf("%lf", &x) != 1) return 2;
    const float s = midagma::np_abs_sum32(W.data(), d, d);
    uint32_t b;
    std::memcpy(&b, &s, 4);
    std::printf("%u\n", b);
  }
  return 0;
}
