// Host-side checks of the integer index math the HIP kernels rely on, built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host pass only
// (tests/test_native_host.py: hipcc -Xarch_host -fsanitize=...).  GPU sanitizers are not
// available on this pool; these helpers are __host__ __device__, so the host build checks
// the very code the kernels run.
//   * FastDiv (csrc/common.h): fdiv(n, d) == n / d for every divisor the kernels build one
//     for (1 .. 65536 densely, larger ones sampled) over n in [0, 2^31)
//   * xcd_remap: a bijection of [0, nwg) for every grid size up to 70000
//   * reflect_idx: PyTorch ReflectionPad semantics for pad < n
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"

using namespace p2p;

static int fails = 0;
#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      if (fails++ < 20) {             \
        std::printf(__VA_ARGS__);     \
        std::printf("\n");            \
      }                               \
    }                                 \
  } while (0)

static uint32_t lcg(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(s >> 33);
}

int main() {
  // FastDiv
  uint64_t seed = 12345;
  for (uint32_t d = 1; d <= 65536 || d < (1u << 30); d = d <= 65536 ? d + 1 : d * 3 + 7) {
    const FastDiv f = make_fastdiv(d);
    const uint32_t edge[] = {0u, 1u, d - 1, d, d + 1, 2 * d - 1, 2 * d, 0x7fffffffu, 0x7ffffffeu,
                             (0x7fffffffu / d) * d, (0x7fffffffu / d) * d - 1};
    for (uint32_t n : edge) {
      if (n > 0x7fffffffu) continue;
      CHECK(fdiv(n, f) == n / d, "fdiv(%u, %u) = %u, want %u", n, d, fdiv(n, f), n / d);
    }
    const int samples = d <= 4096 ? 64 : 8;
    for (int i = 0; i < samples; ++i) {
      const uint32_t n = lcg(seed) & 0x7fffffffu;
      CHECK(fdiv(n, f) == n / d, "fdiv(%u, %u) = %u, want %u", n, d, fdiv(n, f), n / d);
    }
  }
  // xcd_remap bijectivity
  for (int nwg = 1; nwg <= 70000; nwg = nwg < 4096 ? nwg + 1 : nwg + 997) {
    std::vector<char> seen(nwg, 0);
    for (int b = 0; b < nwg; ++b) {
      const int r = xcd_remap(b, nwg);
      CHECK(r >= 0 && r < nwg, "xcd_remap(%d, %d) = %d out of range", b, nwg, r);
      if (r >= 0 && r < nwg) {
        CHECK(!seen[r], "xcd_remap not injective: nwg %d hits %d twice", nwg, r);
        seen[r] = 1;
      }
    }
  }
  // reflect_idx == PyTorch reflection for -n < i < 2n - 1
  for (int n = 2; n <= 300; ++n)
    for (int i = -(n - 1); i < 2 * n - 1; ++i) {
      int want = i < 0 ? -i : (i >= n ? 2 * (n - 1) - i : i);
      CHECK(reflect_idx(i, n) == want && want >= 0 && want < n, "reflect_idx(%d, %d) = %d", i, n,
            reflect_idx(i, n));
    }
  std::printf("host_checks: %s (%d failures)\n", fails ? "FAIL" : "PASS", fails);
  return fails ? 1 : 0;
}
