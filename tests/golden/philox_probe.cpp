// Host-side probe: Philox4x32-10 outputs from rocRAND's header-only engine
// (/opt/rocm/include/rocrand/rocrand_philox4x32_10.h), used to pin the build's own
// Philox (mmb_math.h).  Built and run by tests/golden/make_golden.py; output committed
// as tests/golden/philox_kat.json.  Not shipped.
#include <rocrand/rocrand_philox4x32_10.h>
#include <cstdio>
struct probe : rocrand_device::philox4x32_10_engine {
  probe() : rocrand_device::philox4x32_10_engine(0, 0, 0) {}
  uint4 rounds(uint4 c, uint2 k) { return ten_rounds(c, k); }
};
int main() {
  const unsigned int cases[][6] = {
      {0u, 0u, 0u, 0u, 0u, 0u},
      {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu},
      {0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u, 0xa4093822u, 0x299f31d0u},
      {7u, 16u + 1u, 1234u, 4095u, 0x9e3779b9u, 0x00000001u},
      {3u, 33u, 10000u, 131071u, 123u, 0u},
  };
  probe eng;
  std::printf("[");
  for (int i = 0; i < 5; ++i) {
    const unsigned int* c = cases[i];
    uint4 ctr{c[0], c[1], c[2], c[3]};
    uint2 key{c[4], c[5]};
    uint4 r = eng.rounds(ctr, key);
    std::printf("%s{\"ctr\":[%u,%u,%u,%u],\"key\":[%u,%u],\"out\":[%u,%u,%u,%u]}", i ? "," : "",
                c[0], c[1], c[2], c[3], c[4], c[5], r.x, r.y, r.z, r.w);
  }
  std::printf("]\n");
  return 0;
}
