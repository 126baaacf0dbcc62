// Bit-for-bit check of device.h's in-range sqrt / reciprocal sequences against the compiler's
// IEEE sqrt() and 1.0 / s on the GPU (the oracle computes sqrt and / in C, IEEE as well).
// x sweeps the fast range [2^-700, 2^700] (uniform exponent, random mantissa) plus dense
// samples in [0.5, 8).  Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
//   -I include tools/sqrt_rcp_check.hip -o tools/sqrt_rcp_check ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../mamba.jl_amd/csrc/device.h"

__global__ void check(uint64_t seed, int64_t n, unsigned long long* bad) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long b[4] = {0, 0, 0, 0};
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const uint64_t mant = z & 0xFFFFFFFFFFFFFull;
    const int ex = (i & 1) ? (int)((z >> 52) % 1400u) - 700 : (int)((z >> 52) & 3u) - 1;
    const double x = ldexp(__builtin_bit_cast(double, (uint64_t)0x3FF0000000000000ull | mant), ex);
    if (!mmb_fast_range(x)) continue;
    const double s_ref = sqrt(x), r_ref = 1.0 / s_ref;
    double s, r;
    mmb_sqrt_rcp_inrange(x, &s, &r);
    const double s_old = mmb_sqrt_inrange(x), r_old = mmb_rcp_inrange(s_old);
    b[0] += s != s_ref;
    b[1] += r != r_ref;
    b[2] += s_old != s_ref;
    b[3] += r_old != r_ref;
  }
  for (int k = 0; k < 4; ++k) if (b[k]) atomicAdd(bad + k, b[k]);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (int64_t)1 << 32;
  unsigned long long* bad;
  if (hipMalloc(&bad, 4 * sizeof(unsigned long long)) != hipSuccess) return 2;
  hipMemset(bad, 0, 4 * sizeof(unsigned long long));
  check<<<4096, 256>>>(12345, n, bad);
  unsigned long long h[4];
  if (hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("{\"samples\": %lld, \"sqrt_mismatch\": %llu, \"rcp_mismatch\": %llu, "
         "\"old_sqrt_mismatch\": %llu, \"old_rcp_mismatch\": %llu}\n", (long long)n, h[0], h[1], h[2], h[3]);
  return (h[0] || h[1]) ? 1 : 0;
}
