// Bit-for-bit check of device.h's in-range sqrt / reciprocal sequences against the compiler's
// IEEE sqrt() and 1.0 / s on the GPU (the oracle computes sqrt and / in C, IEEE as well).
// Sampled, not exhaustive: x sweeps the fast range [2^-700, 2^700] (uniform exponent, random
// mantissa) plus dense samples in [0.5, 8), and a directed set of the cases random sampling
// almost never hits (the kernel `directed`): exact squares k^2 scaled by powers of 4, every
// power of two in the range, the bounds 2^-700 / 2^700 and their neighbours, and the
// neighbourhoods (+-8 ulps of x) of the squares of g with an all-ones / near-all-ones or
// near-1 significand and of rounding midpoints (g + half an ulp) -- where the final
// corrections fma(d, h, g) / fma(e, q, q) from a one-ulp estimate could round wrongly.  Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
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

// directed case i -> x (0 when the case is out of the fast range or unused)
__device__ double directed_x(int64_t i) {
  const int64_t fam = i % 8, k = i / 8;
  const int nb = (int)(k % 17) - 8;          // neighbour offset in ulps of x
  const int64_t q = k / 17;
  double x = 0.0;
  if (fam == 0) {                             // exact squares k^2 * 4^e
    const double r = (double)(q % (1 << 26) + 1);
    x = ldexp(r * r, 2 * (int)((q >> 26) % 700) - 700);
    return x;                                  // no neighbours: the exact case itself
  } else if (fam == 1) {                       // powers of two and the range bounds
    x = ldexp(1.0, (int)(q % 1401) - 700);
  } else if (fam == 2 || fam == 3) {           // g with an all-ones / near-all-ones significand
    const double g = ldexp(2.0 - ldexp((double)(q % 64 + 1), -52), (int)((q / 64) % 700) - 350);
    x = g * g;
  } else if (fam == 4) {                       // g just above a power of two
    const double g = ldexp(1.0 + ldexp((double)(q % 64 + 1), -52), (int)((q / 64) % 700) - 350);
    x = g * g;
  } else {                                     // sqrt(x) at a rounding midpoint: x = RN(g (g + ulp))
    uint64_t z = (uint64_t)q * 0x9E3779B97F4A7C15ull + (uint64_t)fam;
    z = (z ^ (z >> 29)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 32;
    const uint64_t gb = 0x3FF0000000000000ull | (z & 0xFFFFFFFFFFFFFull);
    const double g = ldexp(__builtin_bit_cast(double, gb), (int)((q >> 3) % 700) - 350);
    const double gn = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, g) + 1);
    x = g * gn;
  }
  uint64_t u = __builtin_bit_cast(uint64_t, x);
  u = (uint64_t)((int64_t)u + nb);
  return __builtin_bit_cast(double, u);
}

// candidate: the Goldschmidt sequence with two Newton steps on q before the final correction
__device__ __forceinline__ void sqrt_rcp_2n(double x, double* s, double* rcp) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  g = fma(d, h, g);
  double q = h + h;
  double e = fma(-g, q, 1.0);
  q = fma(q, e, q);
  e = fma(-g, q, 1.0);
  q = fma(q, e, q);
  e = fma(-g, q, 1.0);
  *rcp = fma(e, q, q);
  *s = g;
}

// bad[fam * 4 + {sqrt, rcp, old sqrt, old rcp}], bad[32 + fam] = cases used, bad[40 + fam] = 2-Newton rcp
__global__ void directed(int64_t n, unsigned long long* bad) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double x = directed_x(i);
    if (!(x > 0.0) || !mmb_fast_range(x)) continue;
    const int fam = (int)(i % 8);
    const double s_ref = sqrt(x), r_ref = 1.0 / s_ref;
    double s, r;
    mmb_sqrt_rcp_inrange(x, &s, &r);
    const double s_old = mmb_sqrt_inrange(x), r_old = mmb_rcp_inrange(s_old);
    if (s != s_ref) atomicAdd(bad + fam * 4, 1ull);
    if (r != r_ref) atomicAdd(bad + fam * 4 + 1, 1ull);
    if (s_old != s_ref) atomicAdd(bad + fam * 4 + 2, 1ull);
    if (r_old != r_ref) atomicAdd(bad + fam * 4 + 3, 1ull);
    double s2, r2;
    sqrt_rcp_2n(x, &s2, &r2);
    if (r2 != r_ref || s2 != s_ref) atomicAdd(bad + 40 + fam, 1ull);
    if ((i & 1023) < 8) atomicAdd(bad + 32 + fam, 1ull);   // 1/128 of the cases counted
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (int64_t)1 << 32;
  unsigned long long* bad;
  if (hipMalloc(&bad, 4 * sizeof(unsigned long long)) != hipSuccess) return 2;
  hipMemset(bad, 0, 4 * sizeof(unsigned long long));
  check<<<4096, 256>>>(12345, n, bad);
  unsigned long long h[4];
  if (hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  unsigned long long* dbad;
  if (hipMalloc(&dbad, 48 * sizeof(unsigned long long)) != hipSuccess) return 2;
  hipMemset(dbad, 0, 48 * sizeof(unsigned long long));
  const int64_t nd = (int64_t)1 << 31;
  directed<<<4096, 256>>>(nd, dbad);
  unsigned long long hd[48];
  if (hipMemcpy(hd, dbad, sizeof hd, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  unsigned long long dsum[4] = {0, 0, 0, 0};
  for (int f = 0; f < 8; ++f) for (int k = 0; k < 4; ++k) dsum[k] += hd[f * 4 + k];
  printf("{\"samples\": %lld, \"sqrt_mismatch\": %llu, \"rcp_mismatch\": %llu, "
         "\"old_sqrt_mismatch\": %llu, \"old_rcp_mismatch\": %llu, \"directed_cases\": %lld, "
         "\"directed_sqrt_mismatch\": %llu, \"directed_rcp_mismatch\": %llu, "
         "\"directed_old_sqrt_mismatch\": %llu, \"directed_old_rcp_mismatch\": %llu, \"by_family\": [",
         (long long)n, h[0], h[1], h[2], h[3], (long long)nd, dsum[0], dsum[1], dsum[2], dsum[3]);
  for (int f = 0; f < 8; ++f)
    printf("%s[%llu, %llu, %llu, %llu, %llu, %llu]", f ? ", " : "", hd[32 + f] * 128, hd[f * 4], hd[f * 4 + 1],
           hd[f * 4 + 2], hd[f * 4 + 3], hd[40 + f]);
  printf("]}\n");
  return (h[0] || h[1] || dsum[0] || dsum[1]) ? 1 : 0;
}
