// summary.hip — on-device posterior summaries of the device-kept draws.
//
// summarystats(c; etype=:bm) (src/output/stats.jl:85-94) pools each monitored param over
// all chains: Mean, SD, Naive SE = sem, MCSE = mcse_bm(vec(x), size=100)
// (src/output/mcse.jl:10-19) and ESS = min((SD/MCSE)^2, n).  vec(x) concatenates the chains
// (global chain order), so a batch of `bs` consecutive elements may straddle chains.
//
// ss_chain_kernel: one thread per (chain, param) streams that chain's n kept draws
// (draws[(i*P + j)*K + k]: adjacent threads = adjacent chains, coalesced) and emits
//   [s1, q, B1, B2, nfull, hsum, hcnt, tsum, tcnt, 0]
// with x' = x - shift[j]: s1 = sum x', q = sum x'^2, and for the batches of vec(x) that lie
// wholly inside the chain (global id kg occupies flat positions kg*n .. kg*n+n-1)
// B1 = sum d_b, B2 = sum d_b^2, d_b = (sum over batch of x') / bs = mbar_b - shift; the
// partial batch at the chain's start (head) and end (tail) are returned as raw sums and
// counts and are joined across chains (and GPUs) by the host (mamba.jl_amd/summary.py).
//
// os_hist_kernel: quantile(c) (stats.jl:73-80) needs exact order statistics of the
// pooled draws of one param.  Radix select over the order-preserving 64-bit key of a
// double, 8 bits per pass from the top: for each requested target (its key prefix so far)
// the kernel histograms the next digit of the matching elements in LDS, flushed with
// 64-bit atomics.  The host picks the bin holding the target rank (after an all-reduce of
// the counts across GPUs) and descends; 8 passes give the exact element.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SS_THREADS 256
#define SS_FIELDS 10
#define OS_THREADS 256
#define OS_MAXT 16

__global__ __launch_bounds__(SS_THREADS) void ss_chain_kernel(int P, int64_t n, int K, int64_t kg0, int64_t bs,
                                                               const double* __restrict__ draws,
                                                               const double* __restrict__ shift,
                                                               double* __restrict__ out) {
  const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int j = (int)blockIdx.y;
  if (k >= K) return;
  const double sh = shift[j];
  const int64_t t0 = (kg0 + k) * n;          // flat position of this chain's first draw in vec(x)
  int64_t rem = bs - t0 % bs;                // elements until the current batch closes
  const bool starts_inside = (t0 % bs) == 0; // the first batch begins at this chain's first draw
  bool inside = starts_inside;
  double s1 = 0.0, q = 0.0, b1 = 0.0, b2 = 0.0, acc = 0.0, nfull = 0.0, hsum = 0.0, hcnt = 0.0;
  int64_t cnt = 0;
  const double inv = 1.0 / (double)bs;
  const double* p = draws + (size_t)j * K + k;
  const size_t stride = (size_t)P * K;
  // SS_U independent loads in flight per thread (the chain's draws are a strided stream),
  // then the sequential batch bookkeeping on registers
  constexpr int SS_U = 16;
  for (int64_t i0 = 0; i0 < n; i0 += SS_U) {
    double xs[SS_U];
#pragma unroll
    for (int u = 0; u < SS_U; ++u) xs[u] = i0 + u < n ? p[(size_t)(i0 + u) * stride] : 0.0;
#pragma unroll
    for (int u = 0; u < SS_U; ++u) {
      if (i0 + u < n) {
        const double x = xs[u] - sh;
        s1 += x;
        q = fma(x, x, q);
        acc += x;
        ++cnt;
        if (--rem == 0) {                    // batch closes at this element
          if (inside) {
            const double d = acc * inv;
            b1 += d;
            b2 = fma(d, d, b2);
            nfull += 1.0;
          } else {                           // it began in an earlier chain: head piece
            hsum = acc;
            hcnt = (double)cnt;
          }
          inside = true;
          acc = 0.0;
          cnt = 0;
          rem = bs;
        }
      }
    }
  }
  double tsum = 0.0, tcnt = 0.0;
  if (cnt > 0) {
    if (inside) { tsum = acc; tcnt = (double)cnt; }   // continues into the next chain
    else { hsum = acc; hcnt = (double)cnt; }          // the whole chain sits inside one batch
  }
  double* o = out + ((size_t)k * P + j) * SS_FIELDS;
  o[0] = s1; o[1] = q; o[2] = b1; o[3] = b2; o[4] = nfull;
  o[5] = hsum; o[6] = hcnt; o[7] = tsum; o[8] = tcnt; o[9] = 0.0;
}

// order-preserving key: negative doubles reversed, positive ones above them
__device__ __forceinline__ uint64_t os_key(double x) {
  const uint64_t u = (uint64_t)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__global__ __launch_bounds__(OS_THREADS) void os_hist_kernel(int P, int j, int64_t n, int K,
                                                              const double* __restrict__ draws, int nt,
                                                              const uint64_t* __restrict__ prefix, int pass,
                                                              unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[OS_MAXT][256];
  for (int q = threadIdx.x; q < nt * 256; q += blockDim.x) h[q >> 8][q & 255] = 0u;
  __syncthreads();
  const int dsh = 56 - 8 * pass;             // this pass's digit: bits dsh .. dsh+7
  uint64_t pre[OS_MAXT];
#pragma unroll
  for (int t = 0; t < OS_MAXT; ++t) pre[t] = t < nt ? prefix[t] : 0ull;
  const size_t stride = (size_t)P * K;
  for (int64_t i = blockIdx.y; i < n; i += gridDim.y) {
    const double* row = draws + (size_t)i * stride + (size_t)j * K;
    for (int k = (int)(blockIdx.x * blockDim.x + threadIdx.x); k < K; k += gridDim.x * blockDim.x) {
      const uint64_t key = os_key(row[k]);
      const unsigned dg = (unsigned)(key >> dsh) & 255u;
      const uint64_t hi = pass == 0 ? 0ull : key >> (dsh + 8);
#pragma unroll
      for (int t = 0; t < OS_MAXT; ++t)
        if (t < nt && hi == pre[t]) atomicAdd(&h[t][dg], 1u);
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < nt * 256; q += blockDim.x) {
    const unsigned v = h[q >> 8][q & 255];
    if (v) atomicAdd(&counts[q], (unsigned long long)v);
  }
}

hipError_t mmb_launch_chain_summary(int P, int64_t n, int K, int64_t kg0, int64_t bs, const double* draws,
                                    const double* shift, double* out, hipStream_t st) {
  const dim3 grid((K + SS_THREADS - 1) / SS_THREADS, P), blk(SS_THREADS);
  hipLaunchKernelGGL(ss_chain_kernel, grid, blk, 0, st, P, n, K, kg0, bs, draws, shift, out);
  return hipGetLastError();
}

// prefix[t] = the key bits above this pass's digit (key >> (56 - 8*pass + 8)); nt <= 16
hipError_t mmb_launch_order_hist(int P, int j, int64_t n, int K, const double* draws, int nt,
                                 const uint64_t* prefix, int pass, unsigned long long* counts, hipStream_t st) {
  if (nt < 1 || nt > OS_MAXT || pass < 0 || pass > 7) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(counts, 0, (size_t)nt * 256 * sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  // ~1024 workgroups (4 per CU), each striding over many rows: the per-workgroup LDS
  // clear and atomic flush of nt x 256 bins stays small against its share of the n*K draws
  int gx = (K + OS_THREADS - 1) / OS_THREADS;
  if (gx > 64) gx = 64;
  int64_t gy = 1024 / gx;
  if (gy > n) gy = n;
  if (gy < 1) gy = 1;
  hipLaunchKernelGGL(os_hist_kernel, dim3(gx, (unsigned)gy), dim3(OS_THREADS), 0, st, P, j, n, K, draws, nt,
                     prefix, pass, counts);
  return hipGetLastError();
}
