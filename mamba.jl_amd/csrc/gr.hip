// gr.hip — on-device Gelman-Rubin sufficient statistics (src/output/gelmandiag.jl:3-60).
//
// gelmandiag needs per chain k the mean psibar_k and covariance S2_k of its n kept
// draws (after link(), chains.jl:237-246), and then only sums over chains.  Each
// thread owns one chain (draws are [n][p][K], chain fastest: coalesced), does a
// two-pass mean/covariance, and the block reduces the per-chain terms in LDS.  The
// per-block partials are summed on the host in block order (deterministic); across
// GPUs the L-vector is all-reduced (RCCL) before the host applies the PSRF formula.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mmb_math.h"

#define GR_PMAX 4
#define GR_THREADS 256

__device__ __forceinline__ double gr_link(int kind, double x) {
  if (kind == 1) return mmb_log(x);
  if (kind == 2) return mmb_log(x / (1.0 - x));  // Mamba logit (utils.jl:67)
  return x;
}

template <int P>
__global__ __launch_bounds__(GR_THREADS) void gr_stats_kernel(int64_t n, int K, const double* __restrict__ draws,
                                                              const int32_t* __restrict__ link,
                                                              const double* __restrict__ shift,
                                                              double* __restrict__ partial) {
  constexpr int L = 1 + P + P * P + P * P + 3 * P;
  __shared__ double red[GR_THREADS];
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  double t[L];
#pragma unroll
  for (int i = 0; i < L; ++i) t[i] = 0.0;
  if (k < K) {
    double mean[P], c[P][P];
#pragma unroll
    for (int j = 0; j < P; ++j) mean[j] = 0.0;
    for (int64_t i = 0; i < n; ++i)
#pragma unroll
      for (int j = 0; j < P; ++j) mean[j] += gr_link(link[j], draws[(size_t)(i * P + j) * K + k]);
#pragma unroll
    for (int j = 0; j < P; ++j) mean[j] = mean[j] / (double)n;
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int l = 0; l < P; ++l) c[j][l] = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      double dv[P];
#pragma unroll
      for (int j = 0; j < P; ++j) dv[j] = gr_link(link[j], draws[(size_t)(i * P + j) * K + k]) - mean[j];
#pragma unroll
      for (int j = 0; j < P; ++j)
#pragma unroll
        for (int l = 0; l < P; ++l) c[j][l] = fma(dv[j], dv[l], c[j][l]);
    }
    const double den = 1.0 / (double)(n - 1);
    double phi[P];
#pragma unroll
    for (int j = 0; j < P; ++j) phi[j] = mean[j] - shift[j];
    int o = 0;
    t[o++] = 1.0;
#pragma unroll
    for (int j = 0; j < P; ++j) t[o++] = phi[j];
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int l = 0; l < P; ++l) t[o++] = phi[j] * phi[l];
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int l = 0; l < P; ++l) t[o++] = c[j][l] * den;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      double s2 = c[j][j] * den;
      t[o + j] = s2 * s2;
      t[o + P + j] = s2 * phi[j];
      t[o + 2 * P + j] = s2 * phi[j] * phi[j];
    }
  }
#pragma unroll
  for (int i = 0; i < L; ++i) {
    red[threadIdx.x] = t[i];
    __syncthreads();
    for (int s = GR_THREADS / 2; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) partial[(size_t)blockIdx.x * L + i] = red[0];
    __syncthreads();
  }
}

// Many monitored values (p > GR_PMAX, e.g. logistic p = 50): one workgroup per chunk of
// chains, one chain at a time; means by thread-per-parameter, the p x p covariance by
// thread-owned (j, l) pairs over draws staged in LDS tiles of GR_TI iterations.  The
// workgroup accumulates the L-vector in LDS and writes one partial per workgroup.
#define GR_BIG_PMAX 64
#define GR_TI 32
#define GR_BIG_CHAINS 16
#define GR_NPR ((GR_BIG_PMAX * GR_BIG_PMAX + GR_THREADS - 1) / GR_THREADS)
__global__ __launch_bounds__(GR_THREADS) void gr_stats_big_kernel(int P, int64_t n, int K,
                                                                  const double* __restrict__ draws,
                                                                  const int32_t* __restrict__ link,
                                                                  const double* __restrict__ shift,
                                                                  double* __restrict__ partial) {
  __shared__ double tile[GR_TI][GR_BIG_PMAX];
  __shared__ double mean[GR_BIG_PMAX];
  __shared__ double phi[GR_BIG_PMAX];
  const int L = 1 + P + 2 * P * P + 3 * P;
  double a2[GR_NPR], a3[GR_NPR];  // thread-owned (j, l) pairs of sum phi phi' and sum S2
  double a1 = 0.0, a4 = 0.0, a5 = 0.0, a6 = 0.0, m = 0.0;  // thread j < P
#pragma unroll
  for (int u = 0; u < GR_NPR; ++u) { a2[u] = 0.0; a3[u] = 0.0; }
  const int k0 = blockIdx.x * GR_BIG_CHAINS;
  const double den = 1.0 / (double)(n - 1);
  for (int k = k0; k < k0 + GR_BIG_CHAINS && k < K; ++k) {
    if ((int)threadIdx.x < P) {
      const int j = threadIdx.x;
      double sm = 0.0;
      for (int64_t i = 0; i < n; ++i) sm += gr_link(link[j], draws[(size_t)(i * P + j) * K + k]);
      mean[j] = sm / (double)n;
      phi[j] = mean[j] - shift[j];
    }
    __syncthreads();
    double cp[GR_NPR];
#pragma unroll
    for (int u = 0; u < GR_NPR; ++u) cp[u] = 0.0;
    for (int64_t i0 = 0; i0 < n; i0 += GR_TI) {
      for (int q = threadIdx.x; q < GR_TI * P; q += blockDim.x) {
        const int ii = q / P, j = q % P;
        tile[ii][j] = (i0 + ii < n) ? gr_link(link[j], draws[(size_t)((i0 + ii) * P + j) * K + k]) - mean[j] : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < GR_NPR; ++u) {
        const int pr = u * GR_THREADS + threadIdx.x;
        if (pr < P * P) {
          const int j = pr / P, l = pr % P;
          double c = cp[u];
          for (int ii = 0; ii < GR_TI; ++ii) c = fma(tile[ii][j], tile[ii][l], c);
          cp[u] = c;
        }
      }
      __syncthreads();
    }
    // this chain's terms: [1, phi, phi phi', S2, s2^2, s2 phi, s2 phi^2]
    m += 1.0;
#pragma unroll
    for (int u = 0; u < GR_NPR; ++u) {
      const int pr = u * GR_THREADS + threadIdx.x;
      if (pr < P * P) {
        const int j = pr / P, l = pr % P;
        a2[u] += phi[j] * phi[l];
        a3[u] += cp[u] * den;
      }
    }
    if ((int)threadIdx.x < P) a1 += phi[threadIdx.x];
#pragma unroll
    for (int u = 0; u < GR_NPR; ++u) {
      const int pr = u * GR_THREADS + threadIdx.x;
      if (pr < P * P && pr / P == pr % P) tile[0][pr / P] = cp[u] * den;  // s2_j to its thread j
    }
    __syncthreads();
    if ((int)threadIdx.x < P) {
      const int j = threadIdx.x;
      const double s2 = tile[0][j];
      a4 += s2 * s2;
      a5 += s2 * phi[j];
      a6 += s2 * phi[j] * phi[j];
    }
    __syncthreads();
  }
  double* out = partial + (size_t)blockIdx.x * L;
  if (threadIdx.x == 0) out[0] = m;
  if ((int)threadIdx.x < P) {
    const int j = threadIdx.x;
    out[1 + j] = a1;
    out[1 + 2 * P * P + P + j] = a4;
    out[1 + 2 * P * P + 2 * P + j] = a5;
    out[1 + 2 * P * P + 3 * P + j] = a6;
  }
#pragma unroll
  for (int u = 0; u < GR_NPR; ++u) {
    const int pr = u * GR_THREADS + threadIdx.x;
    if (pr < P * P) {
      out[1 + P + pr] = a2[u];
      out[1 + P + P * P + pr] = a3[u];
    }
  }
}

__global__ __launch_bounds__(GR_THREADS) void gr_range_kernel(int p, int64_t total, const double* __restrict__ draws,
                                                              int K, double* __restrict__ partial) {
  // total = n * p * K elements; param of element q is (q / K) % p
  __shared__ double rmin[GR_THREADS], rmax[GR_THREADS];
  for (int j = 0; j < p; ++j) {
    double lo = __builtin_inf(), hi = -__builtin_inf();
    const int64_t n = total / ((int64_t)p * K);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n * K;
         q += (int64_t)gridDim.x * blockDim.x) {
      int64_t i = q / K, k = q % K;
      double x = draws[(size_t)(i * p + j) * K + k];
      lo = fmin(lo, x);
      hi = fmax(hi, x);
    }
    rmin[threadIdx.x] = lo;
    rmax[threadIdx.x] = hi;
    __syncthreads();
    for (int s = GR_THREADS / 2; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) {
        rmin[threadIdx.x] = fmin(rmin[threadIdx.x], rmin[threadIdx.x + s]);
        rmax[threadIdx.x] = fmax(rmax[threadIdx.x], rmax[threadIdx.x + s]);
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      partial[((size_t)blockIdx.x * p + j) * 2 + 0] = rmin[0];
      partial[((size_t)blockIdx.x * p + j) * 2 + 1] = rmax[0];
    }
    __syncthreads();
  }
}

static const int GR_RANGE_BLOCKS = 512;

hipError_t mmb_launch_gr_range(int pmon, int64_t n, int K, const double* draws, double* out,
                               hipStream_t st) {
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, (size_t)GR_RANGE_BLOCKS * pmon * 2 * sizeof(double), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gr_range_kernel, dim3(GR_RANGE_BLOCKS), dim3(GR_THREADS), 0, st, pmon,
                     n * pmon * (int64_t)K, draws, K, part);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  double* h = new double[(size_t)GR_RANGE_BLOCKS * pmon * 2];
  e = hipMemcpyAsync(h, part, (size_t)GR_RANGE_BLOCKS * pmon * 2 * sizeof(double), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess) {
    double res[2 * GR_BIG_PMAX];
    for (int j = 0; j < pmon; ++j) {
      double lo = __builtin_inf(), hi = -__builtin_inf();
      for (int b = 0; b < GR_RANGE_BLOCKS; ++b) {
        lo = fmin(lo, h[((size_t)b * pmon + j) * 2]);
        hi = fmax(hi, h[((size_t)b * pmon + j) * 2 + 1]);
      }
      res[2 * j] = lo;
      res[2 * j + 1] = hi;
    }
    e = hipMemcpyAsync(out, res, 2 * pmon * sizeof(double), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  delete[] h;
  (void)hipFreeAsync(part, st);
  return e;
}

hipError_t mmb_launch_gr_stats(int pmon, int64_t n, int K, const double* draws, const int32_t* link,
                               const double* shift, double* stats, hipStream_t st) {
  if (pmon < 1 || pmon > GR_BIG_PMAX) return hipErrorInvalidValue;
  const int L = 1 + pmon + 2 * pmon * pmon + 3 * pmon;
  const bool big = pmon > GR_PMAX;
  const int blocks = big ? (K + GR_BIG_CHAINS - 1) / GR_BIG_CHAINS : (K + GR_THREADS - 1) / GR_THREADS;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, (size_t)blocks * L * sizeof(double), st);
  if (e != hipSuccess) return e;
  if (big)
    hipLaunchKernelGGL(gr_stats_big_kernel, dim3(blocks), dim3(GR_THREADS), 0, st, pmon, n, K, draws, link, shift,
                       part);
  else switch (pmon) {
    case 1: hipLaunchKernelGGL(gr_stats_kernel<1>, dim3(blocks), dim3(GR_THREADS), 0, st, n, K, draws, link, shift, part); break;
    case 2: hipLaunchKernelGGL(gr_stats_kernel<2>, dim3(blocks), dim3(GR_THREADS), 0, st, n, K, draws, link, shift, part); break;
    case 3: hipLaunchKernelGGL(gr_stats_kernel<3>, dim3(blocks), dim3(GR_THREADS), 0, st, n, K, draws, link, shift, part); break;
    default: hipLaunchKernelGGL(gr_stats_kernel<4>, dim3(blocks), dim3(GR_THREADS), 0, st, n, K, draws, link, shift, part); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  double* h = new double[(size_t)blocks * L];
  e = hipMemcpyAsync(h, part, (size_t)blocks * L * sizeof(double), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess) {
    double* res = new double[L];
    for (int i = 0; i < L; ++i) {
      double s = 0.0;
      for (int b = 0; b < blocks; ++b) s += h[(size_t)b * L + i];
      res[i] = s;
    }
    e = hipMemcpyAsync(stats, res, L * sizeof(double), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    delete[] res;
  }
  delete[] h;
  (void)hipFreeAsync(part, st);
  return e;
}
