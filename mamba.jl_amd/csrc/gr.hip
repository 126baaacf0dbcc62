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
    double res[2 * GR_PMAX * 16];
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
  if (pmon < 1 || pmon > GR_PMAX) return hipErrorInvalidValue;
  const int L = 1 + pmon + 2 * pmon * pmon + 3 * pmon;
  const int blocks = (K + GR_THREADS - 1) / GR_THREADS;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, (size_t)blocks * L * sizeof(double), st);
  if (e != hipSuccess) return e;
  switch (pmon) {
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
    double res[1 + GR_PMAX + 2 * GR_PMAX * GR_PMAX + 3 * GR_PMAX];
    for (int i = 0; i < L; ++i) {
      double s = 0.0;
      for (int b = 0; b < blocks; ++b) s += h[(size_t)b * L + i];
      res[i] = s;
    }
    e = hipMemcpyAsync(stats, res, L * sizeof(double), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  delete[] h;
  (void)hipFreeAsync(part, st);
  return e;
}
