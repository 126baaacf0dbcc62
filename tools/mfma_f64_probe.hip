// mfma_f64_probe.hip — issue rate and dependent latency of v_mfma_f64_16x16x4_f64 on gfx950
// (one wave per SIMD; cycles from s_memtime).  Sizes the logistic gradient kernel's
// accumulator interleave.   hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_probe.hip -o /tmp/probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ void probe(double* out, long long* cyc, int iters) {
  const int l = threadIdx.x & 63;
  double a = 1.0 + l * 1e-3, b = 0.5 - l * 1e-4;
  d4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  __syncthreads();
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
static void run(int waves_per_simd) {
  const int iters = 4096, blocks = 256;
  double* out;
  long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * 64 * 4 * waves_per_simd);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  hipLaunchKernelGGL(probe<CH>, dim3(blocks), dim3(64 * 4 * waves_per_simd), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  long long h[256];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)h[i];
  avg /= blocks;
  // s_memtime ticks at the shader clock per the guide
  printf("chains/wave %d waves/SIMD %d: %.1f cycles per MFMA per wave, %.1f cycles per MFMA per SIMD\n", CH,
         waves_per_simd, avg / (iters * CH), avg / (iters * CH * waves_per_simd));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<1>(1);
  run<2>(1);
  run<4>(1);
  run<8>(1);
  run<1>(2);
  run<2>(2);
  run<4>(2);
  run<1>(4);
  return 0;
}
