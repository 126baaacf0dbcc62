// Probe: cost of a cooperative-groups grid barrier vs a dependent kernel launch on one stream
// (448 workgroups x 256 threads, the persistent-tail grid of the logistic engine).
// Build: hipcc --offload-arch=gfx950 -O3 tools/gridsync_probe.hip -o /tmp/gsp
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
namespace cg = cooperative_groups;

__global__ void sync_kernel(int n, int* out) {
  cg::grid_group g = cg::this_grid();
  int acc = 0;
  for (int i = 0; i < n; ++i) {
    acc += (int)threadIdx.x;
    g.sync();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = acc;
}
__global__ void empty_kernel(int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += 1;
}

int main() {
  int* d;
  hipMalloc(&d, 64);
  hipStream_t st;
  hipStreamCreate(&st);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int wg : {64, 192, 448}) {
    int n = 2000;
    void* args[] = {&n, &d};
    // warm-up
    int n0 = 10;
    void* args0[] = {&n0, &d};
    hipError_t e = hipLaunchCooperativeKernel((const void*)sync_kernel, dim3(wg), dim3(256), args0, 0, st);
    if (e != hipSuccess) { printf("coop launch failed: %s\n", hipGetErrorString(e)); return 1; }
    hipStreamSynchronize(st);
    hipEventRecord(a, st);
    hipLaunchCooperativeKernel((const void*)sync_kernel, dim3(wg), dim3(256), args, 0, st);
    hipEventRecord(b, st);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("wg %d: grid sync %.3f us each\n", wg, ms * 1e3 / n);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(empty_kernel, dim3(wg), dim3(256), 0, st, d);
    hipStreamSynchronize(st);
    hipEventRecord(a, st);
    for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(empty_kernel, dim3(wg), dim3(256), 0, st, d);
    hipEventRecord(b, st);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("wg %d: empty dependent launch %.3f us each\n", wg, ms * 1e3 / 2000);
  }
  return 0;
}
