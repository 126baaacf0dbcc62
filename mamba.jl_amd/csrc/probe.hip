// probe.hip — test entry for the 32-lane pivoted Cholesky of the AMM update (samplers.h pchol32)
// on caller-supplied matrices: the very function the rats / node-IR sweep kernels inline, run on
// packed symmetric matrices the tests craft (ties, zero / negative / NaN / huge / tiny pivots,
// subnormals), so the optimistic pass's post-hoc check and its checked redo can be compared with
// the oracle's dpstf2 (oracle.c orc_pchol; amm.jl:87, LAPACK dpstf2 for n < 64) on inputs the
// sampler rarely produces.  Diagnostics only (mmb_debug_pchol); not on the sampling path.
#include "sweep.h"

namespace {
using PM = Mdl<MMB_MODEL_RATS>;
using PS = Smp<PM>;
constexpr int PB_CHAINS = 8;                        // 256 threads = 8 lane groups
constexpr int PB_LDS = PM::TP + PM::DP + PM::DP / 2;  // mat | pivot-row buffer | pivot order (ints)
}  // namespace

// S: [n][TP] packed lower triangle (slot(i, k) = tri(i) + k, i >= k) of each matrix.
// Out, per matrix: L [n][TP] the factor in position form (row at pivot position t at tri(t) + k;
// written on full rank only), pos [n][32] each element's pivot position, info [n][2] = rank, redo.
__global__ __launch_bounds__(256) void pchol_probe_kernel(int n, int d, const double* S, double* L,
                                                          int32_t* pos, int32_t* info) {
  __shared__ __attribute__((aligned(16))) double sm[PB_CHAINS * PB_LDS];
  const int grp = (int)(threadIdx.x / 32), lane = (int)(threadIdx.x & 31);
  const int c = (int)blockIdx.x * PB_CHAINS + grp;
  if (c >= n) return;  // whole lane groups exit together
  double* mat = sm + grp * PB_LDS;
  double* prow = mat + PM::TP;
  int* pks = (int*)(prow + PM::DP);
  for (int u = lane; u < PM::TP; u += 32) mat[u] = S[(size_t)c * PM::TP + u];
  grp_sync();
  Grp<32> g;
  int pe = 0, redo = 0;
  const int rank = PS::pchol32(d, mat, prow, pks, g, &pe, nullptr, SweepArgs{}, 0, 0u, 0, 0, 0, &redo);
  grp_sync();
  if (rank == d)
    for (int u = lane; u < PM::TP; u += 32) L[(size_t)c * PM::TP + u] = mat[u];
  pos[(size_t)c * 32 + lane] = lane < d ? pe : -1;
  if (lane == 0) {
    info[2 * c] = rank;
    info[2 * c + 1] = redo;
  }
}

hipError_t mmb_launch_pchol_probe(int n, int d, const double* S, double* L, int32_t* pos, int32_t* info,
                                  hipStream_t st) {
  if (n < 1 || d < 1 || d > PM::DMAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pchol_probe_kernel, dim3((n + PB_CHAINS - 1) / PB_CHAINS), dim3(256), 0, st, n, d, S, L, pos,
                     info);
  return hipGetLastError();
}
