// sweep.hip — the static instantiations of the block-sweep kernel (sweep.h) and their
// host-side launchers (line, rats, the node-IR interpreter).
#include "sweep.h"
#include <cstdlib>

#ifdef MMB_PHASE_PROF
#include <cstdio>
__device__ unsigned long long mmb_prof[32];
void mmb_prof_dump() {
  unsigned long long h[32];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(mmb_prof), sizeof h) != hipSuccess) return;
  const char* names[] = {"-", "amm:load m/fl/Mv", "amm:proposal", "amm:logf x2+accept", "amm:moments+Sigma",
                         "amm:pchol", "amm:store", "gibbs", "iteration", "count", "pchol:steps",
                         "pchol:carry", "pchol:writeback", "amwg", "slice", "-"};
  for (int i = 1; i < 15; ++i) fprintf(stderr, "MMB_PROF %-22s %llu\n", names[i], h[i]);
}
#endif

template <int MODEL, unsigned KINDS>
static hipError_t launch(const SweepArgs& A, hipStream_t st, int threads) {
  using M = Mdl<MODEL>;
  const int per_block = threads / M::G;
  const int blocks = (A.K + per_block - 1) / per_block;
  const size_t lds = (size_t)per_block * M::lds_stride(A) * sizeof(double);
  hipLaunchKernelGGL((sweep_kernel<MODEL, KINDS>), dim3(blocks), dim3(threads), lds, st, A);
  return hipGetLastError();
}

hipError_t mmb_launch_line_amm(const SweepArgs& A, hipStream_t st);  // line_amm.hip

// host-side launcher (engine.cpp); kinds = bitmask of the scheme's sampler kinds
#ifndef MMB_RATS_BLOCK
#define MMB_RATS_BLOCK 256
#endif
hipError_t mmb_launch_sweep(int model, unsigned kinds, const SweepArgs& A, hipStream_t st) {
  if (model == MMB_MODEL_RATS) {
    constexpr int TB = MMB_RATS_BLOCK;
    if ((kinds & ~K_GIBBS_AMM) == 0) return launch<MMB_MODEL_RATS, K_GIBBS_AMM>(A, st, TB);
    if ((kinds & ~K_SLICE_AMWG) == 0) return launch<MMB_MODEL_RATS, K_SLICE_AMWG>(A, st, TB);
    return launch<MMB_MODEL_RATS, K_ALL>(A, st, TB);
  }
  if (model == MMB_MODEL_IR) return launch<MMB_MODEL_IR, K_IR>(A, st, 128);
  if (model == MMB_MODEL_LINE) {
    // one AMM block (BASELINE configs[1]): four lanes per chain, tune state in registers
    // (line_amm.hip); bit-identical to the generic kernel, which MMB_LINE_GENERIC=1 selects
    if (kinds == (1u << MMB_SAMPLER_AMM) && A.nb == 1 && !std::getenv("MMB_LINE_GENERIC"))
      return mmb_launch_line_amm(A, st);
    if (kinds & K_GRAD) return launch<MMB_MODEL_LINE, K_ALL_GRAD>(A, st, 64);
    return launch<MMB_MODEL_LINE, K_ALL>(A, st, 64);
  }
  return hipErrorInvalidValue;
}
