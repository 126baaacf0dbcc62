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

// Wavefront pairing (engine.cpp order_chains): the slot -> chain table of the next window as a
// stable counting sort of the chains by class, on the engine stream right behind the previous
// window's last launch (no host round trip).  Class of chain k: per AMM block (the first block
// most significant, at most MMB_ORDER_BLOCKS of them), whether it holds a valid factor (flags
// bit 2).  One workgroup: thread t owns chains [t*C, (t+1)*C); the per-(class, thread) counts sit
// in LDS class-major, so one exclusive scan of that array gives every thread the first slot of
// its chains of each class, and chains of one class keep their index order.
constexpr int ORD_T = 1024;
constexpr int ORD_KC = 16384;  // shards up to this size read the flags once, coalesced, into LDS
__global__ __launch_bounds__(ORD_T) void order_chains_kernel(const OrderArgs a) {
  __shared__ int32_t cnt[(1 << MMB_ORDER_BLOCKS) * ORD_T];
  __shared__ int32_t wsum[ORD_T / 64];
  __shared__ uint8_t ccls[ORD_KC];
  const int t = (int)threadIdx.x;
  const int NC = 1 << a.nblk;
  const int C = (a.K + ORD_T - 1) / ORD_T;
  const int k0 = min(a.K, t * C), k1 = min(a.K, k0 + C);
  auto gcls = [&](int k) {
    int c = 0;
    for (int b = 0; b < a.nblk; ++b) c = (c << 1) | ((a.flags[b][k] >> 2) & 1);
    return c;
  };
  const bool cached = a.K <= ORD_KC;
  if (cached) {
    for (int k = t; k < a.K; k += ORD_T) ccls[k] = (uint8_t)gcls(k);
    __syncthreads();
  }
  auto cls = [&](int k) { return cached ? (int)ccls[k] : gcls(k); };
  for (int c = 0; c < NC; ++c) cnt[c * ORD_T + t] = 0;
  for (int k = k0; k < k1; ++k) cnt[cls(k) * ORD_T + t] += 1;
  __syncthreads();
  // exclusive scan of cnt[0 .. NC*T): thread t owns NC consecutive entries
  int* own = cnt + t * NC;
  int s = 0;
  for (int i = 0; i < NC; ++i) s += own[i];
  const int lane = t & 63, w = t >> 6;
  int inc = s;  // inclusive wave scan
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(inc, d, 64);
    if (lane >= d) inc += v;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < w; ++i) base += wsum[i];
  int run = base + inc - s;
  __syncthreads();  // every thread has read the counts it owns before they are overwritten
  for (int i = 0; i < NC; ++i) {
    const int v = own[i];
    own[i] = run;
    run += v;
  }
  __syncthreads();
  // sorted position -> slot.  mode 1: reversed (slow classes dispatched first).  mode 2: the chain pairs of a wavefront stay consecutive in the
  // sorted order, but the W waves of a workgroup take their pairs from W different stretches of
  // it (pair q -> wave q / NF of workgroup q % NF, NF full workgroups), so every workgroup holds
  // fast and slow classes alike and the second dispatch round does not end on the slowest ones
  const int W = a.cpw / 2, NF = a.K / a.cpw;
  for (int k = k0; k < k1; ++k) {
    int* p = &cnt[cls(k) * ORD_T + t];
    int pos = *p;
    *p += 1;
    if (a.mode == 1) pos = a.K - 1 - pos;
    if (a.mode == 2 && W > 0 && (pos >> 1) < NF * W) {
      const int q = pos >> 1;
      pos = (q % NF) * a.cpw + 2 * (q / NF) + (pos & 1);
    }
    a.perm[pos] = k;
  }
}

hipError_t mmb_launch_order_chains(const OrderArgs& a, hipStream_t st) {
  if (a.nblk < 1 || a.nblk > MMB_ORDER_BLOCKS || a.K < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(order_chains_kernel, dim3(1), dim3(ORD_T), 0, st, a);
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
