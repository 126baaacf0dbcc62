// sweep.h — the fused block-sweep kernel: one launch advances every chain of the
// shard through `n_iters` iterations of sample!(m) (simulation.jl:93-107), i.e.
// mcmc_worker!'s loop body (mcmc.jl:74-80) including the keep rule and the
// Chains write sim[i,:,1] = unlist(m, true) (mcmc.jl:76-77).
//
// Per chain, per iteration: values are held in registers; AMWG/AMM tune state
// and the AMM moment/factor matrices are streamed from/to HBM (chain-major,
// element fastest, coalesced per lane group); the AMM covariance and its
// pivoted Cholesky factor are staged in LDS.  Shared by sweep.hip (the static
// kernels) and the node-IR JIT kernel (engine.cpp ir_jit_source, compiled by hipRTC).
#pragma once
#include "samplers.h"
#include "ir.h"

#ifdef MMB_PHASE_PROF
extern __device__ unsigned long long mmb_prof[32];
#endif

#ifndef MMB_SWEEP_WAVES
#define MMB_SWEEP_WAVES 4  // rats: min waves per SIMD the register allocator must allow
#endif
// Occupancy target per model: rats runs 8192 waves and is latency-bound (4 waves/SIMD
// measured 12 % faster than 3 despite spills); line has 64 waves in all, so it keeps the
// whole register budget (no spills).
#ifndef MMB_IR_WAVES
#define MMB_IR_WAVES 2  // node IR: min waves per SIMD (register budget 512 / waves)
#endif
template <int MODEL>
constexpr int sweep_waves() {
  return MODEL == MMB_MODEL_RATS ? MMB_SWEEP_WAVES : MODEL == MMB_MODEL_IR ? MMB_IR_WAVES : 1;
}

// KINDS: bitmask (1 << mmb_sampler_kind) of the sampler kinds present in the scheme; the
// other block paths are compiled out (register/SGPR allocation is per kernel).
template <int MODEL, unsigned KINDS>
__device__ __forceinline__ void sweep_body(const SweepArgs& A) {
  using M = Mdl<MODEL>;
  using S = Smp<M>;
  constexpr int G = M::G;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  if constexpr ((KINDS >> MMB_SAMPLER_AMM) & 1u) {  // moment-update slot table (before any exit)
    S::ik_fill();
    __syncthreads();
  }
  const int slot = (int)((blockIdx.x * blockDim.x + threadIdx.x) / G);
  if (slot >= A.K) return;  // whole lane groups exit together
  // chain of this lane group: the engine may order the chains so that chains whose pivoted
  // Cholesky stops early share wavefronts (engine.cpp order_chains); every index below --
  // state, tune, draws column, Philox chain id -- is the chain's own, so results do not depend
  // on the order
  const int c = A.cperm != nullptr ? A.cperm[slot] : slot;
  Grp<G> g;
  double* lds = smem + (size_t)(threadIdx.x / G) * M::lds_stride(A);
  typename M::St s;
  typename M::Lc l;
  M::load(A, c, g.lane, s, l, lds);
  const uint32_t chain = A.chain_offset + (uint32_t)c;
#ifdef MMB_PHASE_PROF
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < 16; ++i) mmb_prof_lds()[i] = 0;
#endif
  for (int step = 0; step < A.n_iters; ++step) {
    const int64_t it = A.iter0 + 1 + step;
#ifdef MMB_PHASE_PROF
    const uint64_t _it0 = __builtin_amdgcn_s_memtime();
#endif
    // state-independent draws of the whole iteration, one block per lane (32-lane groups)
    double pre = 0.0;
    if constexpr (G == 32 && (KINDS & ((1u << MMB_SAMPLER_GIBBS) | (1u << MMB_SAMPLER_AMM))) != 0u)
      pre = S::predraw(A, chain, it, g);
    for (int b = 0; b < A.nb; ++b) {
      // descriptor read through the constant address space: uniform scalar loads (s_load,
      // scalar cache) instead of vector loads that wait on the vector memory path
      const DBlock& B = mmb_block(A.blocks, b);
      const mmb_rng rn = mmb_rng_make(A.seed, chain, (uint32_t)it, (uint32_t)b, MMB_SUB_NORMAL);
      const mmb_rng ru = mmb_rng_make(A.seed, chain, (uint32_t)it, (uint32_t)b, MMB_SUB_UNIFORM);
      const bool adapt = B.adapt == MMB_ADAPT_ALL ? true
                         : B.adapt == MMB_ADAPT_BURNIN ? (it <= A.model_burnin) : false;
      switch (B.kind) {
        case MMB_SAMPLER_AMWG:
          if constexpr ((KINDS >> MMB_SAMPLER_AMWG) & 1u) {
            MMB_PROF_START
            S::amwg(A, B, c, rn, ru, adapt, s, l, g);
            MMB_PROF_MARK(13, g.lane)
          }
          break;
        case MMB_SAMPLER_AMM:
          if constexpr ((KINDS >> MMB_SAMPLER_AMM) & 1u) S::amm(A, B, c, chain, it, b, rn, ru, adapt, s, l, g, lds,
                                                                        G == 32 ? S::lane_value(pre, b) : 0.0);
          break;
        case MMB_SAMPLER_SLICE:
          if constexpr ((KINDS >> MMB_SAMPLER_SLICE) & 1u) {
            MMB_PROF_START
            if (B.form == MMB_SLICE_UNIVARIATE) S::slice_uni(A, B, ru, s, l, g, lds);
            else S::slice_multi(A, B, ru, s, l, g, lds);
            MMB_PROF_MARK(14, g.lane)
          }
          break;
        case MMB_SAMPLER_NUTS:
          if constexpr ((KINDS >> MMB_SAMPLER_NUTS) & 1u) S::nuts(A, B, c, it, b, s, g);
          break;
        case MMB_SAMPLER_HMC:
          if constexpr ((KINDS >> MMB_SAMPLER_HMC) & 1u) S::template hmc<false>(A, B, c, rn, ru, s, g);
          break;
        case MMB_SAMPLER_MALA:
          if constexpr ((KINDS >> MMB_SAMPLER_MALA) & 1u) S::template hmc<true>(A, B, c, rn, ru, s, g);
          break;
        case MMB_SAMPLER_GIBBS: if constexpr ((KINDS >> MMB_SAMPLER_GIBBS) & 1u) {
          const mmb_rng gn = mmb_rng_make(A.seed, chain, (uint32_t)it, (uint32_t)b, MMB_SUB_GAMMA_N);
          const mmb_rng gu = mmb_rng_make(A.seed, chain, (uint32_t)it, (uint32_t)b, MMB_SUB_GAMMA_U);
          MMB_PROF_START
          M::gibbs(A, B, s, l, g, &rn, &gn, &gu, G == 32 ? S::lane_value(pre, b) : 0.0);
          MMB_PROF_MARK(7, g.lane)
        }
          break;
        default:
          break;
      }
    }
#ifdef MMB_PHASE_PROF
    if ((threadIdx.x & 63) == 0) {
      mmb_prof_lds()[8] += __builtin_amdgcn_s_memtime() - _it0;
      mmb_prof_lds()[9] += 1;
    }
#endif
    if (A.draws && it > A.burnin && (it - A.burnin) % A.thin == 0) {
      const int64_t row = (it - A.burnin) / A.thin - 1 - A.kept_origin;
      M::write_draws(A, s, g, row, c);
    }
  }
  M::store(A, c, g.lane, s);
#ifdef MMB_PHASE_PROF
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < 16; ++i) atomicAdd(&mmb_prof[i], mmb_prof_lds()[i]);
#endif
}

template <int MODEL, unsigned KINDS>
__global__ __launch_bounds__(256, sweep_waves<MODEL>()) void sweep_kernel(const SweepArgs A) {
  sweep_body<MODEL, KINDS>(A);
}

constexpr unsigned K_ALL = (1u << MMB_SAMPLER_AMWG) | (1u << MMB_SAMPLER_AMM) |
                         (1u << MMB_SAMPLER_SLICE) | (1u << MMB_SAMPLER_GIBBS);
constexpr unsigned K_GRAD = (1u << MMB_SAMPLER_NUTS) | (1u << MMB_SAMPLER_HMC) | (1u << MMB_SAMPLER_MALA);
constexpr unsigned K_ALL_GRAD = K_ALL | K_GRAD;
constexpr unsigned K_GIBBS_AMM = (1u << MMB_SAMPLER_AMM) | (1u << MMB_SAMPLER_GIBBS);
constexpr unsigned K_SLICE_AMWG = (1u << MMB_SAMPLER_AMWG) | (1u << MMB_SAMPLER_SLICE);
constexpr unsigned K_IR = (1u << MMB_SAMPLER_AMWG) | (1u << MMB_SAMPLER_AMM) | (1u << MMB_SAMPLER_SLICE) | K_GRAD;

