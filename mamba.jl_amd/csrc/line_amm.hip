// line_amm.hip — BASELINE configs[1]: the `line` regression (doc/tutorial/line.jl:5-25) with
// one AMM block (amm.jl:66-108), four lanes per chain.
//
// The generic sweep kernel runs line with one lane per chain (Mdl<LINE>, G = 1): 4,096
// chains are 64 waves on 1,024 SIMDs, and every chain-update is a serial walk through three
// Box-Muller normals, two logpdf evaluations and HBM round trips for the tune state
// (profiles/r3_line_amm_phase.json: 38 k cycles per update, proposal 28 %, logf x2 28 %,
// moments 18 %, factorization 15 %, tune loads/stores 9 %).  Here a quad of lanes owns a
// chain and runs the generic kernel's arithmetic replicated, except where the work splits:
//   * the Philox blocks: lane e < 3 draws normal pair e of the NORMAL substream (z1[e],
//     z2[e]), lane 3 block 0 of the UNIFORM substream (the accept uniform); the quad shares
//     them by DPP quad_perm broadcasts (no LDS);
//   * logpdf: lane 0 evaluates logf(x), lane 1 logf(v);
//   * the tune state (m, flags, Mv, Mvv, the slot-form factor and its pivot order) and the
//     proposal's chol(Sigma) live in registers for the whole launch: loaded once, stored once.
// Everything else (moments, Sigma, the 3 x 3 pivoted Cholesky of Smp<Mdl<LINE>>::pchol in LDS)
// is the generic kernel's code or its operation order, so the draws, the tune state and the
// factor are bit-identical to sweep_kernel<LINE> and to oracle/oracle.c (tests:
// test_gpu_parity.py::test_line_amm_quad_*).  The engine uses this kernel for a line scheme
// that is one AMM block (any d <= 3, emap, transform, sigl, adapt); MMB_LINE_GENERIC=1
// selects the generic kernel.
#include "samplers.h"

namespace {
using ML = Mdl<MMB_MODEL_LINE>;
using SL = Smp<ML>;
constexpr int LQ = 4;      // lanes per chain
constexpr int LDSC = 16;   // LDS doubles per chain: mat[8] | prow[4] | pks[4 ints]

// lane L of each quad to all four (DPP quad_perm, two 32-bit moves)
template <int L>
__device__ __forceinline__ double qbc(double x) {
  constexpr int ctrl = L | (L << 2) | (L << 4) | (L << 6);
  const uint64_t u = mmb_d2u(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), ctrl, 0xf, 0xf, false);
  return mmb_u2d((uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32));
}

// factor entry L[slot(e, q)] of the register copy (d <= 3: slots 0..5), q a run-time index
__device__ __forceinline__ double lsel(const double (&L)[6], int e, int q) {
  const int t = mmb_slot(e, q);
  double r = L[0];
#pragma unroll
  for (int u = 1; u < 6; ++u) r = t == u ? L[u] : r;
  return r;
}
__device__ __forceinline__ double zsel(const double (&z)[3], int k) {
  return k == 0 ? z[0] : k == 1 ? z[1] : z[2];
}
}  // namespace

__global__ __launch_bounds__(64) void line_amm_kernel(const SweepArgs A) {
  __shared__ __attribute__((aligned(16))) double lds_all[64 / LQ * LDSC];
  const int c = (int)((blockIdx.x * blockDim.x + threadIdx.x) / LQ);
  if (c >= A.K) return;  // whole quads exit together
  const int lane = (int)(threadIdx.x & (LQ - 1));
  double* const mat = lds_all + (threadIdx.x / LQ) * LDSC;
  double* const prow = mat + 8;
  int* const pks = (int*)(mat + 12);
  const Grp<1> g1;  // the replicated (one-lane) arithmetic of Mdl<LINE>
  const DBlock& B = mmb_block(A.blocks, 0);
  const int d = B.d;
  const int T = mmb_tri(d);
  const uint32_t chain = A.chain_offset + (uint32_t)c;

  ML::St s;
  ML::Lc l{};
  ML::load(A, c, 0, s, l, mat);
  // proposal factor chol(Sigma) (amm.jl:72): d x d row-major, d <= 3
  double sg[9];
#pragma unroll
  for (int u = 0; u < 9; ++u) sg[u] = u < d * d ? B.sigl[u] : 0.0;
  // tune state (AMMTune, amm.jl:5-35), registers for the launch
  int m = B.t_m[c], fl = B.t_flags[c];
  double mv[3], Mvv[6], L[6];
  int piv[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    mv[r] = r < d ? B.t_Mv[(size_t)c * ML::DP + r] : 0.0;
    piv[r] = r < d ? (int)B.t_piv[(size_t)c * ML::DP + r] : 0;
  }
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    Mvv[t] = t < T ? B.t_Mvv[(size_t)c * ML::TP + t] : 0.0;
    L[t] = t < T ? B.t_Ls[(size_t)c * ML::TP + t] : 0.0;
  }

  for (int step = 0; step < A.n_iters; ++step) {
    const int64_t it = A.iter0 + 1 + step;
    const bool adapt = B.adapt == MMB_ADAPT_ALL ? true : B.adapt == MMB_ADAPT_BURNIN ? (it <= A.model_burnin) : false;
    double v[3];
    ML::unlist(B, s, 0, v);
    const bool fresh = adapt && !(fl & 1);
    if (fresh) {  // setadapt!: m = 0, Mv = v (aliased), Mvv = v v', SigmaLm = 0
      m = 0;
      fl = (fl | 2) & ~4;
#pragma unroll
      for (int r = 0; r < 3; ++r) mv[r] = v[r];
    }
    fl = adapt ? (fl | 1) : (fl & ~1);
    // the iteration's Philox blocks, one per lane: normal pairs 0..2, then the accept uniform
    {
      const mmb_rng rq = mmb_rng_make(A.seed, chain, (uint32_t)it, 0u, lane < 3 ? MMB_SUB_NORMAL : MMB_SUB_UNIFORM);
      uint64_t ba, bb;
      mmb_rng_block(&rq, lane < 3 ? (uint32_t)lane : 0u, &ba, &bb);
      double n0, n1;
      mmb_normal_pair_bits(ba, bb, &n0, &n1);
      const double uown = mmb_u01(ba);
      double z1[3], z2[3];
      z1[0] = qbc<0>(n0); z2[0] = qbc<0>(n1);
      z1[1] = qbc<1>(n0); z2[1] = qbc<1>(n1);
      z1[2] = qbc<2>(n0); z2[2] = qbc<2>(n1);
      const double ua = qbc<3>(uown);
#pragma unroll
      for (int r = 0; r < 3; ++r)
        if (r >= d) { z1[r] = 0.0; z2[r] = 0.0; }
      // proposal: x = SigmaL z1 [; beta x + (1 - beta) SigmaLm z2]; x += v  (amm.jl:72-76)
      double x[3];
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        double a = 0.0;
        if (e < d) {
          if (B.sigl_diag) {
            a = fma(sg[e * d + e], z1[e], a);
          } else {
#pragma unroll
            for (int k = 0; k <= e; ++k) a = fma(sg[e * d + k], z1[k], a);
          }
        }
        x[e] = a;
      }
      if (m > 2 * d) {
        double y[3] = {0.0, 0.0, 0.0};
        if (fl & 4) {  // slot-form factor, pivot order piv: the generic kernel's matvec
#pragma unroll
          for (int e = 0; e < 3; ++e) {
            if (e < d) {
              int pe = 0;
#pragma unroll
              for (int k = 0; k < 3; ++k)
                if (k < d && piv[k] == e) pe = k;
              double a = 0.0;
#pragma unroll
              for (int k = 0; k < 3; ++k)
                if (k < d) a = (k < pe) ? fma(lsel(L, e, piv[k]), z2[k], a) : a;
              y[e] = fma(L[mmb_tri(e) + e], zsel(z2, pe), a);
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) x[r] = B.beta * x[r] + (1.0 - B.beta) * y[r];
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) x[r] = x[r] + v[r];
      // logf(x) on lane 0, logf(v) on lane 1 (the others repeat lane 1's)
      double xin[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) xin[r] = lane == 0 ? x[r] : v[r];
      const double lf = ML::logf(A, B, s, l, g1, xin);
      const double lx = qbc<0>(lf), lv = qbc<1>(lf);
      if (ua < mmb_exp(lx - lv)) {
#pragma unroll
        for (int r = 0; r < 3; ++r) v[r] = x[r];
      }
    }
    if (adapt) {  // amm.jl:81-91
      m += 1;
      const double p = (double)m / ((double)m + 1.0);
      const double q = 1.0 - p;
      if (fl & 2) {
#pragma unroll
        for (int r = 0; r < 3; ++r) mv[r] = p * v[r] + q * v[r];
        fl &= ~2;
      } else {
#pragma unroll
        for (int r = 0; r < 3; ++r) mv[r] = p * mv[r] + q * v[r];
      }
      const double cc = (B.scale * B.scale / (double)d) / p;
      double vold[3];
      ML::unlist(B, s, 0, vold);  // fresh: Mvv = v_old v_old' (s still holds v_old)
      // packed slots t = tri(i) + k, k <= i < d
#pragma unroll
      for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int k = 0; k <= i; ++k) {
          const int t = mmb_tri(i) + k;
          if (i < d) {
            const double old = fresh ? vold[i] * vold[k] : Mvv[t];
            const double nv = p * old + (q * v[k]) * v[i];
            Mvv[t] = nv;
            mat[t] = cc * (nv - mv[k] * mv[i]);
          }
        }
      }
      ML::relist(B, s, g1, v);
      grp_sync();
      const int rank = SL::pchol(d, mat, prow, pks, g1);
      grp_sync();
      if (rank == d) {
#pragma unroll
        for (int t = 0; t < 6; ++t)
          if (t < T) L[t] = mat[t];
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (k < d) piv[k] = pks[k];
        fl |= 4;
      }
      grp_sync();
    } else {
      ML::relist(B, s, g1, v);
    }
    if (A.draws && it > A.burnin && (it - A.burnin) % A.thin == 0 && lane == 0) {
      const int64_t row = (it - A.burnin) / A.thin - 1 - A.kept_origin;
      ML::write_draws(A, s, g1, row, c);
    }
  }
  if (lane == 0) {
    ML::store(A, c, 0, s);
    B.t_m[c] = m;
    B.t_flags[c] = fl;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      if (r < d) {
        B.t_Mv[(size_t)c * ML::DP + r] = mv[r];
        B.t_piv[(size_t)c * ML::DP + r] = (uint8_t)piv[r];
      }
    }
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      if (t < T) {
        B.t_Mvv[(size_t)c * ML::TP + t] = Mvv[t];
        B.t_Ls[(size_t)c * ML::TP + t] = L[t];
      }
    }
  }
}

hipError_t mmb_launch_line_amm(const SweepArgs& A, hipStream_t st) {
  const int threads = 64;
  const int blocks = (int)(((int64_t)A.K * LQ + threads - 1) / threads);
  hipLaunchKernelGGL(line_amm_kernel, dim3(blocks), dim3(threads), 0, st, A);
  return hipGetLastError();
}
