// line_amm.hip — BASELINE configs[1]: the `line` regression (doc/tutorial/line.jl:5-25) with
// one AMM block (amm.jl:66-108), four lanes per chain.
//
// The generic sweep kernel runs line with one lane per chain (Mdl<LINE>, G = 1): 4,096
// chains are 64 waves on 1,024 SIMDs, and every chain-update is a serial walk through three
// Box-Muller normals, two logpdf evaluations and HBM round trips for the tune state
// (profiles/r3_line_amm_phase.json: 38 k cycles per update, proposal 28 %, logf x2 28 %,
// moments 18 %, factorization 15 %, tune loads/stores 9 %).  Here a quad of lanes owns a
// chain and runs the generic kernel's arithmetic replicated, except where the work splits or
// can be taken off the update's dependency chain:
//   * the Philox blocks: lane e < 3 draws normal pair e of the NORMAL substream (z1[e],
//     z2[e]), lane 3 block 0 of the UNIFORM substream (the accept uniform); they do not depend
//     on the chain state, so each iteration draws the next one's while its own update runs, and
//     the quad shares them by DPP quad_perm broadcasts (no LDS);
//   * logpdf: lane 0 evaluates logf(x), lane 1 logf(v), each on its own relisted state, which
//     is also the state after the accept (the relist's exp is not repeated); the early exit of
//     Mdl<LINE>::logf becomes selects (line_logf_st);
//   * the tune state (m, flags, Mv, Mvv, the slot-form factor and its pivot order) and the
//     proposal's chol(Sigma) live in registers for the whole launch: loaded once, stored once;
//   * the 3 x 3 pivoted Cholesky runs in registers without branches (pchol3_fast: in-range
//     sqrt / reciprocal of device.h, bit-identical there; pchol3, the exact restatement of
//     Smp<Mdl<LINE>>::pchol, when a pivot falls outside [2^-700, 2^700]).
// The moments, Sigma, the factorization's pivot replay and dot products keep the generic
// kernel's operation order, so the draws, the tune state and the factor are bit-identical to
// sweep_kernel<LINE> and to oracle/oracle.c (tests/test_gpu_line_amm.py at the configuration's
// 4,096 chains).  Measured: 5.61e8 chain-updates/s vs 2.57e8 for the generic kernel (2.2x).
// The engine uses this kernel for a line scheme that is one AMM block (any d <= 3, emap,
// transform, sigl, adapt); MMB_LINE_GENERIC=1 selects the generic kernel.
#include "samplers.h"

#ifdef MMB_PHASE_PROF
#include <cstdio>
__device__ unsigned long long mmb_prof_l[32];
void mmb_prof_dump_line() {
  unsigned long long h[32];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(mmb_prof_l), sizeof h) != hipSuccess) return;
  const char* names[] = {"-", "line:draws", "line:proposal", "line:logf+accept", "line:moments",
                         "line:pchol", "line:tail"};
  for (int i = 1; i < 7; ++i) fprintf(stderr, "MMB_PROF %-22s %llu\n", names[i], h[i]);
}
#endif

namespace {
using ML = Mdl<MMB_MODEL_LINE>;
constexpr int LQ = 4;      // lanes per chain

// lane L of each quad to all four (DPP quad_perm, two 32-bit moves)
template <int L>
__device__ __forceinline__ double qbc(double x) {
  constexpr int ctrl = L | (L << 2) | (L << 4) | (L << 6);
  const uint64_t u = mmb_d2u(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), ctrl, 0xf, 0xf, false);
  return mmb_u2d((uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32));
}

// factor entry L[slot(e, q)] of the register copy (d <= 3: slots 0..5), q a run-time index.
// Bitwise blends, not selects: a chain of `t == u ? L[u] : r` was turned back into an indexed
// array, placed in LDS by the compiler, with a load and a full lgkmcnt wait per entry read.
__device__ __forceinline__ double lsel(const double (&L)[6], int e, int q) {
  const int t = mmb_slot(e, q);
  uint64_t r = 0;
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    uint64_t msk = (uint64_t)0 - (uint64_t)(t == u);
    asm volatile("" : "+v"(msk));
    r |= mmb_d2u(L[u]) & msk;
  }
  return mmb_u2d(r);
}
__device__ __forceinline__ double zsel(const double (&z)[3], int k) {
  return k == 0 ? z[0] : k == 1 ? z[1] : z[2];
}
// Smp<Mdl<LINE>>::pchol (G = 1, dpstf2, oracle.c orc_pchol; amm.jl:86-90) with the d <= 3 matrix in
// registers: the same pivot replay (dpstf2's position swaps), first strict maximum in position
// order, sqrt() and 1.0 / ajj, two-accumulator dot products and in-place slot-form write-back
// (entries after a row's own pivot keep Sigma's value, as in the LDS version), so the factor and
// the pivot order are bit-identical.  S: Sigma in, factor out (when the rank is d).
__device__ __forceinline__ int pchol3(int d, double (&S)[6], int (&pks)[3]) {
  double diag0[3], work[3], Lr[3][3];
  bool done[3];
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    done[e] = !(e < d);
    diag0[e] = e < d ? S[mmb_tri(e) + e] : 0.0;
    work[e] = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) Lr[e][k] = 0.0;
  }
  int rank = d;
  bool live = true;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (live && j < d) {
      double dl[3];
#pragma unroll
      for (int e = 0; e < 3; ++e) dl[e] = diag0[e] - work[e];
      // dpstf2's position swaps replayed from the pivot history
      int perm[3] = {0, 1, 2};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (k < j) {
          const int q = pks[k];
          int qpos = k;
#pragma unroll
          for (int t = 0; t < 3; ++t) qpos = (t >= k && perm[t] == q) ? t : qpos;
          const int tmp = perm[k];
#pragma unroll
          for (int t = 0; t < 3; ++t) perm[t] = (t == qpos) ? tmp : perm[t];
          perm[k] = q;
        }
      }
      int best = -1;
      double bv = 0.0;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        if (t >= j && t < d) {
          const int e = perm[t];
          const double de = e == 0 ? dl[0] : e == 1 ? dl[1] : dl[2];
          if (best < 0) { best = e; bv = de; }
          else if (de > bv) { best = e; bv = de; }
        }
      }
      const int p = best;
      if (!(bv > 0.0)) {
        rank = j;
        live = false;
      } else {
        pks[j] = p;
        const double ajj = sqrt(bv);
        const double rinv = 1.0 / ajj;
        double prow[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) prow[k] = p == 0 ? Lr[0][k] : p == 1 ? Lr[1][k] : Lr[2][k];
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          if (e == p) {
            done[e] = true;
            Lr[e][j] = ajj;
          }
        }
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          if (!done[e]) {
            double t0 = 0.0, t1 = 0.0;
#pragma unroll
            for (int k = 0; k + 1 < j; k += 2) {
              t0 = fma(Lr[e][k], prow[k], t0);
              t1 = fma(Lr[e][k + 1], prow[k + 1], t1);
            }
            if (j & 1) t0 = fma(Lr[e][j - 1], prow[j - 1], t0);
            const int t = mmb_slot(e, p);
            const double sep = t == 0 ? S[0] : t == 1 ? S[1] : t == 2 ? S[2] : t == 3 ? S[3] : t == 4 ? S[4] : S[5];
            const double lij = (sep - (t0 + t1)) * rinv;
            Lr[e][j] = lij;
            work[e] = work[e] + lij * lij;
          }
        }
      }
    }
  }
  if (rank == d) {
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      if (e < d) {
        bool before = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (k < d) {
            const int q = pks[k];
            if (q == e) {
              S[mmb_tri(e) + e] = Lr[e][k];
              before = false;
            } else if (before) {
              const int t = mmb_slot(e, q);
#pragma unroll
              for (int u = 0; u < 6; ++u) S[u] = t == u ? Lr[e][k] : S[u];
            }
          }
        }
      }
    }
  }
  return rank;
}

// pchol3 without branches (every step computed, updates masked by `live`; one basic block the
// scheduler can interleave with the next iteration's independent work), taking the pivot's
// square root and reciprocal from the in-range sequences of device.h (bit-identical to sqrt()
// and 1.0 / x in [2^-700, 2^700]).  Returns false if a taken pivot was outside that range:
// the caller then runs pchol3 (exact sqrt / division) on the saved Sigma.
__device__ __forceinline__ bool pchol3_fast(int d, double (&S)[6], int (&pks)[3], int& rank) {
  double diag0[3], work[3], Lr[3][3];
  bool done[3];
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    done[e] = !(e < d);
    diag0[e] = e < d ? S[mmb_tri(e) + e] : 0.0;
    work[e] = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) Lr[e][k] = 0.0;
  }
  rank = d;
  bool live = true, ok = true;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const bool act = live && j < d;
    double dl[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) dl[e] = diag0[e] - work[e];
    int perm[3] = {0, 1, 2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k < j) {
        const int q = pks[k];
        int qpos = k;
#pragma unroll
        for (int t = 0; t < 3; ++t) qpos = (t >= k && perm[t] == q) ? t : qpos;
        const int tmp = perm[k];
#pragma unroll
        for (int t = 0; t < 3; ++t) perm[t] = (t == qpos) ? tmp : perm[t];
        perm[k] = q;
      }
    }
    int best = -1;
    double bv = 0.0;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      if (t >= j) {
        const int e = perm[t];
        const double de = e == 0 ? dl[0] : e == 1 ? dl[1] : dl[2];
        const bool take = t < d && (best < 0 || de > bv);
        best = take ? e : best;
        bv = take ? de : bv;
      }
    }
    const int p = best < 0 ? 0 : best;
    const bool stop = act && !(bv > 0.0);
    rank = stop ? j : rank;
    const bool step = act && !stop;
    live = live && !stop;
    ok = ok && !(step && !mmb_fast_range(bv));
    double ajj, rinv;
    mmb_sqrt_rcp_inrange(bv, &ajj, &rinv);
    pks[j] = step ? p : pks[j];
    double prow[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) prow[k] = p == 0 ? Lr[0][k] : p == 1 ? Lr[1][k] : Lr[2][k];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const bool pe = step && e == p;
      const bool upd = step && !done[e] && !pe;
      double t0 = 0.0, t1 = 0.0;
#pragma unroll
      for (int k = 0; k + 1 < j; k += 2) {
        t0 = fma(Lr[e][k], prow[k], t0);
        t1 = fma(Lr[e][k + 1], prow[k + 1], t1);
      }
      if (j & 1) t0 = fma(Lr[e][j - 1], prow[j - 1], t0);
      const int t = mmb_slot(e, p);
      const double sep = t == 0 ? S[0] : t == 1 ? S[1] : t == 2 ? S[2] : t == 3 ? S[3] : t == 4 ? S[4] : S[5];
      const double lij = (sep - (t0 + t1)) * rinv;
      Lr[e][j] = pe ? ajj : upd ? lij : Lr[e][j];
      work[e] = upd ? work[e] + lij * lij : work[e];
      done[e] = done[e] || pe;
    }
  }
  if (rank == d) {
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      if (e < d) {
        bool before = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (k < d) {
            const int q = pks[k];
            const int tq = mmb_slot(e, q);
#pragma unroll
            for (int u = 0; u < 6; ++u) S[u] = (before && u == tq) ? Lr[e][k] : S[u];
            before = before && q != e;
          }
        }
      }
    }
  }
  return ok;
}

// logf of Mdl<LINE> (line.jl:5-25) from an already relisted state, without branches: every node
// term and ylp are evaluated, and the early exit of Mdl<LINE>::logf (a non-finite partial sum is
// returned as is) becomes selects -- the same value, bit for bit.
__device__ __forceinline__ double line_logf_st(const SweepArgs& A, const DBlock& B, const ML::St& s) {
  const double tb = (!isfinite(s.v[0]) || !isfinite(s.v[1])) ? -__builtin_inf()
                    : d_iso(2, sqrt(1000.0), s.v[0] * s.v[0] + s.v[1] * s.v[1]);
  const double ts = d_iglogpdf(A.ig_c, s.v[2], B.transform);
  const double t0 = B.nodes[0] == MMB_LINE_BETA ? tb : ts;
  const double t1 = B.nodes[1] == MMB_LINE_BETA ? tb : ts;
  const double yl = ML::ylp(A, s);
  const double lp1 = 0.0 + t0;
  if (B.nn < 2) return isfinite(lp1) ? lp1 + yl : lp1;
  const double lp2 = lp1 + t1;
  return !isfinite(lp1) ? lp1 : isfinite(lp2) ? lp2 + yl : lp2;
}

// the iteration's Philox block for this lane: normal pair `lane` (lanes 0..2) or the accept
// uniform (lane 3) -- state-independent, so it is drawn one iteration ahead
__device__ __forceinline__ void line_draw(const SweepArgs& A, uint32_t chain, int64_t it, int lane, double& n0,
                                          double& n1, double& u) {
  const mmb_rng rq = mmb_rng_make(A.seed, chain, (uint32_t)it, 0u, lane < 3 ? MMB_SUB_NORMAL : MMB_SUB_UNIFORM);
  uint64_t ba, bb;
  mmb_rng_block(&rq, lane < 3 ? (uint32_t)lane : 0u, &ba, &bb);
  mmb_normal_pair_bits(ba, bb, &n0, &n1);
  u = mmb_u01(ba);
}
}  // namespace

__global__ __launch_bounds__(64) void line_amm_kernel(const SweepArgs Ak) {
  const int c = (int)((blockIdx.x * blockDim.x + threadIdx.x) / LQ);
  if (c >= Ak.K) return;  // whole quads exit together
  const int lane = (int)(threadIdx.x & (LQ - 1));
  const Grp<1> g1;  // the replicated (one-lane) arithmetic of Mdl<LINE>
  // the descriptor and the arguments the update loop reads, copied once into registers: read
  // through their constant-memory references, the compiler re-issued scalar loads of them inside
  // the loop under SGPR pressure, each followed by a full lgkmcnt wait (18 per iteration)
  DBlock B = mmb_block(Ak.blocks, 0);
  SweepArgs A = Ak;
  asm volatile("" : "+v"(B.adapt), "+v"(B.sigl_diag), "+v"(B.transform), "+v"(B.nn), "+v"(B.d));
  asm volatile("" : "+v"(B.nodes[0]), "+v"(B.nodes[1]), "+v"(B.nodes[2]), "+v"(B.emap[0]), "+v"(B.emap[1]),
               "+v"(B.emap[2]));
  asm volatile("" : "+v"(B.beta), "+v"(B.scale), "+v"(A.ig_c), "+v"(A.burnin), "+v"(A.thin),
               "+v"(A.model_burnin), "+v"(A.kept_origin));
#pragma unroll
  for (int i = 0; i < 5; ++i) asm volatile("" : "+v"(A.lx[i]), "+v"(A.ly[i]));
  const int d = B.d;
  const int T = mmb_tri(d);
  const uint32_t chain = A.chain_offset + (uint32_t)c;
#ifdef MMB_PHASE_PROF
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < 16; ++i) mmb_prof_lds()[i] = 0;
#endif

  ML::St s;
  ML::Lc l{};
  ML::load(A, c, 0, s, l, nullptr);
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
  const double sc2 = B.scale * B.scale / (double)d;
  double v[3];
  ML::unlist(B, s, 0, v);
  double n0, n1, uown;
  line_draw(A, chain, A.iter0 + 1, lane, n0, n1, uown);
  uint32_t st_fac = 0, st_full = 0, st_rank = 0, st_steps = 0, st_redo = 0;  // mmb_amm_stats

  for (int step = 0; step < A.n_iters; ++step) {
    MMB_PROF_START
    const int64_t it = A.iter0 + 1 + step;
    const bool adapt = B.adapt == MMB_ADAPT_ALL ? true : B.adapt == MMB_ADAPT_BURNIN ? (it <= A.model_burnin) : false;
    const bool fresh = adapt && !(fl & 1);
    if (fresh) {  // setadapt!: m = 0, Mv = v (aliased), Mvv = v v', SigmaLm = 0
      m = 0;
      fl = (fl | 2) & ~4;
#pragma unroll
      for (int r = 0; r < 3; ++r) mv[r] = v[r];
    }
    fl = adapt ? (fl | 1) : (fl & ~1);
    // moment weights of this update (amm.jl:83-84), state-independent: off the critical path
    const int m1 = m + 1;
    const double p = (double)m1 / ((double)m1 + 1.0);
    const double q = 1.0 - p;
    const double cc = sc2 / p;
    // this iteration's draws (drawn one iteration ahead) to the whole quad
    double z1[3], z2[3];
    z1[0] = qbc<0>(n0); z2[0] = qbc<0>(n1);
    z1[1] = qbc<1>(n0); z2[1] = qbc<1>(n1);
    z1[2] = qbc<2>(n0); z2[2] = qbc<2>(n1);
    const double ua = qbc<3>(uown);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      z1[r] = r < d ? z1[r] : 0.0;
      z2[r] = r < d ? z2[r] : 0.0;
    }
    // the next iteration's draws: an independent instruction stream for the scheduler
    line_draw(A, chain, it + 1, lane, n0, n1, uown);
    MMB_PROF_MARK(1, lane)
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
    MMB_PROF_MARK(2, lane)
    // logf(x) on lane 0, logf(v) on lane 1 (the others repeat lane 1's), each on its own
    // relisted state -- which is also the state after the accept decision (relist(m, v))
    double xin[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) xin[r] = lane == 0 ? x[r] : v[r];
    ML::St sx = s;
    ML::relist(B, sx, g1, xin);
    const double lf = line_logf_st(A, B, sx);
    const double lx = qbc<0>(lf), lv = qbc<1>(lf);
    const bool acc = ua < mmb_exp(lx - lv);
    double vold[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      vold[r] = v[r];  // = unlist(m) of the state before this update
      v[r] = acc ? x[r] : v[r];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double a0 = qbc<0>(sx.v[r]), a1 = qbc<1>(sx.v[r]);
      s.v[r] = acc ? a0 : a1;
    }
    MMB_PROF_MARK(3, lane)
    if (adapt) {  // amm.jl:81-91
      m = m1;
      if (fl & 2) {
#pragma unroll
        for (int r = 0; r < 3; ++r) mv[r] = p * v[r] + q * v[r];
        fl &= ~2;
      } else {
#pragma unroll
        for (int r = 0; r < 3; ++r) mv[r] = p * mv[r] + q * v[r];
      }
      double Sg[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // Sigma (amm.jl:87), factorized in place
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
            Sg[t] = cc * (nv - mv[k] * mv[i]);
          }
        }
      }
      MMB_PROF_MARK(4, lane)
      double S0[6];
#pragma unroll
      for (int t = 0; t < 6; ++t) S0[t] = Sg[t];
      int pk[3] = {0, 0, 0};
      int rank;
      if (!pchol3_fast(d, Sg, pk, rank)) {  // rare: a pivot outside the in-range sqrt's domain
#pragma unroll
        for (int t = 0; t < 6; ++t) Sg[t] = S0[t];
        rank = pchol3(d, Sg, pk);
        st_redo += 1u;
      }
      st_fac += 1u;
      st_full += rank == d ? 1u : 0u;
      st_rank += (uint32_t)rank;
      st_steps += (uint32_t)(rank < d ? rank + 1 : d);
      if (rank == d) {
#pragma unroll
        for (int t = 0; t < 6; ++t)
          if (t < T) L[t] = Sg[t];
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (k < d) piv[k] = pk[k];
        fl |= 4;
      }
      MMB_PROF_MARK(5, lane)
    }
    // the next update's unlist(m) (the transform's log) -- independent of the factorization
    ML::unlist(B, s, 0, v);
    if (A.draws && it > A.burnin && (it - A.burnin) % A.thin == 0 && lane == 0) {
      const int64_t row = (it - A.burnin) / A.thin - 1 - A.kept_origin;
      ML::write_draws(A, s, g1, row, c);
    }
    MMB_PROF_MARK(6, lane)
  }
#ifdef MMB_PHASE_PROF
  if ((threadIdx.x & 63) == 0) {
    for (int i = 0; i < 16; ++i) atomicAdd(&mmb_prof_l[i], mmb_prof_lds()[i]);
  }
#endif
  if (lane == 0) {
    ML::store(A, c, 0, s);
    if (B.t_astat != nullptr && st_fac != 0u) {
      uint64_t* a = B.t_astat + (size_t)c * MMB_AMM_STAT_STRIDE;
      a[0] += st_fac;
      a[1] += st_full;
      a[2] += st_rank;
      a[3] += st_steps;
      a[4] += st_redo;
    }
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
