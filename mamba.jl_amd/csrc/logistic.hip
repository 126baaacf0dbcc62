// logistic.hip — NUTS on the logistic model with batched MFMA gradients (config 4).
//
// Step s of a window: lg_ctl_kernel(parity = s & 1) advances every chain's NUTS machine
// (nuts.h) to its next gradient request, appending the chain's leapfrog position to
// pos[slot] (slot = atomic counter; a chain's arithmetic does not depend on its slot);
// lg_grad_kernel(parity) evaluates, for all requested slots,
//   eta = X * B                      (N x 64)·(64 x slots), f64 MFMA 16x16x4
//   lp  = y .* eta - softplus(eta),  res = y - invlogit(eta)      (fused, registers; the
//         log(1 + exp(-|eta|)) terms as one product per lane and one log at the end)
//   G   = X' * res                   (64 x N)·(N x slots), f64 MFMA, D regs of the first
//                                    GEMM reused directly as B operands of the second
// as MMB_LG_NG x MMB_LG_NS sub-range partials; the next lg_ctl_kernel folds them per group and
// sums the groups in order (no atomics: the summation order is the mmb_math.h spec, restated
// by oracle/oracle.c).
#include "hmc.h"
#include "logistic.h"
#include "nuts.h"

typedef double mmb_d4 __attribute__((ext_vector_type(4)));

using NU = Nuts<64, 1>;
using LgFr = NutsFrames<64>;

__device__ __forceinline__ static void lg_load(const LgArgs& A, int c, int lane, NU::St& S) {
  const double* vb = A.vec + (size_t)c * MMB_LG_NVEC * 64 + lane;
  S.x[0] = vb[0 * 64]; S.r[0] = vb[1 * 64]; S.g[0] = vb[2 * 64];
  S.xm[0] = vb[3 * 64]; S.rm[0] = vb[4 * 64]; S.gm[0] = vb[5 * 64];
  S.xp[0] = vb[6 * 64]; S.rp[0] = vb[7 * 64]; S.gp[0] = vb[8 * 64];
  S.r0[0] = vb[9 * 64]; S.g0[0] = vb[10 * 64]; S.cxp[0] = vb[11 * 64];
  S.v[0] = A.vals[(size_t)c * 64 + lane];
  const double* s = A.sc + (size_t)c * MMB_LG_NSC;
  S.logp0 = s[0]; S.logu0 = s[1]; S.n = s[2]; S.cn = s[3]; S.calpha = s[4]; S.cnalpha = s[5];
  S.eps = s[6]; S.logf0 = s[7]; S.prob = s[8];
  const int32_t* iv = A.iv + (size_t)c * MMB_LG_NIV;
  S.pc = iv[0]; S.j = iv[1]; S.l = iv[2]; S.nxt = iv[3]; S.ku = iv[4]; S.pm = iv[5]; S.s = iv[6];
  S.cs = iv[7]; S.phases = iv[8]; S.eit = iv[9];
  const double* t = A.tune + (size_t)c * 8;
  S.t_eps = t[0]; S.t_epsbar = t[1]; S.t_Hbar = t[2]; S.t_mu = t[3]; S.t_alpha = t[4]; S.t_nalpha = t[5];
  S.t_m = A.tm[c];
  S.t_flags = A.tflags[c];
}

__device__ __forceinline__ static void lg_store(const LgArgs& A, int c, int lane, const NU::St& S, int slot,
                                                int64_t itc) {
  double* vb = A.vec + (size_t)c * MMB_LG_NVEC * 64 + lane;
  vb[0 * 64] = S.x[0]; vb[1 * 64] = S.r[0]; vb[2 * 64] = S.g[0];
  vb[3 * 64] = S.xm[0]; vb[4 * 64] = S.rm[0]; vb[5 * 64] = S.gm[0];
  vb[6 * 64] = S.xp[0]; vb[7 * 64] = S.rp[0]; vb[8 * 64] = S.gp[0];
  vb[9 * 64] = S.r0[0]; vb[10 * 64] = S.g0[0]; vb[11 * 64] = S.cxp[0];
  A.vals[(size_t)c * 64 + lane] = S.v[0];
  if (lane == 0) {
    double* s = A.sc + (size_t)c * MMB_LG_NSC;
    s[0] = S.logp0; s[1] = S.logu0; s[2] = S.n; s[3] = S.cn; s[4] = S.calpha; s[5] = S.cnalpha;
    s[6] = S.eps; s[7] = S.logf0; s[8] = S.prob;
    int32_t* iv = A.iv + (size_t)c * MMB_LG_NIV;
    iv[0] = S.pc; iv[1] = S.j; iv[2] = S.l; iv[3] = S.nxt; iv[4] = S.ku; iv[5] = S.pm; iv[6] = S.s;
    iv[7] = S.cs; iv[8] = S.phases; iv[9] = S.eit; iv[10] = slot;
    double* t = A.tune + (size_t)c * 8;
    t[0] = S.t_eps; t[1] = S.t_epsbar; t[2] = S.t_Hbar; t[3] = S.t_mu; t[4] = S.t_alpha; t[5] = S.t_nalpha;
    A.tm[c] = S.t_m;
    A.tflags[c] = S.t_flags;
    A.itc[c] = itc;
  }
}

// logpdf!(m, x, block) and its gradient at S.x from the range partials (oracle logf_grad):
// lf = 0 + prior, + sum of range partials if finite; grad = -x/sd^2 + partials, non-finite -> 0.
// FOLD: the gradient kernel ran one workgroup per group and already formed each group's
// ((P0 + P1) + ..) in unit slot group * MMB_LG_NS (lg_grad_kernel, fold mode); else the
// MMB_LG_NS sub-range partials are folded here in the same order.
template <bool FOLD, class ST>
__device__ __forceinline__ static void lg_assemble(const LgArgs& A, int slot, int lane, const Grp<64>& g, ST& S) {
  const bool el = lane < A.p;
  const double x = S.x[0];
  const double sd2 = A.prior_sd * A.prior_sd;
  double gg = el ? -x / sd2 : 0.0;
  // group sums added in group order: the summation spec of mmb_math.h.  Loads are issued 16
  // partials at a time ahead of the adds (fewer dependent round trips, bounded registers).
  constexpr int NW = FOLD ? 1 : MMB_LG_NS;  // partials read per group
  constexpr int LG_AB = 16 / NW;            // groups per batch of loads
  const double* gp = A.gpart + (size_t)slot * 64 + lane;
  for (int r0 = 0; r0 < MMB_LG_NG; r0 += LG_AB) {
    double gv[LG_AB * NW];
#pragma unroll
    for (int rg = 0; rg < LG_AB; ++rg)
#pragma unroll
      for (int w = 0; w < NW; ++w) gv[rg * NW + w] = gp[(size_t)((r0 + rg) * MMB_LG_NS + w) * A.K * 64];
#pragma unroll
    for (int rg = 0; rg < LG_AB; ++rg) {
      double gs = gv[rg * NW];
#pragma unroll
      for (int w = 1; w < NW; ++w) gs = gs + gv[rg * NW + w];
      gg = gg + gs;
    }
  }
  if (!isfinite(gg)) gg = 0.0;
  S.g[0] = el ? gg : 0.0;
  const bool bad = el && !isfinite(x);
  double sq = el ? 0.0 + x * x : 0.0;
  const double ssq = g.sum(sq);
  double lf = 0.0 + (__ballot(bad) ? -__builtin_inf() : d_iso(A.p, A.prior_sd, ssq));
  if (isfinite(lf)) {
    double ylp = 0.0;
    for (int r0 = 0; r0 < MMB_LG_NG; r0 += LG_AB) {
      double lv[LG_AB * NW];
#pragma unroll
      for (int rg = 0; rg < LG_AB; ++rg)
#pragma unroll
        for (int w = 0; w < NW; ++w) lv[rg * NW + w] = A.lpart[(size_t)((r0 + rg) * MMB_LG_NS + w) * A.K + slot];
#pragma unroll
      for (int rg = 0; rg < LG_AB; ++rg) {
        double ls = lv[rg * NW];
#pragma unroll
        for (int w = 1; w < NW; ++w) ls = ls + lv[rg * NW + w];
        ylp = ylp + ls;
      }
    }
    lf = lf + ylp;
  }
  S.lf = lf;
}

// logpdf!(m, x, block) and gradlogpdf!(m, x, block; dtype = :forward) at S.x (simulation.jl:47-51,
// oracle logf_grad): Calculus forward differences over the request's nv = p + 1 columns (column 0
// the position, column k its coordinate k - 1 moved by epsilon_{k-1} = 2^-26 max(1, |x|)), each
// column's logpdf! = 0 + prior (the 64-lane butterfly of squares, d_iso) + the group sums of its
// log-likelihood partials in group order when finite; lane e forms column e + 1 and the gradient
// entry (f_{e+1} - f_0) / epsilon_e, non-finite -> 0 (sampler.jl:110).
template <bool FOLD, class ST>
__device__ __forceinline__ static void lg_assemble_fd(const LgArgs& A, int slot, int lane, const Grp<64>& g,
                                                      ST& S) {
  const int p = A.p;
  const bool el = lane < p;
  const double x = S.x[0];
  const double ax = fabs(x);
  const double eps = 0x1p-26 * (isnan(ax) ? ax : (ax > 1.0 ? ax : 1.0));
  const double xp = x + eps;
  const double sq = el ? 0.0 + x * x : 0.0;
  const double sd = A.prior_sd;
  double f0 = 0.0 + (__ballot(el && !isfinite(x)) ? -__builtin_inf() : d_iso(p, sd, g.sum(sq)));
  double fk = 0.0;
  for (int e = 0; e < p; ++e) {  // column e + 1's prior: lane e's square replaced
    const double sqe = lane == e ? 0.0 + xp * xp : sq;
    const bool bad = __ballot(el && !isfinite(lane == e ? xp : x)) != 0;
    const double s = g.sum(sqe);
    const double pr = 0.0 + (bad ? -__builtin_inf() : d_iso(p, sd, s));
    fk = lane == e ? pr : fk;
  }
  constexpr int NW = FOLD ? 1 : MMB_LG_NS;  // partials read per group
  const int64_t c0 = (int64_t)slot * A.nv, ck = c0 + lane + 1;
  if (isfinite(f0)) {
    double ylp = 0.0;
    for (int r = 0; r < MMB_LG_NG; ++r) {
      double ls = A.lpart[(size_t)(r * MMB_LG_NS) * A.Kv + c0];
      for (int w = 1; w < NW; ++w) ls = ls + A.lpart[(size_t)(r * MMB_LG_NS + w) * A.Kv + c0];
      ylp = ylp + ls;
    }
    f0 = f0 + ylp;
  }
  if (el && isfinite(fk)) {
    double ylp = 0.0;
    for (int r = 0; r < MMB_LG_NG; ++r) {
      double ls = A.lpart[(size_t)(r * MMB_LG_NS) * A.Kv + ck];
      for (int w = 1; w < NW; ++w) ls = ls + A.lpart[(size_t)(r * MMB_LG_NS + w) * A.Kv + ck];
      ylp = ylp + ls;
    }
    fk = fk + ylp;
  }
  double gk = (fk - f0) / eps;
  if (!isfinite(gk)) gk = 0.0;
  S.g[0] = el ? gk : 0.0;
  S.lf = f0;
}

// The per-chain sampler machine driven by lg_ctl_kernel: NUTS (nuts.h) or HMC/MALA (hmc.h).
struct LgNuts {
  using St = NU::St;
  static constexpr int IDLE = NPC_IDLE;
  __device__ static bool wants(int pc) { return npc_wants_grad(pc); }
  __device__ static void load(const LgArgs& A, int c, int lane, St& S) { lg_load(A, c, lane, S); }
  __device__ static void store(const LgArgs& A, int c, int lane, const St& S, int slot, int64_t itc) {
    lg_store(A, c, lane, S, slot, itc);
  }
  __device__ static bool advance(const LgArgs& A, St& S, int c, uint32_t chain, int64_t cur, int lane,
                                 const Grp<64>& g) {
    NU::Env E;
    E.d = A.p;
    E.lane = lane;
    E.adapt = cur <= A.model_burnin;
    E.target = A.target;
    E.rn = mmb_rng_make(A.seed, chain, (uint32_t)cur, 0u, MMB_SUB_NORMAL);
    E.ru = mmb_rng_make(A.seed, chain, (uint32_t)cur, 0u, MMB_SUB_UNIFORM);
    E.ri = mmb_rng_make(A.seed, chain, (uint32_t)cur, 0u, MMB_SUB_INIT);
    E.F = A.frames + (size_t)c * LgFr::DBL;
    E.stat = A.nstat;
    return NU::advance(S, E, g);
  }
};

using HM = Hmc<64, 1>;
// HMC/MALA state: x = vec[0], p = vec[1], logf0 = sc[0], k0 = sc[1], pc = iv[0], i = iv[1];
// the gradient is always fresh when a machine resumes, so g is never stored.
template <bool MALA>
struct LgHmc {
  using St = HM::St;
  static constexpr int IDLE = HPC_DONE + 1;
  __device__ static bool wants(int pc) { return pc == HPC_G0 || pc == HPC_STEP || pc == HPC_MG1; }
  __device__ static void load(const LgArgs& A, int c, int lane, St& S) {
    const double* vb = A.vec + (size_t)c * MMB_LG_NVEC * 64 + lane;
    S.x[0] = vb[0];
    S.p[0] = vb[64];
    S.g[0] = 0.0;
    S.v[0] = A.vals[(size_t)c * 64 + lane];
    const double* sc = A.sc + (size_t)c * MMB_LG_NSC;
    S.logf0 = sc[0];
    S.k0 = sc[1];
    const int32_t* iv = A.iv + (size_t)c * MMB_LG_NIV;
    S.pc = iv[0];
    S.i = iv[1];
  }
  __device__ static void store(const LgArgs& A, int c, int lane, const St& S, int slot, int64_t itc) {
    double* vb = A.vec + (size_t)c * MMB_LG_NVEC * 64 + lane;
    vb[0] = S.x[0];
    vb[64] = S.p[0];
    A.vals[(size_t)c * 64 + lane] = S.v[0];
    if (lane == 0) {
      double* sc = A.sc + (size_t)c * MMB_LG_NSC;
      sc[0] = S.logf0;
      sc[1] = S.k0;
      int32_t* iv = A.iv + (size_t)c * MMB_LG_NIV;
      iv[0] = S.pc;
      iv[1] = S.i;
      iv[10] = slot;
      A.itc[c] = itc;
    }
  }
  __device__ static bool advance(const LgArgs& A, St& S, int c, uint32_t chain, int64_t cur, int lane,
                                 const Grp<64>& g) {
    HM::Env E;
    E.d = A.p;
    E.lane = lane;
    E.eps = A.tune[(size_t)c * 2];
    E.L = (int)A.tune[(size_t)c * 2 + 1];
    E.sigl = A.sigl;
    E.rn = mmb_rng_make(A.seed, chain, (uint32_t)cur, 0u, MMB_SUB_NORMAL);
    E.ru = mmb_rng_make(A.seed, chain, (uint32_t)cur, 0u, MMB_SUB_UNIFORM);
    return MALA ? HM::advance_mala(S, E, g) : HM::advance_hmc(S, E, g);
  }
};

#ifndef MMB_LG_CTL_WAVES
#define MMB_LG_CTL_WAVES 1
#endif
template <class MC>
__global__ __launch_bounds__(256, MMB_LG_CTL_WAVES) void lg_ctl_kernel(const LgArgs A, int start, int parity, int fold) {
  // the first step visits every chain; later steps visit the chains that requested the
  // gradient just computed (slot order of the previous control kernel), so the grid and the
  // work shrink with the running chains at the end of a window
  const int si = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
  int c;
  if (start) {
    if (si >= A.K) return;
    c = si;
  } else {
    if (si >= A.count[parity ^ 1]) return;
    c = A.s2c[(size_t)(parity ^ 1) * A.K + si];
  }
  Grp<64> g;
  const int lane = g.lane;
  typename MC::St S;
  MC::load(A, c, lane, S);
  int64_t itc = A.itc[c];
  if (start) {
    S.pc = 0;  // NPC_BEGIN / HPC_BEGIN
    itc = A.iter0;
  }
  if (S.pc == MC::IDLE) return;
  if (MC::wants(S.pc)) {
    // the chain's gradient slot is its index in the request list (slot assignment below)
    const int slot = start ? A.iv[(size_t)c * MMB_LG_NIV + 10] : si;
    if (A.fd) {
      if (fold) lg_assemble_fd<true>(A, slot, lane, g, S);
      else lg_assemble_fd<false>(A, slot, lane, g, S);
    } else {
      if (fold) lg_assemble<true>(A, slot, lane, g, S);
      else lg_assemble<false>(A, slot, lane, g, S);
    }
  }
  const uint32_t chain = A.chain_offset + (uint32_t)c;
  for (;;) {
    const int64_t cur = itc + 1;
    if (MC::advance(A, S, c, chain, cur, lane, g)) {
      int slot = 0;
      if (lane == 0) {
        slot = atomicAdd(&A.count[parity], 1);
        A.s2c[(size_t)parity * A.K + slot] = c;
      }
      slot = __shfl(slot, 0, 64);
      A.pos[(size_t)slot * 64 + lane] = S.x[0];
      MC::store(A, c, lane, S, slot, itc);
      return;
    }
    itc = cur;  // mcmc_worker! keep rule (mcmc.jl:76): sim[i,:,1] = unlist(m, true)
    if (A.draws && itc > A.burnin && (itc - A.burnin) % A.thin == 0 && lane < A.p) {
      const int64_t row = (itc - A.burnin) / A.thin - 1 - A.kept_origin;
      A.draws[(size_t)(row * A.p + lane) * A.Kd + c] = S.v[0];
    }
    if (itc >= A.it_end) {
      S.pc = MC::IDLE;
      MC::store(A, c, lane, S, 0, itc);
      return;
    }
    S.pc = 0;
  }
}

// 1-D grid of MMB_LG_NG * MMB_LG_NS * ceil(K/64) workgroups of 4 waves.  Workgroup -> (unit un =
// group * MMB_LG_NS + sub-range, 64-chain tile ct): blocks are dealt round-robin over the 8 XCDs,
// so XCD x gets units 8x .. 8x+7 (groups 4x .. 4x+3) only and its L2 holds just those rows of X;
// tiles ascend with the block id, so the blocks beyond the active count (the end of a window)
// are the last dispatched and exit at once.  One sub-range per workgroup: a step's latency is
// one sub-range's passes (most steps at the end of a window carry few chains), and the ctl
// kernel folds the MMB_LG_NS partials of a group as ((P0 + P1) + P2) + .. (the spec).
// Wave w owns chains ct*64 + 16w .. +15 (lane l: chain column l & 15, k-group l >> 4) and walks
// its sub-range's 32-row passes in order, accumulating in
// registers (the summation spec the oracle restates).  The workgroup stages each 32-row
// pass of X once in LDS for all 4 waves (4x fewer L2 reads per MFMA than per-wave loads,
// which were the bottleneck: a 16x16x4 f64 MFMA issues every 64 cycles per SIMD and needs
// its 512-B A operand; measured tools/mfma_f64_probe.hip), prefetching the next pass into
// registers while the current one is computed.
// LDS row stride 66 doubles: the first GEMM's A reads (16 rows x 4 k-groups) hit 32
// distinct bank pairs per half-wave; the second GEMM's reads are at most 2-way.
#ifndef MMB_LG_WAVES
#define MMB_LG_WAVES 2
#endif
#define LG_RB 32   // rows per staged pass (two 16-row MFMA blocks)
#define LG_LD 66   // padded LDS row stride (doubles)
#define LG_PER (LG_RB * 64 / 256)  // doubles of a pass staged per thread
// KS: MFMA k-steps of eta = X*B, ceil(p/4) rounded to 13 (p <= 52) or 16 (p <= MMB_LG_DV); the padded
// coefficients are zero in X and in the positions, so both give the same sequential fma chain.
// FOLD (wide steps, engine.cpp): one workgroup per (group, tile) walks the group's MMB_LG_NS
// sub-ranges one after the other -- each its own fma chain from zero, as in the one-unit mode --
// and writes the group's ((P0 + P1) + ..) to unit slot group * MMB_LG_NS: half the partials
// written here and read by the control kernel, the same bits.
// LPONLY (forward differences): column v = request slot * nv + k is the request's position with
// coordinate k - 1 moved by Calculus' epsilon (k = 0: unmoved), formed here from the position in
// the same operation as the oracle (x + eps); only the log-density partials are written.
template <int KS, bool FOLD, bool LPONLY>
__global__ __launch_bounds__(256, MMB_LG_WAVES) void lg_grad_kernel(const LgArgs A, int parity) {
  __shared__ __attribute__((aligned(16))) double xs[LG_RB][LG_LD];
  __shared__ double ys[LG_RB];
  const int nreq = A.count[parity];
  const int nact = nreq * A.nv;  // columns
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (nreq > 0) atomicAdd(A.ngrad, (unsigned long long)nreq);
    A.count[parity ^ 1] = 0;  // the next control kernel's counter (its input list was read before)
  }
  const int b = (int)blockIdx.x;
  constexpr int NW = FOLD ? MMB_LG_NS : 1;                 // sub-ranges per workgroup
  constexpr int UPX = MMB_LG_NG * MMB_LG_NS / (8 * NW);   // work units per XCD
  const int idx = b >> 3;
  const int un0 = (UPX * (b & 7) + idx % UPX) * NW;        // first sub-range: gi * MMB_LG_NS (+ w)
  const int ct = idx / UPX;
  if (ct * 64 >= nact) return;  // uniform over the workgroup
  const int tid = (int)threadIdx.x;
  const int w = tid >> 6;
  const int l = tid & 63;
  const int lc = l & 15, lq = l >> 4;
  const int slot = ct * 64 + w * 16 + lc;
  const bool live = slot < nact;
  double bpos[KS];
  const int rs = LPONLY ? slot / A.nv : slot, kcol = LPONLY ? slot - rs * A.nv : 0;
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    double b = live ? A.pos[(size_t)rs * 64 + 4 * kk + lq] : 0.0;
    if (LPONLY && 4 * kk + lq == kcol - 1) {  // oracle logf_grad: xx[k] = x[k] + eps
      const double ax = fabs(b);
      b = b + 0x1p-26 * (isnan(ax) ? ax : (ax > 1.0 ? ax : 1.0));
    }
    bpos[kk] = b;
  }
  mmb_d4 tot[4], acc[4];
  double ltot = 0.0;
  const int rps = A.rps;
  const int npass = (rps + LG_RB - 1) / LG_RB;
  // staging map: thread tid moves X[r0 + e*8 + (tid >> 3)... ] -- 8 consecutive doubles of one row
  const int srow = tid >> 3, scol = (tid & 7) * 8;  // 32 rows x 8 segments of 8 doubles
  double pf[LG_PER];
  double pfy = 0.0;
  auto fetch = [&](int r0, int nrows) {
    const double* src = A.X + (size_t)(r0 + srow) * 64 + scol;
#pragma unroll
    for (int e = 0; e < LG_PER; e += 2) {
      const double2 v = srow < nrows ? *(const double2*)(src + e) : make_double2(0.0, 0.0);
      pf[e] = v.x;
      pf[e + 1] = v.y;
    }
    pfy = tid < nrows ? A.y[r0 + tid] : 0.0;
  };
  fetch(un0 * rps, rps < LG_RB ? rps : LG_RB);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) acc[mt] = mmb_d4{0.0, 0.0, 0.0, 0.0};
  double lsum = 0.0, lprod = 1.0;
  int lexp = 0;
  for (int q = 0; q < NW * npass; ++q) {
    const int sw = NW == 1 ? 0 : q / npass, ps = NW == 1 ? q : q % npass;
    const int r0 = (un0 + sw) * rps + ps * LG_RB;
    const int nrows = rps - ps * LG_RB < LG_RB ? rps - ps * LG_RB : LG_RB;  // 16 or 32
    __syncthreads();  // previous pass's LDS reads are done
#pragma unroll
    for (int e = 0; e < LG_PER; e += 2) *(double2*)&xs[srow][scol + e] = make_double2(pf[e], pf[e + 1]);
    if (tid < LG_RB) ys[tid] = pfy;
    __syncthreads();
    if (q + 1 < NW * npass) {  // prefetch the next pass (or the next sub-range's first) while this one computes
      const int sw1 = NW == 1 ? 0 : (q + 1) / npass, ps1 = NW == 1 ? q + 1 : (q + 1) % npass;
      int nn = rps - ps1 * LG_RB;
      if (nn > LG_RB) nn = LG_RB;
      fetch((un0 + sw1) * rps + ps1 * LG_RB, nn);
    }
    const bool two = nrows > 16;
    mmb_d4 eta0 = mmb_d4{0.0, 0.0, 0.0, 0.0}, eta1 = eta0;
    if (two) {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        eta0 = __builtin_amdgcn_mfma_f64_16x16x4f64(xs[lc][4 * kk + lq], bpos[kk], eta0, 0, 0, 0);
        eta1 = __builtin_amdgcn_mfma_f64_16x16x4f64(xs[16 + lc][4 * kk + lq], bpos[kk], eta1, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
        eta0 = __builtin_amdgcn_mfma_f64_16x16x4f64(xs[lc][4 * kk + lq], bpos[kk], eta0, 0, 0, 0);
    }
    // residual terms of both blocks first (branch-free), so the scheduler can overlap block 1's
    // VALU work with block 0's X'*res MFMAs; the lane's lin sum and (1 + t) product keep the
    // row order of the spec (mmb_math.h mmb_logistic_row)
    double sres[2][4], lins[2][4], fac[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const mmb_d4 eta = h ? eta1 : eta0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = r0 + 16 * h + lq + 4 * i;
        double lin, a, res;
        mmb_logistic_row(eta[i], ys[16 * h + lq + 4 * i], &lin, &a, &res);
        // padded rows (>= N, or the empty second block of a 16-row pass) have X = 0 and
        // y = 0, so eta = 0, lin = +0 and X' res adds exact zeros: only the factor is masked
        const bool in = row < A.N && (h == 0 || two);
        lins[h][i] = lin;
        fac[h][i] = in ? a : 1.0;
        sres[h][i] = res;
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lsum = lsum + lins[h][i];
        lprod = lprod * fac[h][i];
      }
      if (h == 1 && !two) break;
      if constexpr (!LPONLY) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            acc[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(xs[16 * h + 4 * i + lq][16 * mt + lc], sres[h][i],
                                                           acc[mt], 0, 0, 0);
      }
    }
    mmb_lg_renorm(&lprod, &lexp);  // < 2^9 before: never overflows
    if (ps == npass - 1) {  // end of a sub-range: its partials, folded into the group's in order
      lsum = mmb_lg_lane_lp(lsum, lprod, lexp);
      lsum = lsum + __shfl_xor(lsum, 16, 64);
      lsum = lsum + __shfl_xor(lsum, 32, 64);
      if (sw == 0) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) tot[mt] = acc[mt];
        ltot = lsum;
      } else {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) tot[mt] = tot[mt] + acc[mt];
        ltot = ltot + lsum;
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = mmb_d4{0.0, 0.0, 0.0, 0.0};
      lsum = 0.0;
      lprod = 1.0;
      lexp = 0;
    }
  }
  if (!live) return;
  if constexpr (!LPONLY) {
    // coefficient 16 mt + lq + 4 q of chain lc
    double* gp = A.gpart + ((size_t)un0 * A.K + slot) * 64;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) gp[16 * mt + lq + 4 * qq] = tot[mt][qq];
  }
  if (lq == 0) A.lpart[(size_t)un0 * A.Kv + slot] = ltot;
}

// nbound: an upper bound of the chains still running (the host's last read of the request
// count; requests never increase within a window).  fold: the gradient kernel ran (or will run)
// in group mode; the control kernel that consumes its partials gets the same flag.
hipError_t mmb_lg_launch_ctl(const LgArgs& A, int start, int parity, int nbound, int fold, hipStream_t st) {
  const dim3 grid(((start ? A.K : nbound) + 3) / 4), blk(256);
  if (A.kind == MMB_SAMPLER_HMC)
    hipLaunchKernelGGL(lg_ctl_kernel<LgHmc<false>>, grid, blk, 0, st, A, start, parity, fold);
  else if (A.kind == MMB_SAMPLER_MALA)
    hipLaunchKernelGGL(lg_ctl_kernel<LgHmc<true>>, grid, blk, 0, st, A, start, parity, fold);
  else
    hipLaunchKernelGGL(lg_ctl_kernel<LgNuts>, grid, blk, 0, st, A, start, parity, fold);
  return hipGetLastError();
}
template <bool LPONLY>
static void launch_grad(const LgArgs& A, int parity, int fold, dim3 grid, hipStream_t st) {
  const dim3 blk(256);
  if (A.p <= 52) {
    if (fold) hipLaunchKernelGGL((lg_grad_kernel<13, true, LPONLY>), grid, blk, 0, st, A, parity);
    else hipLaunchKernelGGL((lg_grad_kernel<13, false, LPONLY>), grid, blk, 0, st, A, parity);
  } else {
    if (fold) hipLaunchKernelGGL((lg_grad_kernel<16, true, LPONLY>), grid, blk, 0, st, A, parity);
    else hipLaunchKernelGGL((lg_grad_kernel<16, false, LPONLY>), grid, blk, 0, st, A, parity);
  }
}
// nbound: requests (chains); the grid covers their nbound * nv columns
hipError_t mmb_lg_launch_grad(const LgArgs& A, int parity, int nbound, int fold, hipStream_t st) {
  const int tiles = (int)(((int64_t)nbound * A.nv + 63) / 64);
  const dim3 grid((fold ? MMB_LG_NG : MMB_LG_NG * MMB_LG_NS) * tiles);
  if (A.fd) launch_grad<true>(A, parity, fold, grid, st);
  else launch_grad<false>(A, parity, fold, grid, st);
  return hipGetLastError();
}
