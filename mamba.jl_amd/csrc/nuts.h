// nuts.h — No-U-Turn sampler (src/samplers/nuts.jl:63-205) as a resumable state machine.
//
// The reference builds the trajectory with the recursive buildtree (nuts.jl:139-180).  On
// the GPU every chain is at a different point of its own tree, and for the logistic model
// each gradient is one column of a batched MFMA GEMM over all chains, so the recursion is
// unrolled into an explicit machine that *suspends at every gradient request*:
// advance() runs until it needs logf/grad at x (returns true; the caller fills lf and g and
// calls advance() again) or until the update is complete (returns false).  With an inline
// gradient (line) the caller simply loops.
//
// Recursion -> iteration.  A tree of depth J built in direction pm is a complete binary
// tree over leaf indices 0..2^J-1.  Levels 1..J hold one frame each: the first half of the
// level's current subtree (xprime, n, alpha, nalpha) while its second half is being built.
//   * leaf done, level l, parent frame empty: it is the parent's first half; if its s is
//     true push it and build the second half from the frontier (the newest leaf), else the
//     parent returns it unchanged and its 2^l second-half leaves are skipped;
//   * parent frame full: merge exactly as nuts.jl:160-176 (one uniform draw,
//     xprime choice, n, alpha, nalpha, s = s2 && nouturn(first leaf, newest leaf)).
// The first leaf of the subtree starting at leaf index b is kept in slot ctz(b) (slot J
// for b = 0): no two live subtrees share a slot, so merges read it without copies.
// Draw order (Appendix A.2): d normals for r, 1 uniform for logu0, per doubling 1 uniform
// for the direction, 1 uniform per merge (only when the first half's s is true), 1 top-level
// uniform only if T.s (the `&&` short-circuit of nuts.jl:117).  nutsepsilon (nuts.jl:192-205)
// consumes d normals of the INIT substream at the first update.  The reference's doubling
// loop is unbounded (nuts.jl:106-125); here depth stops at MMB_NUTS_MAX_DEPTH = 30, the
// largest tree the int32 leaf index / level mask address (2^30 leapfrogs in one update, ~10^9
// gradients: no run that finishes reaches it), identically in oracle/oracle.c.  The frames
// are in HBM (31 slots x 3 vectors per chain), so the depth costs memory, not registers.
// Every update that reaches the cap with the trajectory still growing is counted
// (Env::stat[1], mmb_nuts_stats), so a run shows whether the cap ever acted.
#pragma once
#include "device.h"

#ifndef MMB_NUTS_MAX_DEPTH
#define MMB_NUTS_MAX_DEPTH 30
#endif
#define MMB_NUTS_NSLOT (MMB_NUTS_MAX_DEPTH + 1)

enum : int32_t {
  NPC_BEGIN = 0, NPC_EPS0, NPC_EPS12, NPC_SUB, NPC_SUB0, NPC_DOUBLE, NPC_LEAF, NPC_LEAF1,
  NPC_UP, NPC_TREE, NPC_DONE, NPC_IDLE
};
// pc values at which advance() resumes after a gradient
__host__ __device__ inline bool npc_wants_grad(int pc) {
  return pc == NPC_EPS0 || pc == NPC_EPS12 || pc == NPC_SUB0 || pc == NPC_LEAF1;
}

// Frame storage per chain (global memory): slot q in [0, NSLOT): x, r, xprime vectors of
// length DV, then NSLOT x 4 scalars (n, alpha, nalpha, -).
template <int DV>
struct NutsFrames {
  static constexpr int DBL = MMB_NUTS_NSLOT * 3 * DV + MMB_NUTS_NSLOT * 4;
  __device__ __forceinline__ static double* fx(double* F, int q) { return F + (q * 3 + 0) * DV; }
  __device__ __forceinline__ static double* fr(double* F, int q) { return F + (q * 3 + 1) * DV; }
  __device__ __forceinline__ static double* fxp(double* F, int q) { return F + (q * 3 + 2) * DV; }
  __device__ __forceinline__ static double* fs(double* F, int q) { return F + MMB_NUTS_NSLOT * 3 * DV + q * 4; }
};

// Machine state.  Vectors: element e in lane e % G, slot e / G.
template <int G, int R>
struct NutsM {
  double v[R], x[R], r[R], g[R], xm[R], rm[R], gm[R], xp[R], rp[R], gp[R], r0[R], g0[R], cxp[R];
  double lf;                                       // logf at x (filled by the gradient provider)
  double logp0, logu0, n, cn, calpha, cnalpha, eps, logf0, prob;
  double t_eps, t_epsbar, t_Hbar, t_mu, t_alpha, t_nalpha;  // NUTSTune (nuts.jl:5-39)
  int32_t pc, j, l, nxt, ku, pm, s, cs, phases, eit, t_m, t_flags;  // t_flags bit0 adapt, bit3 init
};

template <int G, int R>
struct Nuts {
  static constexpr int DV = G * R;
  using St = NutsM<G, R>;
  using Fr = NutsFrames<DV>;

  struct Env {
    int d;
    int lane;
    bool adapt;        // iter <= burnin (nuts.jl:52)
    double target;
    mmb_rng rn, ru, ri;
    double* F;         // this chain's frames
    unsigned long long* stat;  // null or {updates, depth-cap hits, sum of tree depths}
  };

  // dot1 / nouturn of oracle.c: sequential (mul then add) within a lane, then the group sum
  __device__ __forceinline__ static double dot(const Grp<G>& g, const double* a, const double* b, int d) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r * G + g.lane < d) s = s + a[r] * b[r];
    return G == 1 ? s : g.sum(s);
  }
  __device__ __forceinline__ static bool nouturn(const Grp<G>& g, const double* xm, const double* xp,
                                                 const double* rm, const double* rp, int d) {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r * G + g.lane < d) { double xd = xp[r] - xm[r]; a = a + xd * rm[r]; }
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r * G + g.lane < d) { double xd = xp[r] - xm[r]; b = b + xd * rp[r]; }
    if (G > 1) g.sum2(a, b);
    return a >= 0.0 && b >= 0.0;
  }
  // first half of leapfrog (nuts.jl:129-136): r += (eps/2) grad; x += eps r
  __device__ __forceinline__ static void leap_a(St& S, double e) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      S.r[r] = S.r[r] + (0.5 * e) * S.g[r];
      S.x[r] = S.x[r] + e * S.r[r];
    }
  }
  __device__ __forceinline__ static void leap_b(St& S, double e) {
#pragma unroll
    for (int r = 0; r < R; ++r) S.r[r] = S.r[r] + (0.5 * e) * S.g[r];
  }
  __device__ __forceinline__ static void cpy(double* a, const double* b) {
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = b[r];
  }

  __device__ static bool advance(St& S, const Env& E, const Grp<G>& g) {
    const int d = E.d;
    for (;;) {
      switch (S.pc) {
        case NPC_BEGIN: {
          if (!(S.t_flags & 8)) {  // NUTSTune(x, nutsepsilon(x, logfgrad)): nuts.jl:22-33,192-205
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const int e = r * G + g.lane;
              S.r0[r] = e < d ? mmb_normal(&E.ri, (uint32_t)e) : 0.0;
              S.g0[r] = 0.0;
              S.x[r] = S.v[r];
              S.r0[r] = S.r0[r] + (0.5 * 0.0) * S.g0[r];  // leapfrog(x, r0, g0, 0.0)
              S.x[r] = S.x[r] + 0.0 * S.r0[r];
            }
            S.pc = NPC_EPS0;
            return true;
          }
          S.pc = NPC_SUB;
          continue;
        }
        case NPC_EPS0: {
          S.logf0 = S.lf;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            S.g0[r] = S.g[r];
            S.r0[r] = S.r0[r] + (0.5 * 0.0) * S.g0[r];
            S.x[r] = S.v[r];
            S.r[r] = S.r0[r];
          }
          S.eps = 1.0;
          S.eit = -1;
          leap_a(S, S.eps);
          S.pc = NPC_EPS12;
          return true;
        }
        case NPC_EPS12: {
          leap_b(S, S.eps);
          S.prob = mmb_exp(S.lf - S.logf0 - 0.5 * (dot(g, S.r, S.r, d) - dot(g, S.r0, S.r0, d)));
          if (S.eit < 0) S.pm = (S.prob > 0.5) ? 1 : -1;
          S.eit += 1;
          if (S.eit < 4000) {
            const double lhs = S.pm == 1 ? S.prob : 1.0 / S.prob;
            const double rhs = S.pm == 1 ? 0.5 : 2.0;
            if (lhs > rhs) {
              S.eps *= S.pm == 1 ? 2.0 : 0.5;
#pragma unroll
              for (int r = 0; r < R; ++r) { S.x[r] = S.v[r]; S.r[r] = S.r0[r]; S.g[r] = S.g0[r]; }
              leap_a(S, S.eps);
              return true;  // pc stays NPC_EPS12
            }
          }
          S.t_eps = S.eps; S.t_epsbar = 1.0; S.t_Hbar = 0.0; S.t_mu = __builtin_nan("");
          S.t_alpha = 0.0; S.t_nalpha = 0.0; S.t_m = 0;
          S.t_flags = (S.t_flags & ~1) | 8;
          S.pc = NPC_SUB;
          continue;
        }
        case NPC_SUB: {  // sample!(v::NUTSVariate) / setadapt! (nuts.jl:63-92)
          if (E.adapt && !(S.t_flags & 1)) { S.t_m = 0; S.t_mu = mmb_log(10.0 * S.t_eps); }
          S.t_flags = E.adapt ? (S.t_flags | 1) : (S.t_flags & ~1);
          if (E.adapt) S.t_m += 1;
          else if (S.t_m > 0) S.t_eps = S.t_epsbar;
          S.eps = S.t_eps;
          S.ku = 0;  // nuts_sub! (nuts.jl:95-126)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int e = r * G + g.lane;
            S.x[r] = S.v[r];
            S.r[r] = e < d ? mmb_normal(&E.rn, (uint32_t)e) : 0.0;
            S.g[r] = 0.0;
          }
          leap_a(S, 0.0);
          S.pc = NPC_SUB0;
          return true;
        }
        case NPC_SUB0: {
          leap_b(S, 0.0);
          S.logp0 = S.lf - 0.5 * dot(g, S.r, S.r, d);
          S.logu0 = S.logp0 + mmb_log(mmb_uniform(&E.ru, (uint32_t)S.ku++));
          cpy(S.xm, S.x); cpy(S.xp, S.x); cpy(S.rm, S.r); cpy(S.rp, S.r); cpy(S.gm, S.g); cpy(S.gp, S.g);
          S.j = 0;
          S.n = 1.0;
          S.s = 1;
          S.pc = NPC_DOUBLE;
          continue;
        }
        case NPC_DOUBLE: {
          if (!S.s) {
            if (S.t_flags & 1) {  // dual averaging (nuts.jl:66-75)
              const double m = (double)S.t_m;
              double p = 1.0 / (m + 10.0);
              S.t_Hbar = (1.0 - p) * S.t_Hbar + p * (E.target - S.t_alpha / S.t_nalpha);
              S.t_eps = mmb_exp(S.t_mu - sqrt(m) * S.t_Hbar / 0.05);
              p = mmb_exp(-0.75 * mmb_log(m));
              S.t_epsbar = mmb_exp(p * mmb_log(S.t_eps) + (1.0 - p) * mmb_log(S.t_epsbar));
            }
            if (E.stat && E.lane == 0) {
              atomicAdd(&E.stat[0], 1ull);
              atomicAdd(&E.stat[2], (unsigned long long)S.j);
            }
            S.pc = NPC_DONE;
            return false;
          }
          S.pm = (mmb_uniform(&E.ru, (uint32_t)S.ku++) > 0.5) ? 1 : -1;
          if (S.pm == -1) { cpy(S.x, S.xm); cpy(S.r, S.rm); cpy(S.g, S.gm); }
          else { cpy(S.x, S.xp); cpy(S.r, S.rp); cpy(S.g, S.gp); }
          S.nxt = 0;
          S.phases = 0;
          S.pc = NPC_LEAF;
          continue;
        }
        case NPC_LEAF: {
          leap_a(S, (double)S.pm * S.eps);
          S.pc = NPC_LEAF1;
          return true;
        }
        case NPC_LEAF1: {  // buildtree, j == 0 (nuts.jl:142-152)
          leap_b(S, (double)S.pm * S.eps);
          const double logpp = S.lf - 0.5 * dot(g, S.r, S.r, d);
          S.cn = (S.logu0 < logpp) ? 1.0 : 0.0;
          S.cs = S.logu0 < logpp + 1000.0;
          S.calpha = jmin(1.0, mmb_exp(logpp - S.logp0));
          S.cnalpha = 1.0;
          cpy(S.cxp, S.x);
          const int i = S.nxt;
          const int slot = i == 0 ? S.j : __builtin_ctz((unsigned)i);
          if (slot >= 1) {
            double* fx = Fr::fx(E.F, slot);
            double* fr = Fr::fr(E.F, slot);
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const int e = r * G + g.lane;
              fx[e] = S.x[r];
              fr[e] = S.r[r];
            }
          }
          S.nxt = i + 1;
          S.l = 0;
          S.pc = NPC_UP;
          continue;
        }
        case NPC_UP: {
          if (S.l == S.j) { S.pc = NPC_TREE; continue; }
          const int lv = S.l + 1;
          if (!((S.phases >> lv) & 1)) {  // current subtree is the first half of level lv
            if (S.cs) {
              double* fxp = Fr::fxp(E.F, lv);
#pragma unroll
              for (int r = 0; r < R; ++r) fxp[r * G + g.lane] = S.cxp[r];
              if (g.lane == 0) {
                double* fs = Fr::fs(E.F, lv);
                fs[0] = S.cn; fs[1] = S.calpha; fs[2] = S.cnalpha;
              }
              S.phases |= 1 << lv;
              S.pc = NPC_LEAF;
              continue;
            }
            S.nxt += 1 << S.l;  // the parent returns its first half; second half skipped
            S.l = lv;
            continue;
          }
          // second half done: merge into the parent (nuts.jl:160-176)
          const double* fs = Fr::fs(E.F, lv);
          double Tn = fs[0], Ta = fs[1], Tna = fs[2];
          const double* fxp = Fr::fxp(E.F, lv);
          double txp[R];
#pragma unroll
          for (int r = 0; r < R; ++r) txp[r] = fxp[r * G + g.lane];
          if (mmb_uniform(&E.ru, (uint32_t)S.ku++) < S.cn / (Tn + S.cn)) cpy(txp, S.cxp);
          Tn += S.cn;
          bool ts = false;
          if (S.cs) {
            const int base = S.nxt - (2 << S.l);
            const int slot = base == 0 ? S.j : __builtin_ctz((unsigned)base);
            const double* fx = Fr::fx(E.F, slot);
            const double* fr = Fr::fr(E.F, slot);
            double ax[R], ar[R];
#pragma unroll
            for (int r = 0; r < R; ++r) { ax[r] = fx[r * G + g.lane]; ar[r] = fr[r * G + g.lane]; }
            ts = S.pm == 1 ? nouturn(g, ax, S.x, ar, S.r, d) : nouturn(g, S.x, ax, S.r, ar, d);
          }
          Ta += S.calpha;
          Tna += S.cnalpha;
          cpy(S.cxp, txp);
          S.cn = Tn; S.cs = ts; S.calpha = Ta; S.cnalpha = Tna;
          S.phases &= ~(1 << lv);
          S.l = lv;
          continue;
        }
        case NPC_TREE: {  // back in nuts_sub! (nuts.jl:105-124)
          if (S.pm == -1) { cpy(S.xm, S.x); cpy(S.rm, S.r); cpy(S.gm, S.g); }
          else { cpy(S.xp, S.x); cpy(S.rp, S.r); cpy(S.gp, S.g); }
          if (S.cs && mmb_uniform(&E.ru, (uint32_t)S.ku++) < S.cn / S.n) cpy(S.v, S.cxp);
          S.j += 1;
          S.n += S.cn;
          S.s = S.cs && nouturn(g, S.xm, S.xp, S.rm, S.rp, d);
          S.t_alpha = S.calpha;
          S.t_nalpha = S.cnalpha;
          if (S.j >= MMB_NUTS_MAX_DEPTH && S.s) {  // the reference would keep doubling
            if (E.stat && E.lane == 0) atomicAdd(&E.stat[1], 1ull);
            S.s = 0;
          }
          S.pc = NPC_DOUBLE;
          continue;
        }
        default:
          return false;
      }
    }
  }
};
