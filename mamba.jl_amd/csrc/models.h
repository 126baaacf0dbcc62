// models.h — lowered model kernels: per-chain state, unlist/relist, block logpdf!,
// conjugate Gibbs draws.  One specialisation per model kind.
//
// logf() restates logpdf!(m, x, block, transform) (src/model/simulation.jl:77-90):
// params \ targets in block order with early exit on a non-finite sum, then the
// block's targets in topological order; node densities per
// src/distributions/distributionstruct.jl:136-168 and transformdistribution.jl:53-78.
#pragma once
#include "device.h"

template <int MODEL>
struct Mdl;

// ------------------------------------------------------------------ rats
// doc/examples/rats.jl:48-97.  Device value layout per chain (72 doubles):
//   [0,32) alpha (30 + pad) | [32,64) beta | 64 s2_c | 65 mu_alpha | 66 s2_alpha |
//   67 mu_beta | 68 s2_beta.
// Group = 32 lanes, two chains per wave: rat e <-> lane e (register slot R = 1; the model code
// is written for R rats per lane).  A 16-lane, two-rats-per-lane layout (four chains per wave,
// half the instructions per chain in each pivoted-Cholesky step) was measured at 0.318 vs
// 0.220 ms per sweep: LDS caps both layouts at 32 chains per CU and the factorization is
// latency-bound, so 4 waves of 2 chains beat 2 waves of 4.
template <>
struct Mdl<MMB_MODEL_RATS> {
  static constexpr int G = 32, R = 1, DMAX = 30, DP = 32, TP = 480, VS = 72, PMON = 3;
  static constexpr int LDS_DBL = TP + 4 * DP;  // matrix + 4 vectors (the stash reuses idle ones)
  struct St { double a[R], b[R]; double s2c, mua, s2a, mub, s2b; };
  struct Lc { int dummy; };
  __device__ __forceinline__ static int elem(int r, int lane) { return r * G + lane; }

  __host__ __device__ static int lds_stride(const SweepArgs&) { return LDS_DBL; }
  __device__ __forceinline__ static void load(const SweepArgs& A, int c, int lane, St& s, Lc&, double*) {
    const double* v = A.vals + (size_t)c * VS;
#pragma unroll
    for (int r = 0; r < R; ++r) { s.a[r] = v[elem(r, lane)]; s.b[r] = v[32 + elem(r, lane)]; }
    s.s2c = v[64]; s.mua = v[65]; s.s2a = v[66]; s.mub = v[67]; s.s2b = v[68];
  }
  __device__ __forceinline__ static void store(const SweepArgs& A, int c, int lane, const St& s) {
    double* v = A.vals + (size_t)c * VS;
#pragma unroll
    for (int r = 0; r < R; ++r) { v[elem(r, lane)] = s.a[r]; v[32 + elem(r, lane)] = s.b[r]; }
    if (lane == 0) { v[64] = s.s2c; v[65] = s.mua; v[66] = s.s2a; v[67] = s.mub; v[68] = s.s2b; }
  }
  __device__ __forceinline__ static void monitored(const SweepArgs& A, const St& s, double* out) {
    out[0] = s.s2c;
    out[1] = s.mub;
    out[2] = s.mua - A.xbar * s.mub;  // alpha0 = mu_alpha - xbar * mu_beta (rats.jl:65-67)
  }
  // sim[i, :, 1] = unlist(m, true) for a kept iteration (mcmc.jl:76-77): lane 0 of the group
  __device__ __forceinline__ static void write_draws(const SweepArgs& A, const St& s, const Grp<G>& g,
                                                     int64_t row, int c) {
    if (g.lane != 0) return;
    double mon[PMON];
    monitored(A, s, mon);
#pragma unroll
    for (int j = 0; j < PMON; ++j) A.draws[(size_t)(row * PMON + j) * A.K + c] = mon[j];
  }
  __device__ __forceinline__ static bool is_vec(int node) { return node == MMB_RATS_ALPHA || node == MMB_RATS_BETA; }
  __device__ __forceinline__ static bool positive(int node) {
    return node == MMB_RATS_S2_C || node == MMB_RATS_S2_ALPHA || node == MMB_RATS_S2_BETA;
  }
  // park the chain state in LDS across a register-heavy phase (pivoted Cholesky), in the
  // AMM scratch that is idle during it (samplers.h amm(): lds = mat[TP] | z2s | vvs | mvs |
  // ia): alpha -> vvs, beta -> mvs, scalars -> the tail of z2s (pivot indices use 30 ints)
  __device__ __forceinline__ static void stash(double* lds, const St& s, int lane) {
    double* q = lds + TP;
#pragma unroll
    for (int r = 0; r < R; ++r) { q[DP + elem(r, lane)] = s.a[r]; q[2 * DP + elem(r, lane)] = s.b[r]; }
    if (lane == 0) { q[16] = s.s2c; q[17] = s.mua; q[18] = s.s2a; q[19] = s.mub; q[20] = s.s2b; }
  }
  __device__ __forceinline__ static void unstash(const double* lds, St& s, int lane) {
    const double* q = lds + TP;
#pragma unroll
    for (int r = 0; r < R; ++r) { s.a[r] = q[DP + elem(r, lane)]; s.b[r] = q[2 * DP + elem(r, lane)]; }
    s.s2c = q[16]; s.mua = q[17]; s.s2a = q[18]; s.mub = q[19]; s.s2b = q[20];
  }
  // select chains (a switch here is turned into a dynamically indexed private array)
  // c ? a : b as an integer bit blend: the optimiser folds a select chain over struct
  // fields into a load at a computed offset, which forces the chain state to scratch
  __device__ __forceinline__ static double blend(bool c, double a, double b) {
    const uint64_t m = 0ull - (uint64_t)c;
    return mmb_u2d((mmb_d2u(a) & m) | (mmb_d2u(b) & ~m));
  }
  __device__ __forceinline__ static double scalar(const St& s, int node) {
    double v = s.s2b;
    v = blend(node == MMB_RATS_S2_C, s.s2c, v);
    v = blend(node == MMB_RATS_MU_ALPHA, s.mua, v);
    v = blend(node == MMB_RATS_S2_ALPHA, s.s2a, v);
    v = blend(node == MMB_RATS_MU_BETA, s.mub, v);
    return v;
  }
  __device__ __forceinline__ static void set_scalar(St& s, int node, double v) {
    s.s2c = blend(node == MMB_RATS_S2_C, v, s.s2c);
    s.mua = blend(node == MMB_RATS_MU_ALPHA, v, s.mua);
    s.s2a = blend(node == MMB_RATS_S2_ALPHA, v, s.s2a);
    s.mub = blend(node == MMB_RATS_MU_BETA, v, s.mub);
    s.s2b = blend(node == MMB_RATS_S2_BETA, v, s.s2b);
  }
  __device__ __forceinline__ static int lane_node(const DBlock& B, int lane) {
    int n = B.nodes[0];
    n = lane == 1 ? B.nodes[1] : n;
    n = lane == 2 ? B.nodes[2] : n;
    n = lane == 3 ? B.nodes[3] : n;
    return n;
  }
  // unlist(block, transform) into lane-owned element slots
  __device__ __forceinline__ static void unlist(const DBlock& B, const St& s, int lane, double* x) {
    if (is_vec(B.nodes[0])) {
      const bool al = B.nodes[0] == MMB_RATS_ALPHA;
#pragma unroll
      for (int r = 0; r < R; ++r) x[r] = elem(r, lane) < 30 ? (al ? s.a[r] : s.b[r]) : 0.0;
    } else {
      int n = lane_node(B, lane);
      double v = scalar(s, n);
      x[0] = lane < B.d ? ((B.transform && positive(n)) ? mmb_log(v) : v) : 0.0;
#pragma unroll
      for (int r = 1; r < R; ++r) x[r] = 0.0;
    }
  }
  __device__ __forceinline__ static void relist(const DBlock& B, St& s, const Grp<G>& g, const double* x) {
    if (is_vec(B.nodes[0])) {
      const bool al = B.nodes[0] == MMB_RATS_ALPHA;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool in = elem(r, g.lane) < 30;
        if (al) s.a[r] = in ? x[r] : s.a[r];
        else s.b[r] = in ? x[r] : s.b[r];
      }
    } else {
      for (int e = 0; e < B.d; ++e) {
        double v = g.bcast(x[0], e);
        int n = B.nodes[e];
        set_scalar(s, n, (B.transform && positive(n)) ? mmb_exp(v) : v);
      }
    }
  }
  // lane partial of sum_t (y - (alpha + beta*Xm))^2 over this lane's rats (slot order)
  __device__ __forceinline__ static double ssr_lane(const SweepArgs& A, const Lc&, const double* a, const double* b,
                                                    int lane) {
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = elem(r, lane);
      const double* y = A.data0 + (e < 30 ? e : 0) * 5;
      double part = 0.0;
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        double mu = a[r] + b[r] * A.xm[t];
        double rr = y[t] - mu;
        part = fma(rr, rr, part);
      }
      acc += e < 30 ? part : 0.0;
    }
    return acc;
  }
  __device__ __forceinline__ static double normsum_lane(double mu, double sig, double logsig, const double* x,
                                                        int lane) {
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) acc += elem(r, lane) < 30 ? d_normlogpdf(mu, sig, logsig, x[r]) : 0.0;
    return acc;
  }
  // Invariants of a vector block's logpdf! that do not depend on the block vector:
  // prior sd / log sd of the block node and y's ScalMat constants.  Computed once per
  // block update with the same operations logf would do, so results are bit-identical.
  struct VecCtx { double mu, sig, logsig, yk; double invv; bool al; };
  __device__ __forceinline__ static VecCtx vec_ctx(const DBlock& B, const St& s) {
    VecCtx c;
    c.al = B.nodes[0] == MMB_RATS_ALPHA;
    c.mu = c.al ? s.mua : s.mub;
    c.sig = sqrt(c.al ? s.s2a : s.s2b);
    c.logsig = mmb_log(c.sig);
    const double sc = sqrt(s.s2c);
    const double value = sc * sc;
    c.invv = 1.0 / value;
    c.yk = 150 * MMB_LOG2PI + 150 * mmb_log(value);
    return c;
  }
  // logpdf!([alpha] or [beta], x): prior (params \ targets) then y (d_iso expanded)
  __device__ __forceinline__ static double logf_vec(const SweepArgs& A, const VecCtx& c,
                                                    const St& s, const Lc& l, const Grp<G>& g,
                                                    const double* x) {
    double pr = normsum_lane(c.mu, c.sig, c.logsig, x, g.lane);
    double ss = c.al ? ssr_lane(A, l, x, s.b, g.lane) : ssr_lane(A, l, s.a, x, g.lane);
    g.sum2(pr, ss);
    double lp = 0.0 + pr;
    if (!isfinite(lp)) return lp;
    return lp + (-0.5 * (c.yk + ss * c.invv));
  }
  // logpdf! at two block vectors (AMM: the proposal and the current value) with one joint
  // butterfly of the four lane partials: each sum takes the same partners in the same order as
  // logf_vec's, so both values are bit-identical to two logf_vec calls, with half the DPP
  // dependency stages
  __device__ __forceinline__ static void logf_vec2(const SweepArgs& A, const VecCtx& c, const St& s, const Lc& l,
                                                   const Grp<G>& g, const double* x, const double* v, double& lx,
                                                   double& lv) {
    double px = normsum_lane(c.mu, c.sig, c.logsig, x, g.lane);
    double sx = c.al ? ssr_lane(A, l, x, s.b, g.lane) : ssr_lane(A, l, s.a, x, g.lane);
    double pv = normsum_lane(c.mu, c.sig, c.logsig, v, g.lane);
    double sv = c.al ? ssr_lane(A, l, v, s.b, g.lane) : ssr_lane(A, l, s.a, v, g.lane);
    g.sum4(px, sx, pv, sv);
    const double ax = 0.0 + px, av = 0.0 + pv;
    lx = isfinite(ax) ? ax + (-0.5 * (c.yk + sx * c.invv)) : ax;
    lv = isfinite(av) ? av + (-0.5 * (c.yk + sv * c.invv)) : av;
  }
  // AMWG on a vector block (samplers.h amwg, lane-parallel path): changing element j of alpha
  // (beta) changes only lane j's prior term and lane j's part of the residual sum of squares, so
  // logf_vec at any state is the same butterfly over per-lane terms, and the lane's two terms
  // at its own element value are what logf_vec would form on that lane
  static constexpr bool AMWG_SEP = true;
  __device__ __forceinline__ static bool amwg_sep(const DBlock& B) { return is_vec(B.nodes[0]); }
  __device__ __forceinline__ static void amwg_terms(const SweepArgs& A, const VecCtx& c, const St& s, const Lc& l,
                                                    int lane, double xv, double& tp, double& ts) {
    double xa[R];
#pragma unroll
    for (int r = 0; r < R; ++r) xa[r] = xv;
    tp = normsum_lane(c.mu, c.sig, c.logsig, xa, lane);
    ts = c.al ? ssr_lane(A, l, xa, s.b, lane) : ssr_lane(A, l, s.a, xa, lane);
  }
  // logf_vec = (0 + sum tp) + (-0.5 * (yk + (sum ts) * invv)).  Coordinate j's exact difference
  // d_j = (tp_j' - tp_j) - 0.5 invv (ts_j' - ts_j); each rounded logf is within 9 u (sum_i |tp_i| +
  // |yk| + invv sum_i |ts_i|) of its exact value (a depth-5 tree sum, then three roundings):
  // band = 2^-46 (128 u) times that magnitude plus the difference's own terms (samplers.h amwg_lanes)
  static constexpr bool AMWG_PROBE = true;
  __device__ __forceinline__ static double amwg_epsf(const DBlock&) { return 0x1p-46; }
  __device__ __forceinline__ static void amwg_dm(const SweepArgs& A, const DBlock&, const VecCtx& c, const St& s,
                                                 const Lc& l, const Grp<G>& g, double x0, double x1, double& del,
                                                 double& epsm, bool& bad) {
    double tp0, ts0, tp1, ts1;
    amwg_terms(A, c, s, l, g.lane, x0, tp0, ts0);
    amwg_terms(A, c, s, l, g.lane, x1, tp1, ts1);
    bad = !(isfinite(tp0) && isfinite(ts0) && isfinite(tp1) && isfinite(ts1));
    double ap = fmax(fabs(tp0), fabs(tp1)), as = fmax(fabs(ts0), fabs(ts1));
    g.sum2(ap, as);  // bounds of sum |terms| over both states
    const double dp = tp1 - tp0, ds = ts1 - ts0;
    del = dp + (-0.5 * c.invv) * ds;
    const double mag = ap + fabs(c.yk) + c.invv * as;
    epsm = mag + fabs(dp) + c.invv * fabs(ds) + fabs(del);
    bad = bad || !isfinite(c.invv) || !isfinite(c.yk);
  }
  // block-update-invariant context (vector blocks); scalar blocks fall back to logf
  using Prep = VecCtx;
  __device__ __forceinline__ static Prep prep(const DBlock& B, const St& s) { return vec_ctx(B, s); }
  __device__ __forceinline__ static double logf_p(const SweepArgs& A, const DBlock& B, const Prep& c,
                                                  const St& s, const Lc& l, const Grp<G>& g,
                                                  const double* x) {
    if (is_vec(B.nodes[0])) return logf_vec(A, c, s, l, g, x);
    return logf(A, B, s, l, g, x);
  }
  __device__ __forceinline__ static void logf_p2(const SweepArgs& A, const DBlock& B, const Prep& c, const St& s,
                                                 const Lc& l, const Grp<G>& g, const double* x, const double* v,
                                                 double& lx, double& lv) {
#ifndef MMB_EXP_LOGF1
    if (is_vec(B.nodes[0])) {
      logf_vec2(A, c, s, l, g, x, v, lx, lv);
      return;
    }
#endif
    lx = logf_p(A, B, c, s, l, g, x);
    lv = logf_p(A, B, c, s, l, g, v);
  }
  // logpdf!(block, x)
  // (ssp: y's residual sum of squares already formed from this state -- slice_logf0)
  __device__ __forceinline__ static double logf(const SweepArgs& A, const DBlock& B, const St& s0, const Lc& l,
                                const Grp<G>& g, const double* x, const double* ssp = nullptr) {
    St s = s0;
    relist(B, s, g, x);
    if (is_vec(B.nodes[0])) return logf_vec(A, vec_ctx(B, s0), s0, l, g, x);
    // scalar block: params (none is a target of another) in block order
    unsigned tm = 0;
    double lp = 0.0;
    bool stop = false;
    for (int a = 0; a < B.nn; ++a) {
      int n = B.nodes[a];
      tm |= (n == MMB_RATS_S2_C) ? 4u : (n == MMB_RATS_MU_ALPHA || n == MMB_RATS_S2_ALPHA) ? 1u : 2u;
      if (stop) continue;
      double t = positive(n) ? d_iglogpdf(A.ig_c, scalar(s, n), B.transform)
                             : d_normlogpdf(0.0, 1000.0, mmb_log(1000.0), scalar(s, n));
      lp += t;
      if (!isfinite(lp)) stop = true;
    }
    if (stop) return lp;
    // targets in topological order: alpha, beta, y
    if (tm & 1u) {
      double sig = sqrt(s.s2a);
      double v = normsum_lane(s.mua, sig, mmb_log(sig), s.a, g.lane);
      lp += g.sum(v);
      if (!isfinite(lp)) return lp;
    }
    if (tm & 2u) {
      double sig = sqrt(s.s2b);
      double v = normsum_lane(s.mub, sig, mmb_log(sig), s.b, g.lane);
      lp += g.sum(v);
      if (!isfinite(lp)) return lp;
    }
    if (tm & 4u) {
      double ss = ssp ? *ssp : g.sum(ssr_lane(A, l, s.a, s.b, g.lane));
      lp += d_iso(150, sqrt(s.s2c), ss);
    }
    return lp;
  }
  // Slice (Univariate) on a scalar block with its candidates evaluated four at a time
  // (samplers.h slice_uni_cand): lanes 8q .. 8q+7 of the chain's 32 evaluate candidate q, lane
  // l of the eight holding rats 4l .. 4l+3.  A lane sums its four leaves as ((v0 + v1) + (v2 +
  // v3)) -- levels 0 and 1 of logf's 32-lane butterfly -- and levels 2, 3 and 4 (quad pairs,
  // 8-lane pairs, 16-lane halves) are xor 1, xor 2 and the half-row mirror of the eight lanes:
  // the same tree over the same leaves, so the sum is logf's bit for bit.  Everything else in
  // slice_cand_logf is logf's code on the candidate's node values.
  static constexpr bool SLICE_CAND = true;
  static constexpr int SLICE_CAND_D = 2;  // scalar blocks of up to two nodes
#ifndef MMB_SLICE_NC
#define MMB_SLICE_NC 4
#endif
  // candidates per round: NC groups of 32 / NC lanes, NC leaves (rats) per lane
  static constexpr int SLICE_NC = MMB_SLICE_NC;
  static_assert(SLICE_NC == 2 || SLICE_NC == 4 || SLICE_NC == 8, "2, 4 or 8 candidates per round");
  struct SCtx {
    const double* ab;  // LDS: alpha[32] | beta[32] of the chain
    double ss;         // y's residual sum of squares (alpha, beta are not in the block)
    unsigned tm;       // target mask as logf forms it
  };
  __device__ __forceinline__ static bool slice_cand_ok(const DBlock& B) {
    return !is_vec(B.nodes[0]) && B.nn == B.d && B.d <= SLICE_CAND_D;
  }
  __device__ __forceinline__ static void slice_cand_prep(const SweepArgs& A, const DBlock& B, const St& s, const Lc& l,
                                                         const Grp<G>& g, double* lds, SCtx& c) {
    unsigned tm = 0;
    for (int a = 0; a < B.nn; ++a) {
      const int n = B.nodes[a];
      tm |= (n == MMB_RATS_S2_C) ? 4u : (n == MMB_RATS_MU_ALPHA || n == MMB_RATS_S2_ALPHA) ? 1u : 2u;
    }
    c.tm = tm;
    c.ss = (tm & 4u) ? g.sum(ssr_lane(A, l, s.a, s.b, g.lane)) : 0.0;
    lds[g.lane] = s.a[0];
    lds[32 + g.lane] = s.b[0];
    c.ab = lds;
    grp_sync();
  }
  // normsum_lane + g.sum over the candidate group (see above); v: alpha or beta in LDS.  NC = 8:
  // groups of four lanes with eight leaves each, levels 0-2 in the lane, 3-4 by xor 1 and xor 2;
  // NC = 2: groups of sixteen lanes with two leaves each, level 0 in the lane, 1-4 across it.
  __device__ __forceinline__ static double normsum_grp8(double mu, double sig, double logsig, const double* v,
                                                        int lane) {
    constexpr int L = SLICE_NC, LPC = 32 / SLICE_NC;
    const int r0 = L * (lane & (LPC - 1));
    double lf[L];
#pragma unroll
    for (int m = 0; m < L; m += 2) {
      const double2 p = *(const double2*)(v + r0 + m);
      lf[m] = 0.0 + (r0 + m < 30 ? d_normlogpdf(mu, sig, logsig, p.x) : 0.0);
      lf[m + 1] = 0.0 + (r0 + m + 1 < 30 ? d_normlogpdf(mu, sig, logsig, p.y) : 0.0);
    }
    double q;
    if constexpr (L == 2) {
      q = lf[0] + lf[1];
    } else {
      q = (lf[0] + lf[1]) + (lf[2] + lf[3]);
      if constexpr (L == 8) q = q + ((lf[4] + lf[5]) + (lf[6] + lf[7]));
    }
    q += Grp<G>::template other_d<0>(q);
    q += Grp<G>::template other_d<1>(q);
    if constexpr (LPC >= 8) q += Grp<G>::template other_d<2>(q);
    if constexpr (LPC >= 16) q += Grp<G>::template other_d<3>(q);
    return q;
  }
  // The pieces of slice_cand_logf that only depend on one node value -- each block node's prior
  // term, the target variance's square root and log -- memoised per lane by the bits of that
  // value: the nodes other than the coordinate being sampled keep their values through all of
  // the coordinate's candidates, so their priors (a log and a division for a variance node) and,
  // for a mean coordinate, the target scale (a square root and a log) are formed once.  A hit
  // returns the value the same function gave for the same input bits; a NaN input is never
  // cached (the keys start as a NaN pattern).
  struct SMemo {
    uint64_t pk[SLICE_CAND_D];
    double pt[SLICE_CAND_D];
    uint64_t sk;
    double sg, lsg;
    __device__ __forceinline__ SMemo() : sk(0x7ff0000000000001ull), sg(0.0), lsg(0.0) {
#pragma unroll
      for (int a = 0; a < SLICE_CAND_D; ++a) { pk[a] = 0x7ff0000000000001ull; pt[a] = 0.0; }
    }
    __device__ __forceinline__ void scale(double var, double& sig, double& lsig) {
      const uint64_t vb = mmb_d2u(var);
      if (vb == sk && var == var) {
        sig = sg;
        lsig = lsg;
      } else {
        sig = sqrt(var);
        lsig = mmb_log(sig);
        sk = vb;
        sg = sig;
        lsg = lsig;
      }
    }
  };
  // logf at the start of a Slice update, after slice_cand_prep: the s2_c block takes y's sum of
  // squares from the prep (the same g.sum over the same lane terms: alpha and beta are not in the block)
  __device__ __forceinline__ static double slice_logf0(const SweepArgs& A, const DBlock& B, const St& s, const Lc& l,
                                                       const Grp<G>& g, const double* x, const SCtx& c) {
    return logf(A, B, s, l, g, x, (c.tm & 4u) ? &c.ss : nullptr);
  }
  // logf(block) at the block vector xv[] (group-uniform values, the candidate's)
  __device__ __forceinline__ static double slice_cand_logf(const SweepArgs& A, const DBlock& B, const St& s0,
                                                           const SCtx& c, const double* xv, int lane, SMemo& mm) {
    St s = s0;
#pragma unroll
    for (int a = 0; a < SLICE_CAND_D; ++a) {  // relist (B.nn <= SLICE_CAND_D: slice_cand_ok)
      if (a < B.nn) {
        const int n = B.nodes[a];
        set_scalar(s, n, (B.transform && positive(n)) ? mmb_exp(xv[a]) : xv[a]);
      }
    }
    double lp = 0.0;
    bool stop = false;
#pragma unroll
    for (int a = 0; a < SLICE_CAND_D; ++a) {
      if (a >= B.nn || stop) continue;
      const int n = B.nodes[a];
      const double v = scalar(s, n);
      const uint64_t vb = mmb_d2u(v);
      double t;
      if (vb == mm.pk[a] && v == v) {
        t = mm.pt[a];
      } else {
        t = positive(n) ? d_iglogpdf(A.ig_c, v, B.transform) : d_normlogpdf(0.0, 1000.0, mmb_log(1000.0), v);
        mm.pk[a] = vb;
        mm.pt[a] = t;
      }
      lp += t;
      if (!isfinite(lp)) stop = true;
    }
    if (stop) return lp;
    if (c.tm & 1u) {
      double sig, lsig;
      mm.scale(s.s2a, sig, lsig);
      lp += normsum_grp8(s.mua, sig, lsig, c.ab, lane);
      if (!isfinite(lp)) return lp;
    }
    if (c.tm & 2u) {
      double sig, lsig;
      mm.scale(s.s2b, sig, lsig);
      lp += normsum_grp8(s.mub, sig, lsig, c.ab + 32, lane);
      if (!isfinite(lp)) return lp;
    }
    if (c.tm & 4u) lp += d_iso(150, sqrt(s.s2c), c.ss);
    return lp;
  }
  // The random draw of a conjugate block does not depend on the chain state: a Gamma(a)
  // variate for the s2 blocks (rand(InverseGamma(a, b)) = b / G, shape a fixed by the
  // model), a standard normal for the mu blocks.  The sweep kernel draws them for all
  // blocks of an iteration at once, one block per lane (predraw), and passes each block
  // its value.  Returns 1 (gamma, shape *a) or 2 (normal).
  __device__ __forceinline__ static int gibbs_draw_kind(const DBlock& B, double* a) {
    const int n = B.nodes[0];
    if (n == MMB_RATS_MU_ALPHA || n == MMB_RATS_MU_BETA) { *a = 0.0; return 2; }
    *a = n == MMB_RATS_S2_C ? 150.0 / 2.0 + 0.001 : 30.0 / 2.0 + 0.001;
    return 1;
  }
  // conjugate full conditionals (Gibbs_s2_c, Gibbs_mu_*, Gibbs_s2_*);
  // `draw` is the block's predrawn Gamma / normal variate (gibbs_draw_kind)
  __device__ __forceinline__ static void gibbs(const SweepArgs& A, const DBlock& B, St& s, const Lc& l,
                               const Grp<G>& g, const mmb_rng*, const mmb_rng*, const mmb_rng*, double draw) {
    int n = B.nodes[0];
    if (n == MMB_RATS_S2_C) {
      double ss = g.sum(ssr_lane(A, l, s.a, s.b, g.lane));
      double b = ss / 2.0 + 0.001;
      s.s2c = b / draw;
    } else if (n == MMB_RATS_MU_ALPHA || n == MMB_RATS_MU_BETA) {
      const bool al = n == MMB_RATS_MU_ALPHA;
      double part = 0.0;
#pragma unroll
      for (int r = 0; r < R; ++r) part += elem(r, g.lane) < 30 ? blend(al, s.a[r], s.b[r]) : 0.0;
      double sum = g.sum(part);
      double s2 = blend(al, s.s2a, s.s2b);
      double var0 = 1000.0 * 1000.0;
      double vv = 1.0 / (30.0 / s2 + 1.0 / var0);
      double mean = vv * (sum / s2 + 0.0 / var0);
      double v = mean + sqrt(vv) * draw;
      s.mua = blend(al, v, s.mua);
      s.mub = blend(al, s.mub, v);
    } else {
      const bool al = n == MMB_RATS_S2_ALPHA;
      double mu = blend(al, s.mua, s.mub);
      double part = 0.0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double rr = blend(al, s.a[r], s.b[r]) - mu;
        part += elem(r, g.lane) < 30 ? rr * rr : 0.0;
      }
      double ss = g.sum(part);
      double v = (ss / 2.0 + 0.001) / draw;
      s.s2a = blend(al, v, s.s2a);
      s.s2b = blend(al, s.s2b, v);
    }
  }
};

// ------------------------------------------------------------------ line
// doc/tutorial/line.jl:5-25.  Device layout per chain: [b1, b2, s2, pad].  G = 1.
template <>
struct Mdl<MMB_MODEL_LINE> {
  static constexpr int G = 1, R = 3, DMAX = 3, DP = 4, TP = 8, VS = 4, PMON = 3;
  static constexpr int LDS_DBL = TP + 4 * DP + 8;
  struct St { double v[3]; };
  struct Lc { int dummy; };
  __device__ __forceinline__ static void stash(double* lds, const St& s, int) {
    double* q = lds + TP + 4 * DP;
    q[0] = s.v[0]; q[1] = s.v[1]; q[2] = s.v[2];
  }
  __device__ __forceinline__ static void unstash(const double* lds, St& s, int) {
    const double* q = lds + TP + 4 * DP;
    s.v[0] = q[0]; s.v[1] = q[1]; s.v[2] = q[2];
  }

  __host__ __device__ static int lds_stride(const SweepArgs&) { return LDS_DBL; }
  __device__ __forceinline__ static void load(const SweepArgs& A, int c, int, St& s, Lc&, double*) {
    const double* v = A.vals + (size_t)c * VS;
    s.v[0] = v[0]; s.v[1] = v[1]; s.v[2] = v[2];
  }
  __device__ __forceinline__ static void store(const SweepArgs& A, int c, int, const St& s) {
    double* v = A.vals + (size_t)c * VS;
    v[0] = s.v[0]; v[1] = s.v[1]; v[2] = s.v[2];
  }
  __device__ __forceinline__ static void monitored(const SweepArgs&, const St& s, double* out) {
    out[0] = s.v[0]; out[1] = s.v[1]; out[2] = s.v[2];
  }
  __device__ __forceinline__ static void write_draws(const SweepArgs& A, const St& s, const Grp<G>&,
                                                     int64_t row, int c) {
#pragma unroll
    for (int j = 0; j < PMON; ++j) A.draws[(size_t)(row * PMON + j) * A.K + c] = s.v[j];
  }
  __device__ __forceinline__ static double pick(const St& s, int vi) {
    return vi == 0 ? s.v[0] : vi == 1 ? s.v[1] : s.v[2];
  }
  __device__ __forceinline__ static void unlist(const DBlock& B, const St& s, int, double* x) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int vi = B.emap[r];
      double v = pick(s, vi);
      x[r] = r < B.d ? ((B.transform && vi == 2) ? mmb_log(v) : v) : 0.0;
    }
  }
  __device__ __forceinline__ static void relist(const DBlock& B, St& s, const Grp<G>&, const double* x) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < B.d) {
        int vi = B.emap[r];
        double v = (B.transform && vi == 2) ? mmb_exp(x[r]) : x[r];
        if (vi == 0) s.v[0] = v;
        else if (vi == 1) s.v[1] = v;
        else s.v[2] = v;
      }
    }
  }
  static constexpr bool AMWG_SEP = false;  // samplers.h amwg: sequential path only
  static constexpr bool SLICE_CAND = false;  // samplers.h slice_uni: one candidate at a time
  static constexpr int SLICE_CAND_D = 1;
  struct SCtx {};
  struct SMemo {};
  struct Prep {};
  __device__ __forceinline__ static Prep prep(const DBlock&, const St&) { return Prep{}; }
  __device__ __forceinline__ static double logf_p(const SweepArgs& A, const DBlock& B, const Prep&,
                                                  const St& s, const Lc& l, const Grp<G>& g,
                                                  const double* x) {
    return logf(A, B, s, l, g, x);
  }
  __device__ __forceinline__ static void logf_p2(const SweepArgs& A, const DBlock& B, const Prep& c, const St& s,
                                                 const Lc& l, const Grp<G>& g, const double* x, const double* v,
                                                 double& lx, double& lv) {
    lx = logf_p(A, B, c, s, l, g, x);
    lv = logf_p(A, B, c, s, l, g, v);
  }
  __device__ __forceinline__ static double ylp(const SweepArgs& A, const St& s) {
    double ssq = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      double mu = s.v[0] + A.lx[i] * s.v[1];
      double r = A.ly[i] - mu;
      ssq += r * r;
    }
    return d_iso(5, sqrt(s.v[2]), ssq);
  }
  __device__ __forceinline__ static double logf(const SweepArgs& A, const DBlock& B, const St& s0, const Lc&,
                                const Grp<G>& g, const double* x) {
    St s = s0;
    relist(B, s, g, x);
    double lp = 0.0;
    for (int a = 0; a < B.nn; ++a) {
      double t;
      if (B.nodes[a] == MMB_LINE_BETA) {
        if (!isfinite(s.v[0]) || !isfinite(s.v[1])) t = -__builtin_inf();
        else t = d_iso(2, sqrt(1000.0), s.v[0] * s.v[0] + s.v[1] * s.v[1]);
      } else {
        t = d_iglogpdf(A.ig_c, s.v[2], B.transform);
      }
      lp += t;
      if (!isfinite(lp)) return lp;
    }
    return lp + ylp(A, s);  // targets: mu (logical, 0), y
  }
  // logpdfgrad!(block, x, dtype) (sampler.jl:106-111): B.fdgrad -> the reference's Calculus
  // forward differences (simulation.jl:47-51; epsilon = sqrt(eps()) * max(1, |x_i|), Julia max
  // propagating NaN; (f(x + epsilon e_i) - f(x)) / epsilon), else the analytic gradient;
  // non-finite entries -> 0 either way
  __device__ __forceinline__ static double logf_grad(const SweepArgs& A, const DBlock& B, const St& s0,
                                     const double* x, double* gr) {
    if (B.fdgrad) {
      Grp<G> g;
      const double fx = logf(A, B, s0, Lc{}, g, x);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        double gk = 0.0;
        if (k < B.d) {
          const double ax = fabs(x[k]);
          const double eps = 0x1p-26 * (isnan(ax) ? ax : (ax > 1.0 ? ax : 1.0));
          double xx[3] = {x[0], x[1], x[2]};
          xx[k] = x[k] + eps;
          gk = (logf(A, B, s0, Lc{}, g, xx) - fx) / eps;
        }
        gr[k] = isfinite(gk) ? gk : 0.0;
      }
      return fx;
    }
    St s = s0;
    Grp<G> g;
    relist(B, s, g, x);
    double lp = logf(A, B, s0, Lc{}, g, x);
    double s2 = s.v[2];
    double sr = 0.0, sxr = 0.0, ssq = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      double mu = s.v[0] + A.lx[i] * s.v[1];
      double r = A.ly[i] - mu;
      sr += r;
      sxr = fma(A.lx[i], r, sxr);
      ssq = fma(r, r, ssq);
    }
    double sb = sqrt(1000.0);
    double ivb = 1.0 / (sb * sb);
    // partials by value slot (beta0, beta1, log s2), then to block elements through emap: a
    // block may list s2 first or hold one of the nodes only ([s2, beta], [s2])
    const double g0 = sr / s2 - s.v[0] * ivb;
    const double g1 = sxr / s2 - s.v[1] * ivb;
    const double g2 = -(0.001 + 2.5) + (0.5 * ssq + 0.001) / s2;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int vi = B.emap[k];
      double gk = vi == 0 ? g0 : vi == 1 ? g1 : g2;
      gk = k < B.d ? gk : 0.0;
      gr[k] = isfinite(gk) ? gk : 0.0;
    }
    return lp;
  }
  __device__ __forceinline__ static int gibbs_draw_kind(const DBlock&, double* a) { *a = 0.0; return 0; }
  __device__ __forceinline__ static void gibbs(const SweepArgs& A, const DBlock& B, St& s, const Lc&,
                               const Grp<G>&, const mmb_rng* rn, const mmb_rng* gn,
                               const mmb_rng* gu, double) {
    if (B.nodes[0] == MMB_LINE_BETA) {  // line.jl:27-36
      double s2 = s.v[2];
      double sb = sqrt(1000.0);
      double ic = 1.0 / (sb * sb);
      double sx = 0.0, sxx = 0.0, sy = 0.0, sxy = 0.0;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        sx += A.lx[i]; sxx += A.lx[i] * A.lx[i]; sy += A.ly[i]; sxy += A.lx[i] * A.ly[i];
      }
      double a = 5.0 / s2 + ic, b = sx / s2, dd = sxx / s2 + ic;
      double det = a * dd - b * b;
      double S11 = dd / det, S12 = -b / det, S22 = a / det;
      double r1 = sy / s2, r2 = sxy / s2;
      double m1 = S11 * r1 + S12 * r2, m2 = S12 * r1 + S22 * r2;
      double l11 = sqrt(S11), l21 = S12 / l11, l22 = sqrt(S22 - l21 * l21);
      double z0, z1;
      mmb_normal_pair(rn, 0u, &z0, &z1);
      s.v[0] = m1 + l11 * z0;
      s.v[1] = m2 + (l21 * z0 + l22 * z1);
    } else {  // line.jl:38-45
      double ssq = 0.0;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        double r = A.ly[i] - (s.v[0] + A.lx[i] * s.v[1]);
        ssq += r * r;
      }
      uint32_t kn = 0, ku = 0;
      s.v[2] = (ssq / 2.0 + 0.001) / mmb_gamma_mt(5.0 / 2.0 + 0.001, gn, gu, &kn, &ku);
    }
  }
};
