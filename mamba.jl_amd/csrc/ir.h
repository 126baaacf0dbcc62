// ir.h — the generic node-IR model of the sweep kernel.
//
// A Mamba Model DAG (src/model/model.jl:5-27, src/model/dependent.jl:75-152) lowered by the
// host (mamba.jl_amd/ir.py) into mmb_ir_node records (include/mamba_hip.h) whose
// distribution parameters are stack-code expressions over the chain state, the data pool
// and the element index i.  One chain per 32-lane group (two chains per wave64), element i
// of a node in lane i % 32, so the samplers of samplers.h run unchanged (R = 1, d <= 32;
// the AMM factorization is pchol32).  LDS per chain:
//
//   [AMM scratch (schemes with AMM)] [cur: chain state] [prop: state + the block's
//   candidate x] [expression stack: depth x 32 doubles]
//
// logpdf!(m, x, block, transform) (src/model/simulation.jl:77-90): relist x into `prop`
// (invlink when transformed, transformdistribution.jl:6-93), then the block's terms —
// params \ targets in block order, then targets in topological order — each a node
// logpdf_sub (distributionstruct.jl:136-168: per element insupport ? logpdf (+ Jacobian)
// : -Inf; lane partials in element order, then the 32-lane butterfly), with the early exit
// on a non-finite running sum (simulation.jl:64,84).  NUTS / HMC / MALA use Calculus'
// forward difference like the reference's gradlogpdf! (simulation.jl:47-51,
// sampler.jl:106-111): d + 1 logpdf! per gradient.
#pragma once
#include "device.h"

// device-only opcodes: a leaf fused with the following binary op (engine.cpp ir_fuse),
// MMB_IR_FUSED + 4 (leaf opcode - 1) + (binary opcode - MMB_IR_OP_ADD)
#define MMB_IR_FUSED 64

template <class T>
__device__ __forceinline__ const T& ir_const_ref(const T* p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const T*)&((const __attribute__((address_space(4))) T*)p)[i];
#else
  return p[i];
#endif
}

// Specialised build (MMB_IR_JIT, engine.cpp ir_jit_source -> hipRTC): the model's node log
// densities and Logical expressions are generated as straight-line code before this header
// (mmb_jit_block_lp, mmb_jit_logical: the interpreter's operations in the interpreter's order,
// so results are bit-identical), and DMAX is the widest AMM block of the scheme (MMB_IR_DMAX),
// so the unrolled factorization has no steps past it.  The LDS layout (TP, DP) is unchanged.
#ifndef MMB_IR_DMAX
#define MMB_IR_DMAX 32
#endif

template <>
struct Mdl<MMB_MODEL_IR> {
  static constexpr int G = 32, R = 1, DMAX = MMB_IR_DMAX, DP = 32, TP = 528, VS = 0, PMON = 0;
  // AMM scratch: mat[TP] | z2 | vv | mv | ia, then pchol32's reciprocal slot prow[DMAX]
  static constexpr int AMM_DBL = TP + 4 * DP + 2;
  static constexpr int LDS_DBL = 0;  // runtime layout: lds_stride()
  struct St {
    double* cur;                 // chain state (LDS)
    double* prop;                // state with the block candidate written in (LDS)
    double* stk;                 // expression stack spills (LDS)
    const mmb_ir_node* nodes;    // node table (uniform)
  };
  struct Lc { int dummy; };
  __host__ __device__ static int lds_stride(const SweepArgs& A) { return A.ir_lds; }

  __device__ __forceinline__ static void load(const SweepArgs& A, int c, int lane, St& s, Lc&, double* lds) {
    s.cur = lds + A.ir_amm;
    s.prop = s.cur + A.ir_vs;
    s.stk = s.prop + A.ir_vs;
    s.nodes = A.ir_nodes;
    const double* v = A.vals + (size_t)c * A.ir_vs;
    for (int j = lane; j < A.ir_vs; j += G) {
      const double t = v[j];
      s.cur[j] = t;
      s.prop[j] = t;
    }
    grp_sync();
  }
  __device__ __forceinline__ static void store(const SweepArgs& A, int c, int lane, const St& s) {
    grp_sync();
    double* v = A.vals + (size_t)c * A.ir_vs;
    for (int j = lane; j < A.ir_vs; j += G) v[j] = s.cur[j];
  }
  __device__ __forceinline__ static void stash(double*, const St&, int) {}  // state already in LDS
  __device__ __forceinline__ static void unstash(const double*, St&, int) {}

  // ---- expressions: stack code, top of stack in a register, spills in this lane's LDS column.
  // The next code word is fetched (scalar load) before the current one is executed, so the
  // fetch latency overlaps the op instead of following it (seeds 1.09e7 -> 1.13e7 /s, rats
  // reference scheme 3.04e6 -> 3.37e6; two words ahead measured 2 % slower).  The device
  // code buffer is padded with END words (engine.cpp).
  __device__ static double ev(const SweepArgs& A, int pc, int i, const double* vals, double* stk, int lane) {
    double acc = 0.0;
    int sp = 0;
    int w = ir_const_ref(A.ir_code, pc);
    for (;;) {
      int wn = ir_const_ref(A.ir_code, pc + 1);
      const int op = (int)((uint32_t)w >> 24), arg = w & 0xffffff;
      if (op == MMB_IR_OP_END) return acc;
      if (op < 16 || op >= MMB_IR_FUSED) {  // a leaf, pushed or (fused) combined with the top
        const int lk = op < 16 ? op : ((op - MMB_IR_FUSED) >> 2) + 1;
        double v;
        if (lk == MMB_IR_OP_CONST) v = A.ir_const[arg];
        else if (lk == MMB_IR_OP_VAL) v = vals[arg];
        else if (lk == MMB_IR_OP_VALI) v = vals[arg + i];
        else if (lk == MMB_IR_OP_VALG) {  // two words: the gather's pool offset follows
          ++pc;
          v = vals[arg + (int)A.ir_pool[wn + i]];
          wn = ir_const_ref(A.ir_code, pc + 1);
        } else if (lk == MMB_IR_OP_DATA) v = A.ir_pool[arg + i];
        else v = A.ir_pool[arg];  // MMB_IR_OP_DATAS
        if (op < 16) {
          // the bottom slot is never popped: no spill for an expression's first leaf
          if (sp > 0) stk[sp * G + lane] = acc;
          ++sp;
          acc = v;
        } else {  // "leaf op" fused by the engine (engine.cpp ir_fuse): left = top, right = leaf
          const int bo = (op - MMB_IR_FUSED) & 3;
          if (bo == 0) acc = acc + v;
          else if (bo == 1) acc = acc - v;
          else if (bo == 2) acc = acc * v;
          else acc = acc / v;
        }
      } else if (op < 32) {
        --sp;
        const double l = stk[sp * G + lane];
        if (op == MMB_IR_OP_ADD) acc = l + acc;
        else if (op == MMB_IR_OP_SUB) acc = l - acc;
        else if (op == MMB_IR_OP_MUL) acc = l * acc;
        else acc = l / acc;  // MMB_IR_OP_DIV
      } else {
        acc = mmb_ir_unary(op, acc);
      }
      w = wn;
      ++pc;
    }
  }

  // logpdf(node[, transform]) (dependent.jl:207-213 -> logpdf_sub), group-uniform result
  __device__ static double node_lp(const SweepArgs& A, int n, const double* vals, double* stk,
                                   const Grp<G>& g, int tr) {
    const mmb_ir_node& N = ir_const_ref(A.ir_nodes, n);
    const double* src = N.fixed ? A.ir_pool + N.off : vals + N.off;
    const int lane = g.lane;
    if (N.family == MMB_IR_ISONORMAL) {  // MvNormal(mu, sigma): PDMats ScalMat, insupport = all finite
      const double sig = ev(A, N.expr[1], 0, vals, stk, lane);
      double ss = 0.0, bad = 0.0;
      for (int i = lane; i < N.len; i += G) {
        const double x = src[i];
        const double r = x - ev(A, N.expr[0], i, vals, stk, lane);
        ss = ss + r * r;
        bad = isfinite(x) ? bad : 1.0;
      }
      g.sum2(ss, bad);
      return bad != 0.0 ? -__builtin_inf() : d_iso(N.len, sig, ss);
    }
    double acc = 0.0;
    for (int i = lane; i < N.len; i += G) {
      const double a = N.expr[0] >= 0 ? ev(A, N.expr[0], i, vals, stk, lane) : 0.0;
      const double b = N.expr[1] >= 0 ? ev(A, N.expr[1], i, vals, stk, lane) : 0.0;
      const double ct = N.cterm >= 0 ? A.ir_pool[N.cterm + i] : 0.0;
      acc = acc + mmb_ir_lp(N.family, src[i], a, b, ct, tr, N.lo, N.hi);
    }
    return g.sum(acc);
  }

  // element e of the block vector: its state slot and its node's link
  __device__ __forceinline__ static int elem(const St& s, const DBlock& B, int e, int* lk, double* lo, double* hi) {
    int base = 0, slot = 0;
    *lk = 0; *lo = 0.0; *hi = 0.0;
    for (int a = 0; a < B.nn; ++a) {
      const mmb_ir_node& N = ir_const_ref(s.nodes, B.nodes[a]);
      if (e >= base && e < base + N.len) {
        slot = N.off + e - base;
        *lk = mmb_ir_link_kind(N.family);
        *lo = N.lo; *hi = N.hi;
      }
      base += N.len;
    }
    return slot;
  }
  // unlist(block, transform) (simulation.jl:110-163): lane e holds element e
  __device__ __forceinline__ static void unlist(const DBlock& B, const St& s, int lane, double* x) {
    x[0] = 0.0;
    if (lane < B.d) {
      int lk; double lo, hi;
      const double v = s.cur[elem(s, B, lane, &lk, &lo, &hi)];
      x[0] = B.transform ? mmb_ir_link(lk, v, lo, hi) : v;
    }
  }
  // write x (invlinked when transformed) at the block's slots of dst (and dst2)
  __device__ __forceinline__ static void put(const DBlock& B, const St& s, int lane, const double* x, double* dst,
                                             double* dst2) {
    grp_sync();
    if (lane < B.d) {
      int lk; double lo, hi;
      const int slot = elem(s, B, lane, &lk, &lo, &hi);
      const double v = B.transform ? mmb_ir_invlink(lk, x[0], lo, hi) : x[0];
      dst[slot] = v;
      if (dst2) dst2[slot] = v;
    }
    grp_sync();
  }
  // relist (m[params] = relist(block, x)): the committed state, mirrored into prop
  __device__ __forceinline__ static void relist(const DBlock& B, St& s, const Grp<G>& g, const double* x) {
    put(B, s, g.lane, x, s.cur, s.prop);
  }

#ifndef MMB_IR_LOGF_ATTR
#define MMB_IR_LOGF_ATTR  // logf is called, not inlined (ir_jit.cpp: MMB_IR_LOGF_INLINE)
#endif
#if defined(MMB_IR_JIT) && defined(MMB_IR_SLICEC)
  struct SCtx {  // per-update sums of the candidate-independent MvNormal terms (ir_jit.cpp mmb_jp_<b>)
    double pre[2 * MMB_IR_SPRE];
  };
#else
  struct SCtx {};
#endif
  struct SMemo {};
  struct Prep {};
#if defined(MMB_IR_JIT) && defined(MMB_IR_SEP)
  // Specialised kernels of schemes with AMWG: blocks whose logpdf! separates by coordinate
  // (engine.cpp ir_sep_table; B.sep) decide every coordinate at once (samplers.h amwg_lanes)
  static constexpr bool AMWG_SEP = true;
#else
  static constexpr bool AMWG_SEP = false;  // samplers.h amwg: sequential path only
#endif
  static constexpr bool AMWG_PROBE = false;  // (the near-threshold test hook is rats-only)
  __device__ __forceinline__ static bool amwg_sep(const DBlock& B) { return B.sep != nullptr; }
  __device__ __forceinline__ static bool slice_cand_ok(const DBlock& B) { return B.d <= SLICE_CAND_D; }
  __device__ __forceinline__ static void slice_cand_prep(const SweepArgs& A, const DBlock& B, const St& s, const Lc&,
                                                         const Grp<G>& g, double*, SCtx& cx) {
#if defined(MMB_IR_JIT) && defined(MMB_IR_SLICEC)
    mmb_jit_slice_prep(A, B.ir_blk, s.cur, g, cx.pre);
#else
    (void)A; (void)B; (void)s; (void)g; (void)cx;
#endif
  }
  // logf at the start of a Slice update, after slice_cand_prep: blocks with candidate-independent
  // MvNormal terms take their sums of squares from the prep (ir_jit.cpp mmb_jit_block_lp_pre)
  __device__ __forceinline__ static double slice_logf0(const SweepArgs& A, const DBlock& B, const St& s, const Lc& l,
                                                       const Grp<G>& g, const double* x, const SCtx& cx) {
#if defined(MMB_IR_JIT) && defined(MMB_IR_SLICEC)
    if (mmb_jit_slice_has_pre(B.ir_blk)) {
      put(B, s, g.lane, x, s.prop, nullptr);
      return mmb_jit_block_lp_pre(A, B.ir_blk, s.prop, g, B.transform, cx.pre);
    }
#else
    (void)cx;
#endif
    return logf(A, B, s, l, g, x);
  }
  // logpdf!(m, x, block) at the candidate xv (this lane's 8-lane group's), as logf: xv relisted
  // (invlinked when transformed, put()) into the coordinates' state values
  __device__ __forceinline__ static double slice_cand_logf(const SweepArgs& A, const DBlock& B, const St& s,
                                                           const SCtx& cx, const double* xv, int lane, SMemo&) {
#if defined(MMB_IR_JIT) && defined(MMB_IR_SLICEC)
    double c[SLICE_CAND_D];
#pragma unroll
    for (int a = 0; a < SLICE_CAND_D; ++a) {
      c[a] = 0.0;
      if (a < B.d) {
        int lk;
        double lo, hi;
        (void)elem(s, B, a, &lk, &lo, &hi);
        c[a] = B.transform ? mmb_ir_invlink(lk, xv[a], lo, hi) : xv[a];
      }
    }
    return mmb_jit_slice_cand(A, B.ir_blk, s.cur, c, lane & (32 / SLICE_NC - 1), B.transform, cx.pre);
#else
    (void)A; (void)B; (void)s; (void)cx; (void)xv; (void)lane;
    return 0.0;
#endif
  }
  __device__ __forceinline__ static double amwg_epsf(const DBlock& B) { return B.sep_eps; }
  // Lane j: d_j = sum over the element terms that read coordinate j of w_t (e' - e), the exact
  // difference of coordinate j's two logpdf! evaluations in amwg_sub! (the other terms are equal in
  // both, whatever the other coordinates' accept history); w_t = 1, or -0.5 / sigma^2 for an
  // MvNormal term (d_iso is affine in the sum of squares).  Every candidate is written into `prop`
  // at once: an element reads at most one coordinate, so its term there is its term with only
  // that coordinate moved.  epsm_j = M + sum_j |w| (|e'| + |e|) + |d_j|, M the sum over every element
  // term of |w| max(|e|, |e'|) plus the MvNormal constants: each rounded logf is within
  // (elements per lane + 5 + nterms + 3) u M of its exact value, and B.sep_eps is 8x that.
  __device__ static void amwg_dm(const SweepArgs& A, const DBlock& B, const Prep&, const St& s, const Lc&,
                                 const Grp<G>& g, double x0, double x1, double& del, double& epsm, bool& bad) {
    (void)x0;
#if defined(MMB_IR_JIT) && defined(MMB_IR_SEP)
    const double xx[1] = {x1};
    put(B, s, g.lane, xx, s.prop, nullptr);
    const int lane = g.lane, d = B.d;
    const int32_t* T = B.sep;
    const mmb_ir_block& IB = ir_const_ref(A.ir_blocks, B.ir_blk);
    // term weights and MvNormal constants, term t on lane t, through the (unused) expression stack
    double mloc = 0.0, nfc = 0.0;
    if (lane < IB.nterms) {
      double w, cst;
      mmb_jit_termw(A, B.ir_blk, lane, s.cur, &w, &cst);
      s.stk[lane] = w;
      mloc = cst;
      nfc = (isfinite(w) && isfinite(cst)) ? 0.0 : 1.0;
    }
    grp_sync();
    double dsum = 0.0, sabs = 0.0;
    bool nf = false;
    if (lane < d) {
      const int q1 = T[lane + 1];
      for (int q = T[lane]; q < q1; ++q) {
        const int ent = T[d + 2 + q];
        const int t = ent >> 24, i = ent & 0xffffff;
        const double w = s.stk[t];
        const double eo = mmb_jit_elem(A, B.ir_blk, t, i, s.cur, B.transform);
        const double en = mmb_jit_elem(A, B.ir_blk, t, i, s.prop, B.transform);
        nf = nf || !isfinite(eo) || !isfinite(en);
        dsum = dsum + w * (en - eo);
        const double aw = fabs(w);
        sabs = sabs + aw * (fabs(en) + fabs(eo));
        mloc = mloc + aw * fmax(fabs(en), fabs(eo));
      }
    }
    for (int q = T[d] + lane; q < T[d + 1]; q += G) {  // element terms that read no coordinate
      const int ent = T[d + 2 + q];
      const int t = ent >> 24, i = ent & 0xffffff;
      const double eo = mmb_jit_elem(A, B.ir_blk, t, i, s.cur, B.transform);
      nfc = isfinite(eo) ? nfc : 1.0;
      mloc = mloc + fabs(s.stk[t]) * fabs(eo);
    }
    g.sum2(mloc, nfc);
    grp_sync();  // the stack slots are free again
    del = dsum;
    epsm = mloc + sabs + fabs(dsum);
    bad = nf || nfc != 0.0 || !isfinite(mloc);
#else
    (void)A; (void)B; (void)s; (void)g; (void)x1;
    del = 0.0;
    epsm = 0.0;
    bad = true;
#endif
  }
#if defined(MMB_IR_JIT) && defined(MMB_IR_SLICEC)
  // Specialised kernels: Slice blocks of up to four coordinates evaluate their shrink candidates
  // four at a time, one per 8-lane group (samplers.h slice_uni_cand / slice_multi_cand), each
  // through the generated mmb_jc_<block> (ir_jit.cpp gen_slice_cand: logf's own summation tree)
  static constexpr bool SLICE_CAND = true;
#else
  static constexpr bool SLICE_CAND = false;  // samplers.h slice_uni: one candidate at a time
#endif
  static constexpr int SLICE_CAND_D = 2;
#ifndef MMB_IR_SLICE_NC
#define MMB_IR_SLICE_NC 4
#endif
  static constexpr int SLICE_NC = MMB_IR_SLICE_NC;  // candidates per round (ir_jit.cpp: 2 or 4)
  __device__ __forceinline__ static Prep prep(const DBlock&, const St&) { return Prep{}; }
  // logpdf!(m, x, block, transform)
  __device__ MMB_IR_LOGF_ATTR static double logf(const SweepArgs& A, const DBlock& B, const St& s, const Lc&, const Grp<G>& g,
                                const double* x) {
    put(B, s, g.lane, x, s.prop, nullptr);
#ifdef MMB_IR_JIT
    return mmb_jit_block_lp(A, B.ir_blk, s.prop, g, B.transform);
#else
    const mmb_ir_block& IB = ir_const_ref(A.ir_blocks, B.ir_blk);
    double lp = 0.0;
    for (int t = 0; t < IB.nterms; ++t) {
      lp += node_lp(A, IB.term[t], s.prop, s.stk, g, IB.trans[t] ? B.transform : 0);
      if (!isfinite(lp)) break;
    }
    return lp;
#endif
  }
  __device__ __forceinline__ static double logf_p(const SweepArgs& A, const DBlock& B, const Prep&, const St& s,
                                                  const Lc& l, const Grp<G>& g, const double* x) {
    return logf(A, B, s, l, g, x);
  }
  __device__ __forceinline__ static void logf_p2(const SweepArgs& A, const DBlock& B, const Prep& c, const St& s,
                                                 const Lc& l, const Grp<G>& g, const double* x, const double* v,
                                                 double& lx, double& lv) {
    lx = logf_p(A, B, c, s, l, g, x);
    lv = logf_p(A, B, c, s, l, g, v);
  }
  // logpdfgrad!(block, x, :forward) (sampler.jl:106-111): Calculus forward differences,
  // epsilon = sqrt(eps()) * max(1, |x_i|); non-finite gradient entries -> 0
  __device__ static double logf_grad(const SweepArgs& A, const DBlock& B, const St& s, const double* x,
                                     double* gr) {
    Grp<G> g;
    const Lc l{};
    const double fx = logf(A, B, s, l, g, x);
    double gi = 0.0;
    for (int e = 0; e < B.d; ++e) {
      const bool own = g.lane == e;
      const double ax = fabs(x[0]);
      const double eps = 0x1p-26 * (isnan(ax) ? ax : (ax > 1.0 ? ax : 1.0));
      double xe[1] = {own ? x[0] + eps : x[0]};
      const double fp = logf(A, B, s, l, g, xe);
      if (own) gi = (fp - fx) / eps;
    }
    gr[0] = (g.lane < B.d && isfinite(gi)) ? gi : 0.0;
    return fx;
  }

  __device__ __forceinline__ static int gibbs_draw_kind(const DBlock&, double* a) { *a = 0.0; return 0; }
  __device__ __forceinline__ static void gibbs(const SweepArgs&, const DBlock&, St&, const Lc&, const Grp<G>&,
                                               const mmb_rng*, const mmb_rng*, const mmb_rng*, double) {}

  // sim[i, :, 1] = unlist(m, true) (mcmc.jl:76-77): monitored nodes in Chains order; logicals
  // are evaluated on the current state (their update! runs after every block, simulation.jl:102)
  __device__ static void write_draws(const SweepArgs& A, const St& s, const Grp<G>& g, int64_t row, int c) {
    grp_sync();
    int col = 0;
    for (int q = 0; q < A.ir_nmon; ++q) {
      const int nid = ir_const_ref(A.ir_mon, q);
      const mmb_ir_node& N = ir_const_ref(A.ir_nodes, nid);
      for (int i = g.lane; i < N.len; i += G) {
#ifdef MMB_IR_JIT
        const double v = N.family == MMB_IR_LOGICAL ? mmb_jit_logical(A, nid, i, s.cur)
#else
        const double v = N.family == MMB_IR_LOGICAL ? ev(A, N.expr[0], i, s.cur, s.stk, g.lane)
#endif
                                                    : (N.fixed ? A.ir_pool + N.off : s.cur + N.off)[i];
        A.draws[(size_t)(row * A.ir_pmon + col + i) * A.K + c] = v;
      }
      col += N.len;
    }
  }
};
