// engine.cpp — host side of libmambahip.so: the C ABI of include/mamba_hip.h.
//
// mmb_run is mcmc_master!/mcmc_worker! (src/model/mcmc.jl:36-83) for every chain of
// this engine's shard: it launches the fused sweep kernel over windows of iterations
// on the engine's stream and copies the kept draws out in Mamba's Chains order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <type_traits>
#include <vector>

#include "device.h"
#include "models.h"
#include "nuts.h"
#include "logistic.h"
#include "ir.h"
#include "ir_jit.h"

#include <rccl/rccl.h>

hipError_t mmb_launch_sweep(int model, unsigned kinds, const SweepArgs& A, hipStream_t st);
hipError_t mmb_launch_order_chains(const OrderArgs& a, hipStream_t st);
hipError_t mmb_launch_pchol_probe(int n, int d, const double* S, double* L, int32_t* pos, int32_t* info,
                                  hipStream_t st);
hipError_t mmb_lg_launch_ctl(const LgArgs& A, int start, int parity, int nbound, int fold, hipStream_t st);
hipError_t mmb_lg_launch_grad(const LgArgs& A, int parity, int nbound, int fold, hipStream_t st);
hipError_t mmb_launch_gr_range(int pmon, int64_t n, int K, const double* draws, double* out,
                               hipStream_t st);
hipError_t mmb_launch_chain_summary(int P, int64_t n, int K, int64_t kg0, int64_t bs, const double* draws,
                                    const double* shift, double* out, hipStream_t st);
hipError_t mmb_launch_order_hist(int P, int j, int64_t n, int K, const double* draws, int nt,
                                 const uint64_t* prefix, int pass, unsigned long long* counts, hipStream_t st);
hipError_t mmb_launch_gr_stats(int pmon, int64_t n, int K, const double* draws, const int32_t* link,
                               const double* shift, double* stats, hipStream_t st);

static thread_local std::string g_last_error;

struct BlockHost {
  mmb_block_spec spec;
  std::vector<double> tuning;
  int d = 0, T = 0, tune_len = 0;
  std::vector<double> sigl;  // AMM chol(Sigma) lower row-major
  bool sigl_diag = false;
  // device
  double *sigma = nullptr, *accept = nullptr, *Mv = nullptr, *Mvv = nullptr, *Ls = nullptr;
  double *nuts = nullptr, *nfr = nullptr, *width = nullptr, *sigl_d = nullptr;
  double* hmc = nullptr;  // HMC/MALA [K][2] epsilon, L
  int32_t *m = nullptr, *flags = nullptr;
  uint8_t* piv = nullptr;
  double* xnext = nullptr;   // AMM carried next proposal [K][DP] (samplers.h amm)
  int64_t* xtag = nullptr;   // AMM [K] tag of the carried proposal
  uint64_t* astat = nullptr; // AMM [K][MMB_AMM_STAT_STRIDE] factorization counters (mmb_amm_stats)
  int32_t* sep_d = nullptr;  // node-IR AMWG: coordinate -> element-term table (ir_sep_table), engine lifetime
  double sep_eps = 0.0;
};

struct mmb_engine {
  mmb_model_spec spec{};
  int device = 0;
  hipStream_t stream = nullptr;
  int model = 0;
  int P = 0, pmon = 0, VS = 0, DP = 0, TP = 0;
  std::vector<BlockHost> blocks;
  unsigned kinds = 0;  // bitmask of sampler kinds in the scheme
  // data
  std::vector<double> x, y, X;
  bool have_data = false;
  double* d_data = nullptr;
  // chains
  int64_t K = 0, chain_offset = 0;
  uint64_t seed = 0;
  int64_t iter = 0;
  double* d_vals = nullptr;
  DBlock* d_blocks = nullptr;
  // logistic (config 4): padded X/y and the NUTS machine state (logistic.h)
  int lg_N = 0, lg_p = 0, lg_rps = 0;
  bool lg_fd = false;  // forward-difference gradient (MMB_GRAD_FORWARD): p + 1 columns per request
  double *lg_X = nullptr, *lg_y = nullptr;
  double *lg_vec = nullptr, *lg_sc = nullptr, *lg_frames = nullptr, *lg_pos = nullptr;
  double *lg_gpart = nullptr, *lg_lpart = nullptr;
  int32_t *lg_iv = nullptr, *lg_count = nullptr, *lg_hcount = nullptr, *lg_s2c = nullptr;
  int64_t* lg_itc = nullptr;
  hipEvent_t lg_cev[2 * MMB_LG_SPLIT_MAX] = {};  // request-count readbacks in flight, 2 per part (run_logistic)
  hipStream_t lg_streamx[MMB_LG_SPLIT_MAX - 1] = {};   // the streams of parts 1.. (part 0: the engine stream)
  hipEvent_t lg_join[MMB_LG_SPLIT_MAX] = {};          // fork / join of the streams
  std::vector<hipEvent_t> evpoolx[MMB_LG_SPLIT_MAX - 1];  // kernel timing events of parts 1..
  int64_t lg_steps = 0;  // gradient steps of the last window
  unsigned long long* lg_ngrad = nullptr;
  int32_t* d_cperm = nullptr;  // lane-group slot -> chain of the 32-lane sweep kernels (order_chains)
  bool cperm_identity = true;
  bool order_fresh = false;    // d_cperm holds a table computed after a window (a host write of the
                               // tune state clears it)
  int64_t order_iter = 0;      // the iteration whose flags d_cperm was computed from
  unsigned long long* d_nstat = nullptr;  // NUTS {updates, depth-cap hits, depth sum}, Slice overflows
                                          // since init_chains
  unsigned long long slice_overflows = 0;  // d_nstat[3] as last reported by mmb_run
  int64_t xepoch = 0;  // bumped by every host write of chain state: invalidates carried AMM proposals
  // draws of the last window
  double* d_draws = nullptr;
  size_t draws_cap = 0;
  int64_t n_kept = 0;
  // node IR (MMB_MODEL_IR): host copies of the lowered model, device tables
  std::vector<mmb_ir_node> ir_nodes;
  std::vector<int32_t> ir_code, ir_mon;
  std::vector<double> ir_const, ir_pool;
  std::vector<mmb_ir_block> ir_blocks;
  int ir_stack = 0;
  mmb_ir_node* d_ir_nodes = nullptr;
  int32_t *d_ir_code = nullptr, *d_ir_mon = nullptr;
  double *d_ir_const = nullptr, *d_ir_pool = nullptr;
  mmb_ir_block* d_ir_blocks = nullptr;
  // node IR specialised kernel (ir_jit.cpp): null when the interpreter kernel runs
  hipModule_t jit_mod = nullptr;
  hipFunction_t jit_fn = nullptr;
  std::string jit_info;
  // timing
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> evpool;  // 2 per launch when time_kernels
  double kernel_ms = 0.0;
  int64_t launches = 0, units = 0;
  std::string err;
};

static int fail(mmb_engine* e, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  if (e) e->err = buf;
  return code;
}

#define HIPCHK(e, call)                                                                  \
  do {                                                                                   \
    hipError_t _st = (call);                                                             \
    if (_st != hipSuccess)                                                               \
      return fail((e), MMB_E_HIP, "%s failed: %s", #call, hipGetErrorString(_st));       \
  } while (0)

static int node_dim(const mmb_model_spec& s, const mmb_ir_model* ir, int node, bool* positive) {
  bool pos = false;
  int d = -1;
  if (s.model == MMB_MODEL_IR) {
    // sampled nodes only: not fixed, not Logical, not a discrete family
    if (ir && node >= 0 && node < ir->nnodes) {
      const mmb_ir_node& n = ir->nodes[node];
      const bool ok = !n.fixed && n.family >= MMB_IR_NORMAL && n.family <= MMB_IR_BETA;
      d = ok ? n.len : -1;
    }
  } else if (s.model == MMB_MODEL_LINE) {
    if (node == MMB_LINE_BETA) d = 2;
    else if (node == MMB_LINE_S2) { d = 1; pos = true; }
  } else if (s.model == MMB_MODEL_RATS) {
    static const int dims[7] = {1, 30, 1, 1, 30, 1, 1};
    static const int posv[7] = {1, 0, 0, 1, 0, 0, 1};
    if (node >= 0 && node < 7) { d = dims[node]; pos = posv[node]; }
  } else if (s.model == MMB_MODEL_LOGISTIC) {
    if (node == MMB_LOGISTIC_BETA) d = s.ncoef;
  }
  if (positive) *positive = pos;
  return d;
}

static int tri(int i) { return i * (i + 1) / 2; }

// ---- node IR: AMWG blocks whose logpdf! separates by coordinate (lane-parallel decisions) ----
// amwg_sub! (amwg.jl:99-115) evaluates logpdf!(m, x, block) once per coordinate.  The block's
// terms (simulation.jl:77-90) are sums over node elements (logpdf_sub, distributionstruct.jl:
// 136-168); when every element's term reads at most one coordinate of the block -- through the
// node's own value or a parameter expression's VAL / VALI / VALG slot -- coordinate j's two
// evaluations differ exactly in the terms of the elements that read j, whatever the accept
// history of the other coordinates, so every coordinate's difference can be formed at once (ir.h
// amwg_dm, samplers.h amwg_lanes).  The table lists, per coordinate, the (term, element) pairs
// that read it, then the pairs that read none; an MvNormal term's sigma must read none.  The
// gather indices are data, so this is built per engine at upload, not in the JIT source.
static void ir_expr_slots(const std::vector<int32_t>& code, const std::vector<double>& pool, int pc, int i,
                          std::vector<int>& slots) {
  for (;; ++pc) {
    const int w = code[pc];
    const int op = (int)((uint32_t)w >> 24), arg = w & 0xffffff;
    if (op == MMB_IR_OP_END) return;
    if (op == MMB_IR_OP_VAL) slots.push_back(arg);
    else if (op == MMB_IR_OP_VALI) slots.push_back(arg + i);
    else if (op == MMB_IR_OP_VALG) slots.push_back(arg + (int)pool[code[++pc] + i]);
  }
}
static bool ir_sep_table(const std::vector<mmb_ir_node>& nodes, const std::vector<int32_t>& code,
                         const std::vector<double>& pool, const mmb_ir_block& IB, const mmb_block_spec& s,
                         int nvalues, std::vector<int32_t>& tab, double* epsf) {
  std::vector<int> coord((size_t)nvalues, -1);
  int d = 0;
  for (int a = 0; a < s.nnodes; ++a) {
    const mmb_ir_node& N = nodes[s.nodes[a]];
    for (int q = 0; q < N.len; ++q) coord[N.off + q] = d + q;
    d += N.len;
  }
  if (d < 2 || d > 32) return false;
  std::vector<std::vector<int32_t>> lists((size_t)d + 1);
  int nmax = 1;
  size_t total = 0;
  std::vector<int> sl;
  for (int t = 0; t < IB.nterms; ++t) {
    const mmb_ir_node& N = nodes[IB.term[t]];
    const bool iso = N.family == MMB_IR_ISONORMAL;
    if (iso) {  // sigma (at element 0) must not read the block
      sl.clear();
      ir_expr_slots(code, pool, N.expr[1], 0, sl);
      for (int q : sl)
        if (coord[q] >= 0) return false;
    }
    nmax = std::max(nmax, (N.len + 31) / 32);
    for (int i = 0; i < N.len; ++i) {
      sl.clear();
      if (!N.fixed) sl.push_back(N.off + i);
      for (int k = 0; k < (iso ? 1 : 2); ++k)
        if (N.expr[k] >= 0) ir_expr_slots(code, pool, N.expr[k], i, sl);
      int c = -1;
      for (int q : sl) {
        const int cq = coord[q];
        if (cq < 0) continue;
        if (c >= 0 && c != cq) return false;  // two coordinates: not separable
        c = cq;
      }
      lists[c >= 0 ? c : d].push_back((int32_t)((t << 24) | i));
      if (++total > (1u << 16)) return false;
    }
  }
  tab.assign((size_t)d + 2, 0);
  for (int j = 0; j <= d; ++j) {
    tab[(size_t)j + 1] = tab[j] + (int32_t)lists[j].size();
  }
  for (int j = 0; j <= d; ++j) tab.insert(tab.end(), lists[j].begin(), lists[j].end());
  // rounding band: each logf is a lane partial of <= nmax element terms, a 5-level butterfly, an
  // MvNormal term's affine map and the sum over the terms, so it is within (nmax + nterms + 8) u
  // of the exact sum of its element terms' magnitudes; 8x that, rounded up to a power of two
  const int n = 8 * (nmax + IB.nterms + 8);
  int e2 = 0;
  while ((1 << e2) < n) ++e2;
  *epsf = std::ldexp(1.0, e2 - 53);
  return true;
}

static int tune_len_of(int kind, int d) {
  switch (kind) {
    case MMB_SAMPLER_AMWG: return 2 + 2 * d;
    case MMB_SAMPLER_AMM: return 4 + 2 * d + 2 * tri(d);
    case MMB_SAMPLER_NUTS: return 9;
    case MMB_SAMPLER_HMC: return 2;   // [epsilon, L]     (HMCTune, hmc.jl:5-10)
    case MMB_SAMPLER_MALA: return 1;  // [epsilon]        (MALATune, mala.jl:5-9)
    default: return 0;
  }
}

static int chol_lower(int d, const double* A, double* L) {  // A column-major
  for (int i = 0; i < d * d; ++i) L[i] = 0.0;
  for (int j = 0; j < d; ++j) {
    double s = A[j * d + j];
    for (int k = 0; k < j; ++k) s -= L[j * d + k] * L[j * d + k];
    if (!(s > 0.0)) return -1;
    double ljj = std::sqrt(s);
    L[j * d + j] = ljj;
    for (int i = j + 1; i < d; ++i) {
      double t = A[j * d + i];
      for (int k = 0; k < j; ++k) t -= L[i * d + k] * L[j * d + k];
      L[i * d + j] = t / ljj;
    }
  }
  return 0;
}

// C linkage comes from the extern "C" declarations in include/mamba_hip.h.

int mmb_abi_version(void) { return MMB_ABI_VERSION; }

const char* mmb_last_error(const mmb_engine* e) {
  if (e && !e->err.empty()) return e->err.c_str();
  return g_last_error.c_str();
}

// Device form of the node IR's expressions: a leaf immediately followed by a binary op
// (postfix "... x leaf op") becomes one fused word MMB_IR_FUSED + 4 (leaf - 1) + (op - ADD)
// with the leaf's argument (VALG keeps its second word): acc = acc op leaf instead of
// spill, load, reload -- the same operands in the same order, so results are bit-identical
// to the oracle, which interprets the unfused code.  Each distinct expression start is
// rewritten once (validated code: every expression ends in END); node offsets are remapped.
static void ir_fuse(const std::vector<int32_t>& code, std::vector<mmb_ir_node>& nodes, std::vector<int32_t>& out) {
  std::map<int32_t, int32_t> start;
  auto op_of = [&](size_t pc) { return (int)((uint32_t)code[pc] >> 24); };
  for (mmb_ir_node& N : nodes)
    for (int k = 0; k < 3; ++k) {
      const int32_t s0 = N.expr[k];
      if (s0 < 0) continue;
      auto it = start.find(s0);
      if (it == start.end()) {
        const int32_t ns = (int32_t)out.size();
        start[s0] = ns;
        for (size_t pc = (size_t)s0;; ++pc) {
          const int op = op_of(pc);
          out.push_back(code[pc]);
          if (op == MMB_IR_OP_END) break;
          if (op >= 1 && op < 16) {
            const size_t nx = pc + (op == MMB_IR_OP_VALG ? 2 : 1);
            const int bo = op_of(nx);
            if (bo >= MMB_IR_OP_ADD && bo <= MMB_IR_OP_DIV) {
              out.back() = (int32_t)(((uint32_t)(MMB_IR_FUSED + 4 * (op - 1) + (bo - MMB_IR_OP_ADD)) << 24) |
                                     ((uint32_t)code[pc] & 0xffffffu));
              if (op == MMB_IR_OP_VALG) out.push_back(code[pc + 1]);
              pc = nx;  // the binary op is folded in
              continue;
            }
            if (op == MMB_IR_OP_VALG) out.push_back(code[++pc]);
          }
        }
        it = start.find(s0);
      }
      N.expr[k] = it->second;
    }
}

static int create_impl(const mmb_model_spec* spec, const mmb_ir_model* ir, int device, mmb_engine** out) {
  if (!spec || !out) return fail(nullptr, MMB_E_ARG, "null argument");
  *out = nullptr;
  if (spec->nblocks < 1 || spec->nblocks > MMB_MAX_BLOCKS)
    return fail(nullptr, MMB_E_ARG, "nblocks must be in 1..%d", MMB_MAX_BLOCKS);
  mmb_engine* e = new mmb_engine();
  e->spec = *spec;
  e->model = spec->model;
  if (e->model == MMB_MODEL_RATS) {
    e->P = 65; e->pmon = 3; e->VS = Mdl<MMB_MODEL_RATS>::VS;
    e->DP = Mdl<MMB_MODEL_RATS>::DP; e->TP = Mdl<MMB_MODEL_RATS>::TP;
  } else if (e->model == MMB_MODEL_LINE) {
    e->P = 3; e->pmon = 3; e->VS = Mdl<MMB_MODEL_LINE>::VS;
    e->DP = Mdl<MMB_MODEL_LINE>::DP; e->TP = Mdl<MMB_MODEL_LINE>::TP;
  } else if (e->model == MMB_MODEL_IR) {
    if (!ir) {
      delete e;
      return fail(nullptr, MMB_E_ARG, "node-IR models are created with mmb_create_ir");
    }
    e->P = ir->nvalues;
    e->pmon = 0;
    for (int q = 0; q < ir->nmon; ++q) e->pmon += ir->nodes[ir->mon[q]].len;
    e->VS = (ir->nvalues + 31) / 32 * 32;
    e->DP = Mdl<MMB_MODEL_IR>::DP; e->TP = Mdl<MMB_MODEL_IR>::TP;
    e->ir_nodes.assign(ir->nodes, ir->nodes + ir->nnodes);
    e->ir_code.assign(ir->code, ir->code + ir->ncode);
    e->ir_const.assign(ir->consts, ir->consts + ir->nconst);
    e->ir_pool.assign(ir->pool, ir->pool + ir->npool);
    e->ir_mon.assign(ir->mon, ir->mon + ir->nmon);
    e->ir_blocks.assign(ir->blocks, ir->blocks + spec->nblocks);
    e->ir_stack = ir->stack;
    e->have_data = true;  // the pool carries the data
  } else if (e->model == MMB_MODEL_LOGISTIC) {
    if (spec->ncoef < 1 || spec->ncoef > MMB_LG_DV || spec->nobs < 1 || !(spec->prior_sd > 0.0)) {
      delete e;
      return fail(nullptr, MMB_E_ARG, "logistic: need 1 <= ncoef <= %d, nobs >= 1, prior_sd > 0", MMB_LG_DV);
    }
    const int k0 = spec->blocks[0].sampler;
    if (spec->nblocks != 1 || !(k0 == MMB_SAMPLER_NUTS || k0 == MMB_SAMPLER_HMC || k0 == MMB_SAMPLER_MALA)) {
      delete e;
      return fail(nullptr, MMB_E_UNSUPPORTED,
                  "logistic: only the [NUTS(:beta)], [HMC(:beta, ...)] and [MALA(:beta, ...)] schemes are lowered");
    }
    e->P = spec->ncoef; e->pmon = spec->ncoef; e->VS = MMB_LG_DV; e->DP = MMB_LG_DV; e->TP = 0;
    e->lg_N = spec->nobs; e->lg_p = spec->ncoef; e->lg_rps = mmb_lg_rps(spec->nobs);
  } else {
    delete e;
    return fail(nullptr, MMB_E_UNSUPPORTED, "unknown model kind %d", spec->model);
  }
  for (int b = 0; b < spec->nblocks; ++b) {
    const mmb_block_spec& s = spec->blocks[b];
    BlockHost h;
    h.spec = s;
    if (s.nnodes < 1 || s.nnodes > MMB_MAX_NODES_PER_BLOCK) {
      delete e;
      return fail(nullptr, MMB_E_ARG, "block %d: bad node count", b);
    }
    int d = 0, nvec = 0;
    for (int a = 0; a < s.nnodes; ++a) {
      for (int a2 = 0; a2 < a; ++a2)
        if (s.nodes[a2] == s.nodes[a]) {
          delete e;
          return fail(nullptr, MMB_E_ARG, "block %d: repeated node", b);
        }
      int nd = node_dim(*spec, ir, s.nodes[a], nullptr);
      if (nd < 0) {
        delete e;
        return fail(nullptr, MMB_E_ARG, "block %d: node id %d invalid for model", b, s.nodes[a]);
      }
      if (nd > 1) nvec++;
      d += nd;
    }
    if (s.dim != 0 && s.dim != d) {
      delete e;
      return fail(nullptr, MMB_E_ARG, "block %d: dim %d != unlisted length %d", b, s.dim, d);
    }
    h.d = d;
    h.T = tri(d);
    if (e->model == MMB_MODEL_IR && d > Mdl<MMB_MODEL_IR>::DMAX) {
      delete e;
      return fail(nullptr, MMB_E_UNSUPPORTED, "node IR: block %d has %d elements (max %d)", b, d,
                  Mdl<MMB_MODEL_IR>::DMAX);
    }
    if (e->model == MMB_MODEL_RATS && nvec > 0 && (s.nnodes != 1)) {
      delete e;
      return fail(nullptr, MMB_E_UNSUPPORTED, "rats: alpha/beta must form their own block");
    }
    if (s.ntuning > 0) h.tuning.assign(s.tuning, s.tuning + s.ntuning);
    // logpdfgrad! scheme of gradient samplers (mmb_gradient): forward differences where the
    // model supports them (line, node IR), the analytic gradient on line and logistic
    if (s.sampler == MMB_SAMPLER_NUTS || s.sampler == MMB_SAMPLER_HMC || s.sampler == MMB_SAMPLER_MALA) {
      const int gr = s.gradient;
      // logistic: the reference's default dtype=:forward (Calculus forward differences,
      // simulation.jl:47-51) runs as p + 1 log-density columns per request through the batched
      // MFMA kernel (logistic.hip lg_grad_kernel<.., LPONLY>, lg_assemble_fd)
      if (e->model == MMB_MODEL_LOGISTIC) e->lg_fd = gr == MMB_GRAD_FORWARD;
      const bool ok = gr == MMB_GRAD_DEFAULT || gr == MMB_GRAD_FORWARD ||
                      (gr == MMB_GRAD_ANALYTIC && e->model != MMB_MODEL_IR);
      if (!ok) {
        delete e;
        return fail(nullptr, MMB_E_ARG, "block %d: gradient %d is not available for this model", b, gr);
      }
    }
    switch (s.sampler) {
      case MMB_SAMPLER_AMWG:
        if (!(s.ntuning == 1 || s.ntuning == d)) {
          delete e;
          return fail(nullptr, MMB_E_ARG, "length(sigma) differs from variate length %d", d);
        }
        if (s.batchsize <= 0) { delete e; return fail(nullptr, MMB_E_ARG, "batchsize must be positive"); }
        break;
      case MMB_SAMPLER_AMM: {
        if (s.ntuning != d * d) {
          delete e;
          return fail(nullptr, MMB_E_ARG, "Sigma dimension differs from variate length %d", d);
        }
        h.sigl.resize((size_t)d * d);
        if (chol_lower(d, s.tuning, h.sigl.data())) {
          delete e;
          return fail(nullptr, MMB_E_ARG, "AMM Sigma is not positive definite");
        }
        h.sigl_diag = true;
        for (int i = 0; i < d; ++i)
          for (int k = 0; k < i; ++k)
            if (h.sigl[i * d + k] != 0.0) h.sigl_diag = false;
        break;
      }
      case MMB_SAMPLER_SLICE:
        if (!(s.ntuning == 1 || s.ntuning == d)) {
          delete e;
          return fail(nullptr, MMB_E_ARG, "length(width) differs from variate length %d", d);
        }
        break;
      case MMB_SAMPLER_GIBBS:
        if (e->model == MMB_MODEL_IR) {
          delete e;
          return fail(nullptr, MMB_E_UNSUPPORTED, "Gibbs (user Sampler closures) cannot be lowered to the node IR");
        }
        if (s.nnodes != 1) {
          delete e;
          return fail(nullptr, MMB_E_UNSUPPORTED, "Gibbs: one node per block");
        }
        break;
      case MMB_SAMPLER_NUTS:
        if (e->model == MMB_MODEL_RATS) {
          delete e;
          return fail(nullptr, MMB_E_UNSUPPORTED, "NUTS for the rats model is not lowered in this version");
        }
        break;
      case MMB_SAMPLER_HMC:
      case MMB_SAMPLER_MALA:  // validate(v) (hmc.jl:33-42, mala.jl:28-37)
        if (e->model == MMB_MODEL_RATS) {
          delete e;
          return fail(nullptr, MMB_E_UNSUPPORTED, "HMC/MALA for the rats model is not lowered in this version");
        }
        if (s.ntuning != 0) {
          if (s.ntuning != d * d) {
            delete e;
            return fail(nullptr, MMB_E_ARG, "Sigma dimension differs from variate length %d", d);
          }
          h.sigl.resize((size_t)d * d);
          if (chol_lower(d, s.tuning, h.sigl.data())) {
            delete e;
            return fail(nullptr, MMB_E_ARG, "PosDefException: Sigma is not positive definite");
          }
        }
        break;
      default:
        delete e;
        return fail(nullptr, MMB_E_ARG, "unknown sampler kind %d", s.sampler);
    }
    h.tune_len = tune_len_of(s.sampler, d);
    e->kinds |= 1u << s.sampler;
    e->blocks.push_back(h);
  }
  hipError_t st = hipSetDevice(device);
  if (st != hipSuccess) {
    delete e;
    return fail(nullptr, MMB_E_HIP, "hipSetDevice(%d): %s", device, hipGetErrorString(st));
  }
  e->device = device;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess) {
    delete e;
    return fail(nullptr, MMB_E_HIP, "stream/event creation failed");
  }
  if (e->model == MMB_MODEL_IR) {  // device copies of the IR tables (read-only for every launch)
    bool ok = true;
    auto up = [&](auto** dst, const auto& v) {
      using T = typename std::remove_reference<decltype(v)>::type::value_type;
      if (!ok) return;
      ok = hipMalloc((void**)dst, std::max<size_t>(v.size(), 1) * sizeof(T)) == hipSuccess &&
           (v.empty() || hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess);
    };
    {  // device code: every expression with its leaf+binop pairs fused (ir_fuse), padded
       // with END words (the interpreter fetches one word ahead, ir.h ev)
      std::vector<mmb_ir_node> nodes(e->ir_nodes);
      std::vector<int32_t> code;
      ir_fuse(e->ir_code, nodes, code);
      code.resize(code.size() + 2, 0);
      up(&e->d_ir_nodes, nodes);
      up(&e->d_ir_code, code);
    }
    up(&e->d_ir_const, e->ir_const);
    up(&e->d_ir_pool, e->ir_pool);
    up(&e->d_ir_mon, e->ir_mon);
    up(&e->d_ir_blocks, e->ir_blocks);
    // AMWG blocks whose logpdf! separates by coordinate: lane-parallel decisions in the specialised
    // kernel (MMB_IR_SEP=0 keeps every block on amwg_sub!'s sequential loop)
    const char* se = std::getenv("MMB_IR_SEP");
    const bool sep_on = !(se && std::string(se) == "0");
    for (size_t b = 0; sep_on && b < e->blocks.size(); ++b) {
      BlockHost& h = e->blocks[b];
      std::vector<int32_t> tab;
      if (h.spec.sampler == MMB_SAMPLER_AMWG &&
          ir_sep_table(e->ir_nodes, e->ir_code, e->ir_pool, e->ir_blocks[b], h.spec, e->P, tab, &h.sep_eps))
        up(&h.sep_d, tab);
    }
    if (!ok) {
      mmb_destroy(e);
      return fail(nullptr, MMB_E_HIP, "node IR upload failed");
    }
  }
  *out = e;
  return 0;
}

int mmb_create(const mmb_model_spec* spec, int device, mmb_engine** out) {
  if (spec && spec->model == MMB_MODEL_IR)
    return fail(nullptr, MMB_E_ARG, "node-IR models are created with mmb_create_ir");
  return create_impl(spec, nullptr, device, out);
}

// Host-side validation of a node IR: every code word, slot, pool range and gather index is
// checked against the node lengths, so no kernel can address outside its LDS row or the pool.
static int ir_check_expr(const mmb_ir_model* ir, int pc, int len, int* depth) {
  int sp = 0, mx = 0;
  for (int steps = 0; steps < ir->ncode + 1; ++steps, ++pc) {
    if (pc < 0 || pc >= ir->ncode) return -1;
    const int w = ir->code[pc];
    const int op = (int)((uint32_t)w >> 24), arg = w & 0xffffff;
    if (op == MMB_IR_OP_END) {
      if (sp != 1) return -1;
      *depth = std::max(*depth, mx);
      return 0;
    }
    if (op < 16) {
      switch (op) {
        case MMB_IR_OP_CONST: if (arg >= ir->nconst) return -1; break;
        case MMB_IR_OP_VAL: if (arg >= ir->nvalues) return -1; break;
        case MMB_IR_OP_VALI: if ((int64_t)arg + len > ir->nvalues) return -1; break;
        case MMB_IR_OP_VALG: {
          if (++pc >= ir->ncode) return -1;
          const int64_t w2 = ir->code[pc];
          if (w2 < 0 || w2 + len > ir->npool) return -1;
          for (int i = 0; i < len; ++i) {
            const double q = ir->pool[w2 + i];
            if (!(q >= 0.0) || q != (double)(int64_t)q || (int64_t)arg + (int64_t)q >= ir->nvalues) return -1;
          }
          break;
        }
        case MMB_IR_OP_DATA: if ((int64_t)arg + len > ir->npool) return -1; break;
        case MMB_IR_OP_DATAS: if ((int64_t)arg >= ir->npool) return -1; break;
        default: return -1;
      }
      ++sp;
      mx = std::max(mx, sp);
    } else if (op < 32) {
      if (op > MMB_IR_OP_DIV || sp < 2) return -1;
      --sp;
    } else if (op > MMB_IR_OP_ABS || sp < 1) {
      return -1;
    }
  }
  return -1;
}

static int ir_validate(const mmb_model_spec* spec, const mmb_ir_model* ir) {
  if (spec->model != MMB_MODEL_IR) return fail(nullptr, MMB_E_ARG, "spec->model must be MMB_MODEL_IR");
  if (ir->nvalues < 1 || ir->nvalues > MMB_IR_MAX_VALUES)
    return fail(nullptr, MMB_E_UNSUPPORTED, "node IR: 1 <= nvalues <= %d", MMB_IR_MAX_VALUES);
  if (ir->nnodes < 1 || !ir->nodes || ir->ncode < 1 || !ir->code || ir->npool < 0 || (ir->npool > 0 && !ir->pool) ||
      ir->nconst < 0 || (ir->nconst > 0 && !ir->consts) || ir->nmon < 0 || (ir->nmon > 0 && !ir->mon))
    return fail(nullptr, MMB_E_ARG, "node IR: missing tables");
  if (ir->npool >= (1 << 24) || ir->nconst >= (1 << 24))  // code-word operands are 24-bit
    return fail(nullptr, MMB_E_UNSUPPORTED, "node IR: pool and constant tables must hold < 2^24 entries");
  if (ir->stack < 1 || ir->stack > MMB_IR_MAX_STACK)
    return fail(nullptr, MMB_E_ARG, "node IR: stack depth must be 1..%d", MMB_IR_MAX_STACK);
  int depth = 0;
  for (int n = 0; n < ir->nnodes; ++n) {
    const mmb_ir_node& N = ir->nodes[n];
    if (N.family < MMB_IR_NORMAL || N.family > MMB_IR_LOGICAL || N.len < 1)
      return fail(nullptr, MMB_E_ARG, "node IR: node %d has a bad family or length", n);
    if (N.family != MMB_IR_LOGICAL) {
      const int64_t end = (int64_t)N.off + N.len;
      if (N.off < 0 || end > (N.fixed ? ir->npool : (int64_t)ir->nvalues))
        return fail(nullptr, MMB_E_ARG, "node IR: node %d values out of range", n);
    }
    if (N.family >= MMB_IR_BINOMIAL && N.family <= MMB_IR_BERNOULLI && !N.fixed)
      return fail(nullptr, MMB_E_UNSUPPORTED, "node IR: discrete node %d must be fixed (observed)", n);
    if (N.cterm >= 0 && (int64_t)N.cterm + N.len > ir->npool)
      return fail(nullptr, MMB_E_ARG, "node IR: node %d constant term out of range", n);
    const int nexpr = N.family == MMB_IR_LOGICAL || N.family == MMB_IR_EXPONENTIAL || N.family == MMB_IR_POISSON ||
                              N.family == MMB_IR_BERNOULLI ? 1 : 2;
    for (int k = 0; k < 3; ++k) {
      if (k >= nexpr) {
        if (N.expr[k] >= 0) return fail(nullptr, MMB_E_ARG, "node IR: node %d has extra parameters", n);
        continue;
      }
      if (ir_check_expr(ir, N.expr[k], N.family == MMB_IR_ISONORMAL && k == 1 ? 1 : N.len, &depth))
        return fail(nullptr, MMB_E_ARG, "node IR: node %d parameter %d has invalid code", n, k);
    }
  }
  if (depth > ir->stack) return fail(nullptr, MMB_E_ARG, "node IR: stack depth %d exceeds %d", depth, ir->stack);
  for (int q = 0; q < ir->nmon; ++q)
    if (ir->mon[q] < 0 || ir->mon[q] >= ir->nnodes) return fail(nullptr, MMB_E_ARG, "node IR: bad monitored node");
  if (spec->nblocks < 1 || spec->nblocks > MMB_MAX_BLOCKS)
    return fail(nullptr, MMB_E_ARG, "nblocks must be in 1..%d", MMB_MAX_BLOCKS);
  for (int b = 0; b < spec->nblocks; ++b) {
    const mmb_ir_block& B = ir->blocks[b];
    if (B.nterms < 1 || B.nterms > MMB_IR_MAX_TERMS) return fail(nullptr, MMB_E_ARG, "node IR: block %d terms", b);
    for (int t = 0; t < B.nterms; ++t)
      if (B.term[t] < 0 || B.term[t] >= ir->nnodes || ir->nodes[B.term[t]].family == MMB_IR_LOGICAL)
        return fail(nullptr, MMB_E_ARG, "node IR: block %d term %d invalid", b, t);
  }
  return 0;
}

// Sampler kinds of the scheme and its widest AMM block (the specialised kernel's parameters)
static void ir_jit_params(const mmb_model_spec* spec, const mmb_ir_model* ir, unsigned* kinds, int* dmax) {
  *kinds = 0;
  *dmax = 0;
  for (int b = 0; b < spec->nblocks; ++b) {
    const mmb_block_spec& s = spec->blocks[b];
    *kinds |= 1u << s.sampler;
    int d = 0;
    for (int a = 0; a < s.nnodes; ++a) d += std::max(0, node_dim(*spec, ir, s.nodes[a], nullptr));
    if (s.sampler == MMB_SAMPLER_AMM) *dmax = std::max(*dmax, d);
  }
  if (*dmax == 0) *dmax = Mdl<MMB_MODEL_IR>::DMAX;  // no AMM block: the factorization is not compiled
}

// The specialised kernel of a node-IR engine (ir_jit.cpp); on any failure the interpreter
// kernel runs (jit_info says why).  MMB_IR_JIT=0 selects the interpreter.
static void ir_jit_setup(mmb_engine* e, const mmb_model_spec* spec, const mmb_ir_model* ir) {
  const char* env = std::getenv("MMB_IR_JIT");
  if (env && std::string(env) == "0") {
    e->jit_info = "interpreter (MMB_IR_JIT=0)";
    return;
  }
  unsigned kinds = 0;
  int dmax = 0;
  ir_jit_params(spec, ir, &kinds, &dmax);
  std::vector<char> code;
  std::string info;
  if (mmb_ir_jit_obtain(mmb_ir_jit_source(*spec, *ir, kinds, dmax), &code, &info)) {
    e->jit_info = "interpreter (specialisation failed: " + info + ")";
    return;
  }
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  hipError_t st = hipSetDevice(e->device);
  if (st == hipSuccess) st = hipModuleLoadData(&mod, code.data());
  if (st == hipSuccess) st = hipModuleGetFunction(&fn, mod, "mmb_ir_jit_kernel");
  if (st != hipSuccess) {
    if (mod) (void)hipModuleUnload(mod);
    e->jit_info = std::string("interpreter (module load failed: ") + hipGetErrorString(st) + ")";
    return;
  }
  e->jit_mod = mod;
  e->jit_fn = fn;
  e->jit_info = "specialised kernel (" + info + ")";
  int namwg = 0, nsep = 0;
  for (const BlockHost& h : e->blocks)
    if (h.spec.sampler == MMB_SAMPLER_AMWG) {
      ++namwg;
      nsep += h.sep_d != nullptr;
    }
  if (namwg) e->jit_info += "; lane-parallel AMWG blocks: " + std::to_string(nsep) + " of " + std::to_string(namwg);
}

int mmb_create_ir(const mmb_model_spec* spec, const mmb_ir_model* ir, int device, mmb_engine** out) {
  if (!spec || !ir || !out) return fail(nullptr, MMB_E_ARG, "null argument");
  int rc = ir_validate(spec, ir);
  if (rc) return rc;
  rc = create_impl(spec, ir, device, out);
  if (rc) return rc;
  ir_jit_setup(*out, spec, ir);
  return 0;
}

int mmb_ir_jit_prebuild(const mmb_model_spec* spec, const mmb_ir_model* ir, char* info, int64_t n) {
  if (!spec || !ir) return fail(nullptr, MMB_E_ARG, "null argument");
  int rc = ir_validate(spec, ir);
  if (rc) return rc;
  unsigned kinds = 0;
  int dmax = 0;
  ir_jit_params(spec, ir, &kinds, &dmax);
  std::vector<char> code;
  std::string msg;
  rc = mmb_ir_jit_obtain(mmb_ir_jit_source(*spec, *ir, kinds, dmax), &code, &msg);
  if (info && n > 0) snprintf(info, (size_t)n, "%s", msg.c_str());
  return rc ? fail(nullptr, MMB_E_UNSUPPORTED, "%s", msg.c_str()) : 0;
}

int mmb_ir_jit_source_text(const mmb_model_spec* spec, const mmb_ir_model* ir, char* buf, int64_t n) {
  if (!spec || !ir) return fail(nullptr, MMB_E_ARG, "null argument");
  int rc = ir_validate(spec, ir);
  if (rc) return rc;
  unsigned kinds = 0;
  int dmax = 0;
  ir_jit_params(spec, ir, &kinds, &dmax);
  const std::string src = mmb_ir_jit_source(*spec, *ir, kinds, dmax);
  if (buf && n > 0) snprintf(buf, (size_t)n, "%s", src.c_str());
  return (int)std::min<size_t>(src.size(), (size_t)INT32_MAX);
}

int mmb_ir_jit_info(const mmb_engine* e, char* buf, int64_t n) {
  if (!e) return fail(nullptr, MMB_E_ARG, "null argument");
  if (buf && n > 0) snprintf(buf, (size_t)n, "%s", e->model == MMB_MODEL_IR ? e->jit_info.c_str() : "not a node-IR engine");
  return e->jit_fn ? 1 : 0;
}

static void free_dev(mmb_engine* e) {
  for (auto& h : e->blocks) {
    void* ptrs[] = {h.sigma, h.accept, h.Mv, h.Mvv, h.Ls, h.nuts, h.nfr, h.width, h.sigl_d, h.hmc, h.m, h.flags,
                    h.piv, h.xnext, h.xtag, h.astat};
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
    h.sigma = h.accept = h.Mv = h.Mvv = h.Ls = h.nuts = h.nfr = h.width = h.sigl_d = h.hmc = nullptr;
    h.m = h.flags = nullptr;
    h.piv = nullptr;
    h.xnext = nullptr;
    h.xtag = nullptr;
    h.astat = nullptr;
  }
  if (e->d_vals) (void)hipFree(e->d_vals);
  if (e->d_blocks) (void)hipFree(e->d_blocks);
  {
    void* lp[] = {e->lg_vec, e->lg_sc, e->lg_frames, e->lg_pos, e->lg_gpart, e->lg_lpart, e->lg_iv,
                  e->lg_count, e->lg_itc, e->lg_s2c};
    for (void* q : lp)
      if (q) (void)hipFree(q);
    e->lg_vec = e->lg_sc = e->lg_frames = e->lg_pos = e->lg_gpart = e->lg_lpart = nullptr;
    e->lg_iv = e->lg_count = e->lg_s2c = nullptr;
    e->lg_itc = nullptr;
    if (e->lg_ngrad) (void)hipFree(e->lg_ngrad);
    e->lg_ngrad = nullptr;
    if (e->d_nstat) (void)hipFree(e->d_nstat);
    e->d_nstat = nullptr;
    if (e->d_cperm) (void)hipFree(e->d_cperm);
    e->d_cperm = nullptr;
    e->cperm_identity = true;
    e->order_fresh = false;
  }
  if (e->d_draws) (void)hipFree(e->d_draws);
  e->d_vals = nullptr;
  e->d_blocks = nullptr;
  e->d_draws = nullptr;
  e->draws_cap = 0;
}

#ifdef MMB_PHASE_PROF
void mmb_prof_dump();
void mmb_prof_dump_line();
#endif

void mmb_destroy(mmb_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
#ifdef MMB_PHASE_PROF
  mmb_prof_dump();
  mmb_prof_dump_line();
#endif
#ifdef MMB_PCHOL_COUNT
  if (e->d_nstat) {
    unsigned long long v[8];
    if (hipMemcpy(v, e->d_nstat, sizeof v, hipMemcpyDeviceToHost) == hipSuccess)
      fprintf(stderr, "MMB_PCHOL exact-path steps %llu\n", v[4]);
  }
#endif
  free_dev(e);
  if (e->d_data) (void)hipFree(e->d_data);
  {
    void* ip[] = {e->d_ir_nodes, e->d_ir_code, e->d_ir_mon, e->d_ir_const, e->d_ir_pool, e->d_ir_blocks};
    for (void* q : ip)
      if (q) (void)hipFree(q);
    for (BlockHost& h : e->blocks)
      if (h.sep_d) (void)hipFree(h.sep_d);
  }
  if (e->lg_X) (void)hipFree(e->lg_X);
  if (e->lg_y) (void)hipFree(e->lg_y);
  if (e->lg_hcount) (void)hipHostFree(e->lg_hcount);
  for (hipEvent_t ev : e->lg_cev)
    if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->lg_join)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& pool : e->evpoolx)
    for (hipEvent_t ev : pool) (void)hipEventDestroy(ev);
  for (hipStream_t q : e->lg_streamx)
    if (q) (void)hipStreamDestroy(q);
  if (e->ev0) (void)hipEventDestroy(e->ev0);
  if (e->ev1) (void)hipEventDestroy(e->ev1);
  for (hipEvent_t ev : e->evpool) (void)hipEventDestroy(ev);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  if (e->jit_mod) (void)hipModuleUnload(e->jit_mod);
  delete e;
}

int mmb_set_data(mmb_engine* e, const char* name, const double* x, int64_t n) {
  if (!e || !name || !x) return fail(e, MMB_E_ARG, "null argument");
  std::string nm(name);
  if (e->model == MMB_MODEL_LINE) {
    if (n != 5) return fail(e, MMB_E_ARG, "line: %s must have 5 elements", name);
    if (nm == "x") e->x.assign(x, x + 5);
    else if (nm == "y") e->y.assign(x, x + 5);
    else return fail(e, MMB_E_ARG, "line: unknown input %s", name);
  } else if (e->model == MMB_MODEL_LOGISTIC) {
    if (nm == "X") {
      if (n != (int64_t)e->lg_N * e->lg_p) return fail(e, MMB_E_ARG, "logistic: X must be nobs x ncoef");
      e->X.assign(x, x + n);
    } else if (nm == "y") {
      if (n != e->lg_N) return fail(e, MMB_E_ARG, "logistic: y must have nobs elements");
      for (int64_t i = 0; i < n; ++i)
        if (!(x[i] == 0.0 || x[i] == 1.0)) return fail(e, MMB_E_ARG, "logistic: y must be 0/1");
      e->y.assign(x, x + n);
    } else {
      return fail(e, MMB_E_ARG, "logistic: unknown input %s", name);
    }
    e->have_data = !e->X.empty() && !e->y.empty();
    if (e->have_data) {  // padded device copies: X [Np][64], y [Np]
      const size_t Np = (size_t)MMB_LG_NG * MMB_LG_NS * e->lg_rps;
      std::vector<double> hx(Np * MMB_LG_DV, 0.0), hy(Np, 0.0);
      for (int i = 0; i < e->lg_N; ++i) {
        for (int k = 0; k < e->lg_p; ++k) {
          hx[(size_t)i * MMB_LG_DV + k] = e->X[(size_t)i * e->lg_p + k];
        }
        hy[i] = e->y[i];
      }
      HIPCHK(e, hipSetDevice(e->device));
      if (!e->lg_X) HIPCHK(e, hipMalloc(&e->lg_X, hx.size() * sizeof(double)));
      if (!e->lg_y) HIPCHK(e, hipMalloc(&e->lg_y, hy.size() * sizeof(double)));
      HIPCHK(e, hipMemcpy(e->lg_X, hx.data(), hx.size() * sizeof(double), hipMemcpyHostToDevice));
      HIPCHK(e, hipMemcpy(e->lg_y, hy.data(), hy.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    return 0;
  } else if (e->model == MMB_MODEL_RATS) {
    if (nm == "y") {
      if (n != 150) return fail(e, MMB_E_ARG, "rats: y must have 150 elements");
      e->y.assign(x, x + 150);
    } else if (nm == "x") {
      if (n != 5) return fail(e, MMB_E_ARG, "rats: x must have 5 elements");
      e->x.assign(x, x + 5);
    } else {
      return fail(e, MMB_E_ARG, "rats: unknown input %s", name);
    }
  }
  e->have_data = !e->x.empty() && !e->y.empty();
  if (e->have_data && e->model == MMB_MODEL_RATS) {
    HIPCHK(e, hipSetDevice(e->device));
    if (!e->d_data) HIPCHK(e, hipMalloc(&e->d_data, 150 * sizeof(double)));
    HIPCHK(e, hipMemcpy(e->d_data, e->y.data(), 150 * sizeof(double), hipMemcpyHostToDevice));
  }
  return 0;
}

int mmb_num_values(const mmb_engine* e) { return e ? e->P : MMB_E_ARG; }
int mmb_num_monitored(const mmb_engine* e) { return e ? e->pmon : MMB_E_ARG; }
int64_t mmb_iter(const mmb_engine* e) { return e ? e->iter : MMB_E_ARG; }
int mmb_set_iter(mmb_engine* e, int64_t iter) {
  if (!e) return fail(e, MMB_E_ARG, "null engine");
  if (!e->d_vals) return fail(e, MMB_E_STATE, "mmb_init_chains not called");
  if (iter < 0 || iter > 0xffffffffLL) return fail(e, MMB_E_ARG, "iteration out of range");
  e->iter = iter;
  ++e->xepoch;
  return 0;
}
int64_t mmb_num_kept(const mmb_engine* e) { return e ? e->n_kept : MMB_E_ARG; }

int64_t mmb_tune_len(const mmb_engine* e) {
  if (!e) return MMB_E_ARG;
  int64_t n = 0;
  for (auto& h : e->blocks) n += h.tune_len;
  return n;
}

// canonical values (K x P) <-> device layout
static void to_device_layout(const mmb_engine* e, const double* v, double* dv) {
  if (e->model == MMB_MODEL_RATS) {
    std::fill(dv, dv + e->VS, 0.0);
    for (int i = 0; i < 30; ++i) { dv[i] = v[1 + i]; dv[32 + i] = v[33 + i]; }
    dv[64] = v[0]; dv[65] = v[31]; dv[66] = v[32]; dv[67] = v[63]; dv[68] = v[64];
  } else if (e->model == MMB_MODEL_LOGISTIC || e->model == MMB_MODEL_IR) {
    std::fill(dv, dv + e->VS, 0.0);
    for (int i = 0; i < e->P; ++i) dv[i] = v[i];
  } else {
    dv[0] = v[0]; dv[1] = v[1]; dv[2] = v[2]; dv[3] = 0.0;
  }
}
static void from_device_layout(const mmb_engine* e, const double* dv, double* v) {
  if (e->model == MMB_MODEL_RATS) {
    for (int i = 0; i < 30; ++i) { v[1 + i] = dv[i]; v[33 + i] = dv[32 + i]; }
    v[0] = dv[64]; v[31] = dv[65]; v[32] = dv[66]; v[63] = dv[67]; v[64] = dv[68];
  } else if (e->model == MMB_MODEL_LOGISTIC || e->model == MMB_MODEL_IR) {
    for (int i = 0; i < e->P; ++i) v[i] = dv[i];
  } else {
    v[0] = dv[0]; v[1] = dv[1]; v[2] = dv[2];
  }
}

int mmb_set_values(mmb_engine* e, const double* values) {
  if (!e || !values) return fail(e, MMB_E_ARG, "null argument");
  if (!e->d_vals) return fail(e, MMB_E_STATE, "mmb_init_chains not called");
  ++e->xepoch;
  std::vector<double> h((size_t)e->K * e->VS);
  for (int64_t k = 0; k < e->K; ++k) to_device_layout(e, values + k * e->P, h.data() + k * e->VS);
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipMemcpy(e->d_vals, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
  return 0;
}

int mmb_get_values(mmb_engine* e, double* values) {
  if (!e || !values) return fail(e, MMB_E_ARG, "null argument");
  if (!e->d_vals) return fail(e, MMB_E_STATE, "mmb_init_chains not called");
  std::vector<double> h((size_t)e->K * e->VS);
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipMemcpy(h.data(), e->d_vals, h.size() * sizeof(double), hipMemcpyDeviceToHost));
  for (int64_t k = 0; k < e->K; ++k) from_device_layout(e, h.data() + k * e->VS, values + k * e->P);
  return 0;
}

static int upload_blocks(mmb_engine* e) {
  std::vector<DBlock> db(e->blocks.size());
  for (size_t b = 0; b < e->blocks.size(); ++b) {
    BlockHost& h = e->blocks[b];
    DBlock& d = db[b];
    std::memset(&d, 0, sizeof d);
    d.kind = h.spec.sampler;
    d.nn = h.spec.nnodes;
    d.d = h.d;
    d.transform = h.spec.sampler == MMB_SAMPLER_SLICE ? h.spec.transform : 1;
    d.form = h.spec.form;
    d.adapt = h.spec.adapt;
    d.batchsize = h.spec.batchsize;
    d.sigl_diag = h.sigl_diag;
    // forward differences (the reference's default) unless the analytic gradient was asked for
    d.fdgrad = h.spec.gradient != MMB_GRAD_ANALYTIC ? 1 : 0;
    for (int a = 0; a < 4; ++a) d.nodes[a] = a < h.spec.nnodes ? h.spec.nodes[a] : -1;
    // line: element -> value index (beta -> 0,1; s2 -> 2)
    int o = 0;
    for (int a = 0; a < h.spec.nnodes && o < 4; ++a) {
      int n = h.spec.nodes[a];
      if (e->model == MMB_MODEL_LINE) {
        if (n == MMB_LINE_BETA) { d.emap[o++] = 0; if (o < 4) d.emap[o++] = 1; }
        else d.emap[o++] = 2;
      } else {
        d.emap[o++] = n;
      }
    }
    d.target = h.spec.target;
    d.beta = h.spec.beta;
    d.scale = h.spec.scale;
    d.width0 = h.tuning.empty() ? 0.0 : h.tuning[0];
    d.width = (h.spec.sampler == MMB_SAMPLER_SLICE && h.tuning.size() > 1) ? h.width : nullptr;
    d.sigl = h.sigl_d;
    d.t_sigma = h.sigma; d.t_accept = h.accept; d.t_m = h.m; d.t_flags = h.flags;
    d.t_Mv = h.Mv; d.t_Mvv = h.Mvv; d.t_Ls = h.Ls; d.t_piv = h.piv; d.t_xnext = h.xnext; d.t_xtag = h.xtag; d.t_nuts = h.nuts; d.t_nfr = h.nfr;
    d.t_astat = h.astat;
    d.t_hmc = h.hmc;
    d.ir_blk = (int32_t)b;
    d.sep = h.sep_d;
    d.sep_eps = h.sep_eps;
  }
  if (!e->d_blocks) HIPCHK(e, hipMalloc(&e->d_blocks, MMB_MAX_BLOCKS * sizeof(DBlock)));
  HIPCHK(e, hipMemcpy(e->d_blocks, db.data(), db.size() * sizeof(DBlock), hipMemcpyHostToDevice));
  return 0;
}

template <class T>
static hipError_t dalloc(T** p, size_t n) {
  return hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T));
}

int mmb_init_chains(mmb_engine* e, const double* init, int64_t K, int64_t chain_offset, uint64_t seed) {
  if (!e || !init) return fail(e, MMB_E_ARG, "null argument");
  if (K < 1 || K > (int64_t)1 << 30) return fail(e, MMB_E_ARG, "K out of range");
  if (chain_offset < 0 || chain_offset + K > ((int64_t)1 << 32))
    return fail(e, MMB_E_ARG, "global chain ids must fit in 32 bits");
  if (!e->have_data) return fail(e, MMB_E_STATE, "inputs must be set before inits");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  free_dev(e);
  e->K = K;
  e->chain_offset = chain_offset;
  e->seed = seed;
  e->iter = 0;
  e->n_kept = 0;
  HIPCHK(e, dalloc(&e->d_vals, (size_t)K * e->VS));
  e->slice_overflows = 0;
  HIPCHK(e, dalloc(&e->d_nstat, 8));  // [4]: pchol32 exact-path steps (-DMMB_PCHOL_COUNT builds)
  HIPCHK(e, hipMemset(e->d_nstat, 0, 8 * sizeof(unsigned long long)));
  const size_t DP = e->DP, TP = e->TP;
  for (auto& h : e->blocks) {
    HIPCHK(e, dalloc(&h.m, K));
    HIPCHK(e, dalloc(&h.flags, K));
    HIPCHK(e, hipMemset(h.m, 0, K * sizeof(int32_t)));
    HIPCHK(e, hipMemset(h.flags, 0, K * sizeof(int32_t)));
    if (h.spec.sampler == MMB_SAMPLER_AMWG) {
      HIPCHK(e, dalloc(&h.sigma, K * DP));
      HIPCHK(e, dalloc(&h.accept, K * DP));
      std::vector<double> sg(K * DP, 0.0);
      for (int64_t k = 0; k < K; ++k)
        for (int i = 0; i < h.d; ++i) sg[k * DP + i] = h.tuning.size() == 1 ? h.tuning[0] : h.tuning[i];
      HIPCHK(e, hipMemcpy(h.sigma, sg.data(), sg.size() * sizeof(double), hipMemcpyHostToDevice));
      HIPCHK(e, hipMemset(h.accept, 0, K * DP * sizeof(double)));
    } else if (h.spec.sampler == MMB_SAMPLER_AMM) {
      HIPCHK(e, dalloc(&h.Mv, K * DP));
      HIPCHK(e, dalloc(&h.Mvv, K * TP));
      HIPCHK(e, dalloc(&h.Ls, K * TP));
      HIPCHK(e, dalloc(&h.piv, K * DP));
      HIPCHK(e, hipMemset(h.Mv, 0, K * DP * sizeof(double)));
      HIPCHK(e, hipMemset(h.Mvv, 0, K * TP * sizeof(double)));
      HIPCHK(e, hipMemset(h.Ls, 0, K * TP * sizeof(double)));
      std::vector<uint8_t> pv(K * DP);
      for (int64_t k = 0; k < K; ++k)
        for (size_t i = 0; i < DP; ++i) pv[k * DP + i] = (uint8_t)i;
      HIPCHK(e, hipMemcpy(h.piv, pv.data(), pv.size(), hipMemcpyHostToDevice));
      HIPCHK(e, dalloc(&h.xnext, K * DP));
      HIPCHK(e, dalloc(&h.xtag, K));
      HIPCHK(e, hipMemset(h.xtag, 0xff, K * sizeof(int64_t)));  // -1: no carried proposal
      HIPCHK(e, dalloc(&h.astat, K * MMB_AMM_STAT_STRIDE));
      HIPCHK(e, hipMemset(h.astat, 0, K * MMB_AMM_STAT_STRIDE * sizeof(uint64_t)));
      HIPCHK(e, dalloc(&h.sigl_d, (size_t)h.d * h.d));
      HIPCHK(e, hipMemcpy(h.sigl_d, h.sigl.data(), h.sigl.size() * sizeof(double), hipMemcpyHostToDevice));
    } else if (h.spec.sampler == MMB_SAMPLER_NUTS) {
      HIPCHK(e, dalloc(&h.nuts, K * 8));
      HIPCHK(e, hipMemset(h.nuts, 0, K * 8 * sizeof(double)));
      if (e->model == MMB_MODEL_LINE) {
        const size_t fr = (size_t)NutsFrames<Mdl<MMB_MODEL_LINE>::G * Mdl<MMB_MODEL_LINE>::R>::DBL;
        HIPCHK(e, dalloc(&h.nfr, K * fr));
      } else if (e->model == MMB_MODEL_IR) {
        const size_t fr = (size_t)NutsFrames<Mdl<MMB_MODEL_IR>::G * Mdl<MMB_MODEL_IR>::R>::DBL;
        HIPCHK(e, dalloc(&h.nfr, K * fr));
      }
    } else if (h.spec.sampler == MMB_SAMPLER_HMC || h.spec.sampler == MMB_SAMPLER_MALA) {
      HIPCHK(e, dalloc(&h.hmc, K * 2));
      std::vector<double> t(K * 2);
      for (int64_t k = 0; k < K; ++k) { t[2 * k] = h.spec.epsilon; t[2 * k + 1] = (double)h.spec.nsteps; }
      HIPCHK(e, hipMemcpy(h.hmc, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
      if (!h.sigl.empty()) {
        HIPCHK(e, dalloc(&h.sigl_d, (size_t)h.d * h.d));
        HIPCHK(e, hipMemcpy(h.sigl_d, h.sigl.data(), h.sigl.size() * sizeof(double), hipMemcpyHostToDevice));
      }
    } else if (h.spec.sampler == MMB_SAMPLER_SLICE && h.tuning.size() > 1) {
      HIPCHK(e, dalloc(&h.width, h.tuning.size()));
      HIPCHK(e, hipMemcpy(h.width, h.tuning.data(), h.tuning.size() * sizeof(double), hipMemcpyHostToDevice));
    }
  }
  if (e->model == MMB_MODEL_LOGISTIC) {
    HIPCHK(e, dalloc(&e->lg_vec, (size_t)K * MMB_LG_NVEC * MMB_LG_DV));
    HIPCHK(e, hipMemset(e->lg_vec, 0, (size_t)K * MMB_LG_NVEC * MMB_LG_DV * sizeof(double)));
    HIPCHK(e, dalloc(&e->lg_sc, (size_t)K * MMB_LG_NSC));
    HIPCHK(e, dalloc(&e->lg_iv, (size_t)K * MMB_LG_NIV));
    HIPCHK(e, hipMemset(e->lg_iv, 0, (size_t)K * MMB_LG_NIV * sizeof(int32_t)));
    HIPCHK(e, dalloc(&e->lg_itc, (size_t)K));
    HIPCHK(e, dalloc(&e->lg_frames, (size_t)K * NutsFrames<MMB_LG_DV>::DBL));
    HIPCHK(e, dalloc(&e->lg_pos, (size_t)K * MMB_LG_DV));
    HIPCHK(e, dalloc(&e->lg_gpart, (size_t)MMB_LG_NG * MMB_LG_NS * K * MMB_LG_DV));
    HIPCHK(e, dalloc(&e->lg_lpart, (size_t)MMB_LG_NG * MMB_LG_NS * K * (e->lg_fd ? e->lg_p + 1 : 1)));
    HIPCHK(e, dalloc(&e->lg_count, 2 * MMB_LG_SPLIT_MAX));
    HIPCHK(e, dalloc(&e->lg_s2c, (size_t)2 * K));
    HIPCHK(e, dalloc(&e->lg_ngrad, 1));
    if (!e->lg_hcount) HIPCHK(e, hipHostMalloc(&e->lg_hcount, 2 * MMB_LG_SPLIT_MAX * sizeof(int32_t), 0));
    for (hipEvent_t& ev : e->lg_cev)
      if (!ev) HIPCHK(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (hipEvent_t& ev : e->lg_join)
      if (!ev) HIPCHK(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (hipStream_t& q : e->lg_streamx)
      if (!q) HIPCHK(e, hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
  }
  int rc = upload_blocks(e);
  if (rc) return rc;
  return mmb_set_values(e, init);
}

static int64_t kept_upto(int64_t t, int64_t burnin, int64_t thin) {
  return t > burnin ? (t - burnin) / thin : 0;
}

static void fill_args(const mmb_engine* e, SweepArgs& A) {
  std::memset(&A, 0, sizeof A);
  A.K = (int32_t)e->K;
  A.chain_offset = (uint32_t)e->chain_offset;
  A.seed = e->seed;
  A.nb = (int32_t)e->blocks.size();
  A.vals = e->d_vals;
  A.xepoch = e->xepoch;
  A.nuts_stat = e->d_nstat;
  A.ig_c = 0.001 * std::log(0.001) - std::lgamma(0.001);
  A.blocks = e->d_blocks;
  A.cperm = e->cperm_identity ? nullptr : e->d_cperm;
  {  // MMB_AMWG_EXACT=1: AMWG updates by amwg_sub!'s sequential loop; 2: wide AMWG band.
     // MMB_SLICE_EXACT=1: Slice shrink candidates one at a time.  MMB_AMWG_PROBE=1: tests only.
    const char* ae = std::getenv("MMB_AMWG_EXACT");
    const int v = ae ? std::atoi(ae) : 0;
    A.amwg_exact = (v == 1 || v == 2) ? v : 0;
    const char* se = std::getenv("MMB_SLICE_EXACT");
    A.slice_exact = (se && std::atoi(se) == 1) ? 1 : 0;
    const char* ap = std::getenv("MMB_AMWG_PROBE");
    A.amwg_probe = (ap && std::atoi(ap) == 1) ? 1 : 0;
  }
  if (e->model == MMB_MODEL_IR) {
    A.ir_nodes = e->d_ir_nodes; A.ir_code = e->d_ir_code; A.ir_const = e->d_ir_const;
    A.ir_pool = e->d_ir_pool; A.ir_blocks = e->d_ir_blocks; A.ir_mon = e->d_ir_mon;
    A.ir_nmon = (int32_t)e->ir_mon.size();
    A.ir_pmon = e->pmon;
    A.ir_vs = e->VS;
    A.ir_amm = (e->kinds & (1u << MMB_SAMPLER_AMM)) ? Mdl<MMB_MODEL_IR>::AMM_DBL : 0;
    A.ir_lds = A.ir_amm + 2 * e->VS + (e->ir_stack + 1) * Mdl<MMB_MODEL_IR>::G;
  } else if (e->model == MMB_MODEL_RATS) {
    double s = 0.0;
    for (int i = 0; i < 5; ++i) s += e->x[i];
    A.xbar = s / 5.0;
    for (int i = 0; i < 5; ++i) A.xm[i] = e->x[i] - A.xbar;
    A.data0 = e->d_data;
  } else {
    for (int i = 0; i < 5; ++i) { A.lx[i] = e->x[i]; A.ly[i] = e->y[i]; }
  }
}

static int iters_per_launch(const mmb_engine* e) {
  const char* s = std::getenv("MMB_ITERS_PER_LAUNCH");
  if (s && std::atoi(s) > 0) return std::atoi(s);
  // rats: 20 (16384 chains: ~2.5 ms launches; 16 was 0.5-0.9 % over 8 and 6 % over 4 in the
  // round-4 A/B, the launch tail amortised; round 5: 20 as fast as 16 and 32 over 400 steps, and a
  // 20-iteration window runs as one launch: 1.226e8 vs 1.21e8 for 10 + 10); line: 256 (an
  // iteration of the quad kernel is ~8 us, so 64 per launch left a launch gap every ~0.5 ms)
  return e->model == MMB_MODEL_RATS ? 20 : e->model == MMB_MODEL_IR ? 16 : e->model == MMB_MODEL_LINE ? 256 : 64;
}

template <class T>
static int d2h(mmb_engine* e, std::vector<T>& h, const T* d, size_t n) {
  h.resize(n);
  HIPCHK(e, hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
  return 0;
}
template <class T>
static int h2d(mmb_engine* e, T* d, const std::vector<T>& h) {
  HIPCHK(e, hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

// Wavefront pairing of the 32-lane kernels (two chains per wavefront step together): a chain whose
// AMM moment matrix is indefinite stops its pivoted Cholesky after a few pivots every update
// (the amm.jl:102 alias leaves about half the chains so, persistently), but its
// wavefront runs until the partner chain has finished.  Before a window the engine orders the
// chains by class -- for each AMM block, whether the chain has a valid factor (flags bit 2) --
// so chains that stop alike share wavefronts; the kernel maps lane-group slot -> chain through
// the table (sweep.h), and every chain keeps its own state, draws column and Philox id, so the
// results are identical for any order.  The table is a stable counting sort computed on the
// device (sweep.hip order_chains_kernel), queued on the engine stream behind the previous
// window: no synchronisation, no copy and no host work per call.  MMB_ORDER_CHAINS=0 keeps the
// identity.
static int order_chains(mmb_engine* e) {
  e->cperm_identity = true;
  if (!(e->model == MMB_MODEL_RATS || e->model == MMB_MODEL_IR) || e->K < 4) return 0;
  const char* env = std::getenv("MMB_ORDER_CHAINS");
  if (env && std::string(env) == "0") return 0;
  OrderArgs oa;
  std::memset(&oa, 0, sizeof oa);
  for (const BlockHost& h : e->blocks)
    if (h.spec.sampler == MMB_SAMPLER_AMM && h.flags && oa.nblk < MMB_ORDER_BLOCKS) oa.flags[oa.nblk++] = h.flags;
  if (oa.nblk == 0) return 0;
  if (!e->d_cperm) HIPCHK(e, dalloc(&e->d_cperm, (size_t)e->K));
  oa.K = (int32_t)e->K;
  oa.perm = e->d_cperm;
  // chains per workgroup of the 32-lane sweep kernels (sweep.hip launch: rats 256 threads, node IR 128)
  oa.cpw = e->model == MMB_MODEL_RATS ? 8 : 4;
  {
    // default 1, slow classes first: the launch's second dispatch round then ends on the fast
    // ones (20-iteration windows: 1.17-1.18e8 -> 1.20-1.21e8 chain-updates/s; balanced
    // workgroups, mode 2, 1.12-1.13e8)
    const char* om = std::getenv("MMB_ORDER_MODE");
    oa.mode = om ? std::atoi(om) : 1;
    if (oa.mode < 0 || oa.mode > 2) oa.mode = 1;
  }
  hipError_t st = mmb_launch_order_chains(oa, e->stream);
  if (st != hipSuccess) return fail(e, MMB_E_HIP, "order_chains launch: %s", hipGetErrorString(st));
  e->cperm_identity = false;
  return 0;
}

static int64_t order_every() {
  const char* s = std::getenv("MMB_ORDER_EVERY");
  return (s && std::atoi(s) > 0) ? std::atoi(s) : 64;
}

// Launch widths of a window: ceil(iters / W) launches of equal length (+-1), so a window of 20
// iterations at W = 16 runs 10 + 10 instead of 16 + 4 (a short launch pays the launch tail on
// few iterations)
static int launch_width(int64_t iters, int W, int64_t li) {
  const int64_t nl = (iters + W - 1) / W;
  const int64_t q = iters / nl, r = iters % nl;
  return (int)(q + (li < r ? 1 : 0));
}


// Config-4 window: ctl / grad kernel pairs until no chain requests a gradient.  The
// request count is read back every LG_CHECK steps (pinned host words, one check behind the
// launches); surplus pairs after the last chain finished are no-ops (the grad kernel exits on
// count 0, idle chains return).
//
// The chains run as independent parts (default 3, MMB_LG_SPLIT=1..4), each on its own stream
// with its own request list, partial buffers and count words: a step is a latency-bound control
// kernel (one wave per chain, little arithmetic) behind an MFMA gradient kernel, and the other
// part's gradient kernel fills the GPU while one part is in its control kernel (and the window's
// tail, where few chains still run, overlaps across the parts).  Every chain keeps its own state,
// Philox id and draws column, so the draws are identical for any split.
#ifndef MMB_LG_FOLD_MIN
#define MMB_LG_FOLD_MIN 1024  // chains: 16 tiles x 32 groups = 512 workgroups
#endif
static int run_logistic(mmb_engine* e, const mmb_run_args* a, double* draws, int64_t kept0, int64_t nk,
                        bool want) {
  constexpr int LG_CHECK = 8;
  const BlockHost& h = e->blocks[0];
  LgArgs A0;
  std::memset(&A0, 0, sizeof A0);
  A0.K = (int32_t)e->K; A0.p = e->lg_p; A0.N = e->lg_N; A0.rps = e->lg_rps;
  A0.Np = MMB_LG_NG * MMB_LG_NS * e->lg_rps;
  A0.chain_offset = (uint32_t)e->chain_offset;
  A0.seed = e->seed;
  A0.iter0 = e->iter;
  A0.it_end = e->iter + a->iters;
  A0.burnin = a->burnin; A0.thin = a->thin; A0.model_burnin = a->model_burnin; A0.kept_origin = kept0;
  A0.prior_sd = e->spec.prior_sd;
  A0.target = h.spec.target;
  A0.X = e->lg_X; A0.y = e->lg_y;
  A0.vals = e->d_vals; A0.vec = e->lg_vec; A0.sc = e->lg_sc; A0.iv = e->lg_iv; A0.itc = e->lg_itc;
  A0.kind = h.spec.sampler;
  A0.frames = e->lg_frames; A0.tm = h.m; A0.tflags = h.flags;
  A0.tune = A0.kind == MMB_SAMPLER_NUTS ? h.nuts : h.hmc;
  const int tune_w = A0.kind == MMB_SAMPLER_NUTS ? 8 : 2;
  A0.sigl = h.sigl_d;
  A0.draws = draws;
  A0.Kd = (int32_t)e->K;
  A0.pos = e->lg_pos; A0.gpart = e->lg_gpart; A0.lpart = e->lg_lpart; A0.count = e->lg_count; A0.s2c = e->lg_s2c;
  A0.ngrad = e->lg_ngrad;
  A0.nstat = e->d_nstat;
  A0.fd = e->lg_fd ? 1 : 0;
  A0.nv = e->lg_fd ? e->lg_p + 1 : 1;
  // default 3 parts: 1.34e6 chain-updates/s on config 4 vs 1.28e6 (2), 1.11e6 (4), 1.12e6 (1)
  int nh = 3;
  if (const char* hs = std::getenv("MMB_LG_SPLIT")) nh = std::max(1, std::min(MMB_LG_SPLIT_MAX, std::atoi(hs)));
  if (e->K < 32 * nh) nh = 1;
  struct Half {
    LgArgs A;
    hipStream_t st;
    std::vector<hipEvent_t>* ev;
    int64_t s = 0;
    int nbound = 0;
    bool done = false;
  } H[MMB_LG_SPLIT_MAX];
  for (int i = 0; i < nh; ++i) {
    // chains [b, b + k) of the engine: every per-chain array offset by b rows, the partial and
    // request buffers split in proportion (each half indexes them with its own K)
    const int64_t b = e->K * i / nh, k = e->K * (i + 1) / nh - b;
    LgArgs& A = H[i].A;
    A = A0;
    A.K = (int32_t)k;
    A.Kv = k * A.nv;
    A.chain_offset = (uint32_t)(e->chain_offset + b);
    A.vals += b * MMB_LG_DV; A.vec += b * MMB_LG_NVEC * MMB_LG_DV; A.sc += b * MMB_LG_NSC;
    A.iv += b * MMB_LG_NIV; A.itc += b; A.frames += b * NutsFrames<MMB_LG_DV>::DBL;
    A.tune += b * tune_w; A.tm += b; A.tflags += b;
    if (A.draws) A.draws += b;
    A.pos += b * MMB_LG_DV;
    A.gpart += (size_t)MMB_LG_NG * MMB_LG_NS * b * MMB_LG_DV;
    A.lpart += (size_t)MMB_LG_NG * MMB_LG_NS * b * A.nv;
    A.count += 2 * i;
    A.s2c += 2 * b;
    H[i].st = i == 0 ? e->stream : e->lg_streamx[i - 1];
    H[i].ev = i == 0 ? &e->evpool : &e->evpoolx[i - 1];
    H[i].nbound = (int)k;
  }
  HIPCHK(e, hipMemsetAsync(e->lg_ngrad, 0, sizeof(unsigned long long), e->stream));
  e->kernel_ms = 0.0;
  e->launches = 0;
  e->units = 0;
  e->lg_steps = 0;
  if (a->iters > 0) {
    // every update needs >= 1 gradient; a NUTS tree has <= 2^depth leaves and nutsepsilon
    // <= 4001; HMC needs L + 1 gradients per update, MALA 2
    int64_t per = (1LL << MMB_NUTS_MAX_DEPTH) + 2, extra = 4002;
    if (A0.kind != MMB_SAMPLER_NUTS) {
      std::vector<double> th;
      int rc = d2h(e, th, h.hmc, e->K * 2);
      if (rc) return rc;
      double lmax = 0.0;
      for (int64_t k = 0; k < e->K; ++k) lmax = std::max(lmax, th[k * 2 + 1]);
      per = A0.kind == MMB_SAMPLER_MALA ? 2 : (int64_t)std::max(lmax, 0.0) + 1;
      extra = 0;
    }
    const int64_t cap = a->iters * per + extra + 4 * LG_CHECK;
    HIPCHK(e, hipMemsetAsync(e->lg_count, 0, 2 * MMB_LG_SPLIT_MAX * sizeof(int32_t), e->stream));
    if (nh > 1) {  // fork: the part streams start behind everything queued on the engine stream
      HIPCHK(e, hipEventRecord(e->lg_join[0], e->stream));
      for (int i = 1; i < nh; ++i) HIPCHK(e, hipStreamWaitEvent(H[i].st, e->lg_join[0], 0));
    }
    for (int i = 0; i < nh; ++i) {
      hipError_t st = mmb_lg_launch_ctl(H[i].A, 1, 0, H[i].A.K, 0, H[i].st);
      if (st != hipSuccess) return fail(e, MMB_E_HIP, "lg_ctl launch: %s", hipGetErrorString(st));
    }
    for (int live = nh; live > 0;) {
      for (int i = 0; i < nh; ++i) {
        Half& q = H[i];
        if (q.done) continue;
        const LgArgs& A = q.A;
        const int64_t s = q.s;
        const int par = (int)(s & 1);
        std::vector<hipEvent_t>& ev = *q.ev;
        if (a->time_kernels) {
          while ((int64_t)ev.size() < 2 * (s + 1)) {
            hipEvent_t x;
            HIPCHK(e, hipEventCreate(&x));
            ev.push_back(x);
          }
          HIPCHK(e, hipEventRecord(ev[2 * s], q.st));
        }
        // group mode once the step is wide enough to fill the GPU with one workgroup per
        // (group, 64-chain tile): half the partial traffic; one workgroup per sub-range below
        // that, where a step's latency is what counts
        const int fold = (int64_t)q.nbound * A.nv * nh >= MMB_LG_FOLD_MIN ? 1 : 0;
        hipError_t st = mmb_lg_launch_grad(A, par, q.nbound, fold, q.st);
        if (st != hipSuccess) return fail(e, MMB_E_HIP, "lg_grad launch: %s", hipGetErrorString(st));
        if (a->time_kernels) HIPCHK(e, hipEventRecord(ev[2 * s + 1], q.st));
        st = mmb_lg_launch_ctl(A, 0, par ^ 1, q.nbound, fold, q.st);
        if (st != hipSuccess) return fail(e, MMB_E_HIP, "lg_ctl launch: %s", hipGetErrorString(st));
        q.s = s + 1;
        if (q.s % LG_CHECK == 0) {
          // two readbacks in flight: wait for the one issued LG_CHECK steps ago, so the
          // stream still holds LG_CHECK queued steps while the host decides (the count is
          // non-increasing, so the older value is still a bound on the running chains)
          const int j = (int)((q.s / LG_CHECK) & 1);
          int32_t* hc = e->lg_hcount + 2 * i;
          hipEvent_t* cev = e->lg_cev + 2 * i;
          HIPCHK(e, hipMemcpyAsync(hc + j, A.count + (q.s & 1), sizeof(int32_t), hipMemcpyDeviceToHost, q.st));
          HIPCHK(e, hipEventRecord(cev[j], q.st));
          const int jw = q.s >= 2 * LG_CHECK ? j ^ 1 : j;  // the first check waits for its own copy
          HIPCHK(e, hipEventSynchronize(cev[jw]));         // (short windows end without surplus)
          if (hc[jw] == 0) {
            q.done = true;
            --live;
          } else {
            q.nbound = hc[jw];
          }
        }
        if (q.s > cap) return fail(e, MMB_E_STATE, "logistic window did not terminate");
      }
    }
    for (int i = 1; i < nh; ++i) {  // join: later work on the engine stream sees every part's results
      HIPCHK(e, hipEventRecord(e->lg_join[i], H[i].st));
      HIPCHK(e, hipStreamWaitEvent(e->stream, e->lg_join[i], 0));
    }
    int64_t steps = 0;
    for (int i = 0; i < nh; ++i) steps = std::max(steps, H[i].s);
    e->lg_steps = steps;
    if (a->time_kernels) {
      // summed gradient-kernel durations of all parts (they may overlap in time)
      for (int i = 0; i < nh; ++i) {
        HIPCHK(e, hipStreamSynchronize(H[i].st));
        for (int64_t t = 0; t < H[i].s; ++t) {
          float ms = 0.f;
          HIPCHK(e, hipEventElapsedTime(&ms, (*H[i].ev)[2 * t], (*H[i].ev)[2 * t + 1]));
          e->kernel_ms += ms;
        }
      }
    }
    e->launches = 0;
    for (int i = 0; i < nh; ++i) e->launches += H[i].s;
    e->units = a->iters * e->K;
  }
  e->iter += a->iters;
  e->n_kept = want ? nk : 0;
  if (a->draws && nk > 0) {
    std::vector<double> hd((size_t)nk * e->pmon * e->K);
    HIPCHK(e, hipMemcpyAsync(hd.data(), e->d_draws, hd.size() * sizeof(double), hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (int64_t i = 0; i < nk; ++i)
      for (int j = 0; j < e->pmon; ++j)
        for (int64_t k = 0; k < e->K; ++k)
          a->draws[i + nk * (j + (int64_t)e->pmon * k)] = hd[(i * e->pmon + j) * e->K + k];
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return 0;
}

int mmb_run(mmb_engine* e, const mmb_run_args* a) {
  if (!e || !a) return fail(e, MMB_E_ARG, "null argument");
  if (!e->d_vals) return fail(e, MMB_E_STATE, "mmb_init_chains not called");
  if (a->iters < 0 || a->thin < 1 || a->burnin < 0)
    return fail(e, MMB_E_ARG, "iters >= 0, thin >= 1, burnin >= 0 required");
  if (e->iter + a->iters > 0xffffffffLL) return fail(e, MMB_E_ARG, "iteration counter overflow");
  HIPCHK(e, hipSetDevice(e->device));
  const int64_t it0 = e->iter;
  const int64_t kept0 = kept_upto(it0, a->burnin, a->thin);
  const int64_t nk = kept_upto(it0 + a->iters, a->burnin, a->thin) - kept0;
  const bool want = (a->draws != nullptr) || a->keep_device;
  if (want && nk > 0) {
    size_t need = (size_t)nk * e->pmon * e->K;
    if (need > e->draws_cap) {
      if (e->d_draws) HIPCHK(e, hipFree(e->d_draws));
      e->d_draws = nullptr;
      HIPCHK(e, dalloc(&e->d_draws, need));
      e->draws_cap = need;
    }
  }
  if (e->model == MMB_MODEL_LOGISTIC) return run_logistic(e, a, (want && nk > 0) ? e->d_draws : nullptr, kept0, nk, want);
  if (a->iters > 0 && !e->order_fresh) {  // else computed right after a previous window
    int orc = order_chains(e);
    if (orc) return orc;
    e->order_iter = it0;
  }
  SweepArgs A;
  fill_args(e, A);
  A.burnin = a->burnin;
  A.thin = a->thin;
  A.model_burnin = a->model_burnin;
  A.kept_origin = kept0;
  A.draws = (want && nk > 0) ? e->d_draws : nullptr;
  const int W = iters_per_launch(e);
  e->kernel_ms = 0.0;
  e->launches = 0;
  e->units = 0;
  const int64_t nl = (a->iters + W - 1) / W;
  if (a->time_kernels) {
    while ((int64_t)e->evpool.size() < 2 * nl) {
      hipEvent_t ev;
      HIPCHK(e, hipEventCreate(&ev));
      e->evpool.push_back(ev);
    }
  }
  for (int64_t done = 0, li = 0, w = 0; done < a->iters; done += w, ++li) {
    w = launch_width(a->iters, W, li);
    A.iter0 = it0 + done;
    A.n_iters = w;
    if (a->time_kernels) HIPCHK(e, hipEventRecord(e->evpool[2 * li], e->stream));
    hipError_t st;
    if (e->jit_fn) {  // node IR, specialised kernel: the interpreter's launch shape (4 chains / 128 threads)
      const int per_block = 128 / Mdl<MMB_MODEL_IR>::G;
      const unsigned grid = (unsigned)((A.K + per_block - 1) / per_block);
      const size_t lds = (size_t)per_block * Mdl<MMB_MODEL_IR>::lds_stride(A) * sizeof(double);
      void* args[] = {(void*)&A};
      st = hipModuleLaunchKernel(e->jit_fn, grid, 1, 1, 128, 1, 1, (unsigned)lds, e->stream, args, nullptr);
    } else {
      st = mmb_launch_sweep(e->model, e->kinds, A, e->stream);
    }
    if (st != hipSuccess) return fail(e, MMB_E_HIP, "sweep launch: %s", hipGetErrorString(st));
    if (a->time_kernels) HIPCHK(e, hipEventRecord(e->evpool[2 * li + 1], e->stream));
    e->launches += 1;
    e->units += (int64_t)w * e->K;
  }
  if (a->iters > 0 && (!e->order_fresh || it0 + a->iters - e->order_iter >= order_every())) {
    // the next window's order from this window's final flags, queued behind its last launch so
    // it runs while the host is between windows (a host write of the tune state invalidates it).
    // The classes persist -- a chain's factor-valid flag is set by its first full-rank update and
    // kept -- so a table less than MMB_ORDER_EVERY iterations old is kept: any table gives the
    // same results, only the pairing could lag a class change (the kernel is ~21 us, ~1 % of a
    // 20-iteration window)
    int orc = order_chains(e);
    if (orc) return orc;
    e->order_fresh = true;
    e->order_iter = it0 + a->iters;
  }
  if (a->time_kernels) {  // per-launch device time, summed after the window (no per-launch sync)
    HIPCHK(e, hipEventSynchronize(e->evpool[2 * nl - 1]));
    for (int64_t li = 0; li < nl; ++li) {
      float ms = 0.f;
      HIPCHK(e, hipEventElapsedTime(&ms, e->evpool[2 * li], e->evpool[2 * li + 1]));
      e->kernel_ms += ms;
    }
  }
  e->iter = it0 + a->iters;
  e->n_kept = want ? nk : 0;
  if ((e->kinds & (1u << MMB_SAMPLER_SLICE)) && a->iters > 0) {
    unsigned long long ov = 0;
    HIPCHK(e, hipMemcpyAsync(&ov, e->d_nstat + 3, sizeof ov, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (ov != e->slice_overflows) {
      const unsigned long long n = ov - e->slice_overflows;
      e->slice_overflows = ov;
      return fail(e, MMB_E_STATE, "Slice: %llu update(s) in iterations %lld..%lld still rejected after %d shrink "
                  "steps (the reference would loop forever; check the widths and the target's support)",
                  n, (long long)it0 + 1, (long long)e->iter, MMB_SLICE_MAX_SHRINK);
    }
  }
  if (a->draws && nk > 0) {
    std::vector<double> h((size_t)nk * e->pmon * e->K);
    HIPCHK(e, hipMemcpyAsync(h.data(), e->d_draws, h.size() * sizeof(double), hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    // Mamba Chains value: n x p x m, column-major (iteration fastest)
    for (int64_t i = 0; i < nk; ++i)
      for (int j = 0; j < e->pmon; ++j)
        for (int64_t k = 0; k < e->K; ++k)
          a->draws[i + nk * (j + (int64_t)e->pmon * k)] = h[(i * e->pmon + j) * e->K + k];
  }
  return 0;
}

int mmb_reserve_draws(mmb_engine* e, int64_t nkept) {
  if (!e || nkept < 0) return fail(e, MMB_E_ARG, "null engine or nkept < 0");
  if (!e->d_vals) return fail(e, MMB_E_STATE, "mmb_init_chains not called");
  const size_t need = (size_t)nkept * e->pmon * e->K;
  if (need > e->draws_cap) {
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));  // the old buffer may still be read by a kernel
    if (e->d_draws) HIPCHK(e, hipFree(e->d_draws));
    e->d_draws = nullptr;
    e->draws_cap = 0;
    e->n_kept = 0;  // the kept draws (if any) went with the old buffer
    HIPCHK(e, dalloc(&e->d_draws, need));
    e->draws_cap = need;
  }
  return 0;
}

int mmb_get_draws(mmb_engine* e, double* draws) {
  if (!e || !draws) return fail(e, MMB_E_ARG, "null argument");
  const int64_t nk = e->n_kept;
  if (nk == 0) return 0;
  std::vector<double> h((size_t)nk * e->pmon * e->K);
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipMemcpy(h.data(), e->d_draws, h.size() * sizeof(double), hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < nk; ++i)
    for (int j = 0; j < e->pmon; ++j)
      for (int64_t k = 0; k < e->K; ++k)
        draws[i + nk * (j + (int64_t)e->pmon * k)] = h[(i * e->pmon + j) * e->K + k];
  return 0;
}

// ---------------------------------------------------------------- tune (canonical layout)

// The 32-lane factorization (samplers.h pchol32: rats, node IR) keeps the AMM factor in
// POSITION form on device -- row at pivot position t at tri(t) + k, k = 0..t, plus one byte per
// element holding its position -- while the canonical tune layout (and the oracle) use the slot
// form L[e][step k] -> slot(e, piv[k]), diagonal at slot(e, e), plus the pivot order.
static bool amm_posform(const mmb_engine* e) { return e->model == MMB_MODEL_RATS || e->model == MMB_MODEL_IR; }
static int tri_(int i) { return i * (i + 1) / 2; }
static int slot_(int i, int k) { return i >= k ? tri_(i) + k : tri_(k) + i; }
// position form (lp, pos) -> slot form (ls, piv); one chain, d x d
static void pos_to_slot(int d, const double* lp, const uint8_t* pos, double* ls, uint8_t* piv) {
  for (int e = 0; e < d; ++e) piv[pos[e] < d ? pos[e] : e] = (uint8_t)e;
  for (int e = 0; e < d; ++e) {
    const int pe = pos[e] < d ? pos[e] : e;
    for (int k = 0; k < pe; ++k) ls[slot_(e, piv[k])] = lp[tri_(pe) + k];
    ls[slot_(e, e)] = lp[tri_(pe) + pe];
  }
}
static void slot_to_pos(int d, const double* ls, const uint8_t* piv, double* lp, uint8_t* pos) {
  for (int k = 0; k < d; ++k) pos[piv[k] < d ? piv[k] : k] = (uint8_t)k;
  for (int e = 0; e < d; ++e) {
    const int pe = pos[e];
    for (int k = 0; k < pe; ++k) lp[tri_(pe) + k] = ls[slot_(e, piv[k])];
    lp[tri_(pe) + pe] = ls[slot_(e, e)];
  }
}

int mmb_get_tune(mmb_engine* e, double* tune) {
  if (!e || !tune) return fail(e, MMB_E_ARG, "null argument");
  if (!e->d_vals) return fail(e, MMB_E_STATE, "mmb_init_chains not called");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  const int64_t TL = mmb_tune_len(e), K = e->K;
  const size_t DP = e->DP, TP = e->TP;
  int64_t off = 0;
  for (auto& h : e->blocks) {
    std::vector<int32_t> m, fl;
    int rc;
    if ((rc = d2h(e, m, h.m, K)) || (rc = d2h(e, fl, h.flags, K))) return rc;
    if (h.spec.sampler == MMB_SAMPLER_AMWG) {
      std::vector<double> sg, ac;
      if ((rc = d2h(e, sg, h.sigma, K * DP)) || (rc = d2h(e, ac, h.accept, K * DP))) return rc;
      for (int64_t k = 0; k < K; ++k) {
        double* t = tune + k * TL + off;
        t[0] = (fl[k] & 1) ? 1.0 : 0.0;
        t[1] = m[k];
        for (int i = 0; i < h.d; ++i) { t[2 + i] = sg[k * DP + i]; t[2 + h.d + i] = ac[k * DP + i]; }
      }
    } else if (h.spec.sampler == MMB_SAMPLER_AMM) {
      std::vector<double> mv, mvv, ls;
      std::vector<uint8_t> pv;
      if ((rc = d2h(e, mv, h.Mv, K * DP)) || (rc = d2h(e, mvv, h.Mvv, K * TP)) ||
          (rc = d2h(e, ls, h.Ls, K * TP)) || (rc = d2h(e, pv, h.piv, K * DP)))
        return rc;
      for (int64_t k = 0; k < K; ++k) {
        double* t = tune + k * TL + off;
        t[0] = (fl[k] & 1) ? 1.0 : 0.0;
        t[1] = m[k];
        t[2] = (fl[k] & 4) ? 1.0 : 0.0;
        t[3] = (fl[k] & 2) ? 1.0 : 0.0;
        double* p = t + 4;
        for (int i = 0; i < h.d; ++i) p[i] = mv[k * DP + i];
        p += h.d;
        for (int s = 0; s < h.T; ++s) p[s] = mvv[k * TP + s];
        p += h.T;
        if (amm_posform(e)) {
          std::vector<uint8_t> piv(h.d);
          std::fill(p, p + h.T, 0.0);
          pos_to_slot(h.d, &ls[k * TP], &pv[k * DP], p, piv.data());
          p += h.T;
          for (int i = 0; i < h.d; ++i) p[i] = piv[i];
        } else {
          for (int s = 0; s < h.T; ++s) p[s] = ls[k * TP + s];
          p += h.T;
          for (int i = 0; i < h.d; ++i) p[i] = pv[k * DP + i];
        }
      }
    } else if (h.spec.sampler == MMB_SAMPLER_NUTS) {
      std::vector<double> nt;
      if ((rc = d2h(e, nt, h.nuts, K * 8))) return rc;
      for (int64_t k = 0; k < K; ++k) {  // [adapt, m, eps, epsbar, Hbar, mu, alpha, nalpha, init]
        double* t = tune + k * TL + off;
        t[0] = (fl[k] & 1) ? 1.0 : 0.0;
        t[1] = m[k];
        for (int i = 0; i < 6; ++i) t[2 + i] = nt[k * 8 + i];
        t[8] = (fl[k] & 8) ? 1.0 : 0.0;
      }
    } else if (h.spec.sampler == MMB_SAMPLER_HMC || h.spec.sampler == MMB_SAMPLER_MALA) {
      std::vector<double> th;
      if ((rc = d2h(e, th, h.hmc, K * 2))) return rc;
      for (int64_t k = 0; k < K; ++k)
        for (int i = 0; i < h.tune_len; ++i) tune[k * TL + off + i] = th[k * 2 + i];
    }
    off += h.tune_len;
  }
  return 0;
}

int mmb_set_tune(mmb_engine* e, const double* tune) {
  if (!e || !tune) return fail(e, MMB_E_ARG, "null argument");
  if (!e->d_vals) return fail(e, MMB_E_STATE, "mmb_init_chains not called");
  const int64_t TL = mmb_tune_len(e), K = e->K;
  const size_t DP = e->DP, TP = e->TP;
  // validate every row before any device state changes: a valid AMM factor (t[2] != 0) needs
  // its pivot order to be a permutation of 0..d-1 (it indexes the caller's row and the device
  // factor); an invalid one is stored with identity positions whatever its pivot bytes hold
  for (int64_t off = 0, b = 0; b < (int64_t)e->blocks.size(); off += e->blocks[b].tune_len, ++b) {
    const auto& h = e->blocks[b];
    if (h.spec.sampler != MMB_SAMPLER_AMM) continue;
    for (int64_t k = 0; k < K; ++k) {
      const double* t = tune + k * TL + off;
      if (t[2] == 0.0) continue;
      const double* pv = t + 4 + h.d + 2 * h.T;
      uint32_t seen = 0;
      for (int i = 0; i < h.d; ++i) {
        const double v = pv[i];
        if (!(v >= 0.0 && v < h.d) || v != (double)(int)v || (seen >> (int)v & 1u))
          return fail(e, MMB_E_ARG, "block %d chain %lld: AMM pivot order is not a permutation of 0..%d",
                      (int)b + 1, (long long)k, h.d - 1);
        seen |= 1u << (int)v;
      }
    }
  }
  ++e->xepoch;
  e->order_fresh = false;  // the factor-valid flags change
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  int64_t off = 0;
  for (auto& h : e->blocks) {
    std::vector<int32_t> m(K, 0), fl(K, 0);
    int rc;
    if (h.spec.sampler == MMB_SAMPLER_AMWG) {
      std::vector<double> sg(K * DP, 0.0), ac(K * DP, 0.0);
      for (int64_t k = 0; k < K; ++k) {
        const double* t = tune + k * TL + off;
        fl[k] = t[0] != 0.0 ? 1 : 0;
        m[k] = (int32_t)t[1];
        for (int i = 0; i < h.d; ++i) { sg[k * DP + i] = t[2 + i]; ac[k * DP + i] = t[2 + h.d + i]; }
      }
      if ((rc = h2d(e, h.sigma, sg)) || (rc = h2d(e, h.accept, ac))) return rc;
    } else if (h.spec.sampler == MMB_SAMPLER_AMM) {
      std::vector<double> mv(K * DP, 0.0), mvv(K * TP, 0.0), ls(K * TP, 0.0);
      std::vector<uint8_t> pv(K * DP, 0);
      for (int64_t k = 0; k < K; ++k) {
        const double* t = tune + k * TL + off;
        fl[k] = (t[0] != 0.0 ? 1 : 0) | (t[2] != 0.0 ? 4 : 0) | (t[3] != 0.0 ? 2 : 0);
        m[k] = (int32_t)t[1];
        const double* p = t + 4;
        for (int i = 0; i < h.d; ++i) mv[k * DP + i] = p[i];
        p += h.d;
        for (int s = 0; s < h.T; ++s) mvv[k * TP + s] = p[s];
        p += h.T;
        const bool valid = t[2] != 0.0;
        if (amm_posform(e)) {
          std::vector<uint8_t> piv(h.d);
          for (int i = 0; i < h.d; ++i) piv[i] = valid ? (uint8_t)p[h.T + i] : (uint8_t)i;
          slot_to_pos(h.d, p, piv.data(), &ls[k * TP], &pv[k * DP]);
        } else {
          for (int s = 0; s < h.T; ++s) ls[k * TP + s] = p[s];
          p += h.T;
          for (int i = 0; i < h.d; ++i) pv[k * DP + i] = valid ? (uint8_t)p[i] : (uint8_t)i;
        }
      }
      if ((rc = h2d(e, h.Mv, mv)) || (rc = h2d(e, h.Mvv, mvv)) || (rc = h2d(e, h.Ls, ls)) ||
          (rc = h2d(e, h.piv, pv)))
        return rc;
    } else if (h.spec.sampler == MMB_SAMPLER_NUTS) {
      std::vector<double> nt(K * 8, 0.0);
      for (int64_t k = 0; k < K; ++k) {
        const double* t = tune + k * TL + off;
        fl[k] = (t[0] != 0.0 ? 1 : 0) | (t[8] != 0.0 ? 8 : 0);
        m[k] = (int32_t)t[1];
        for (int i = 0; i < 6; ++i) nt[k * 8 + i] = t[2 + i];
      }
      if ((rc = h2d(e, h.nuts, nt))) return rc;
    } else if (h.spec.sampler == MMB_SAMPLER_HMC || h.spec.sampler == MMB_SAMPLER_MALA) {
      std::vector<double> th(K * 2);
      for (int64_t k = 0; k < K; ++k) {
        const double* t = tune + k * TL + off;
        th[k * 2] = t[0];
        th[k * 2 + 1] = h.tune_len > 1 ? t[1] : (double)h.spec.nsteps;
      }
      if ((rc = h2d(e, h.hmc, th))) return rc;
    }
    if ((rc = h2d(e, h.m, m)) || (rc = h2d(e, h.flags, fl))) return rc;
    off += h.tune_len;
  }
  return 0;
}

// ---------------------------------------------------------------- Gelman-Rubin partials
int64_t mmb_gr_len(const mmb_engine* e) {
  if (!e) return MMB_E_ARG;
  const int64_t p = e->pmon;
  return 1 + p + p * p + p * p + 3 * p;
}

int mmb_gr_range(mmb_engine* e, double* minmax) {
  if (!e || !minmax) return fail(e, MMB_E_ARG, "null argument");
  if (e->n_kept < 1) return fail(e, MMB_E_STATE, "no device-kept draws (run with keep_device=1)");
  HIPCHK(e, hipSetDevice(e->device));
  double* d = nullptr;
  HIPCHK(e, hipMalloc(&d, 2 * e->pmon * sizeof(double)));
  hipError_t st = mmb_launch_gr_range(e->pmon, e->n_kept, (int)e->K, e->d_draws, d, e->stream);
  if (st != hipSuccess) { (void)hipFree(d); return fail(e, MMB_E_HIP, "gr_range: %s", hipGetErrorString(st)); }
  HIPCHK(e, hipMemcpyAsync(minmax, d, 2 * e->pmon * sizeof(double), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipFree(d));
  return 0;
}

int mmb_gr_partials(mmb_engine* e, const int32_t* link, const double* shift, double* out) {
  if (!e || !link || !shift || !out) return fail(e, MMB_E_ARG, "null argument");
  if (e->n_kept < 2) return fail(e, MMB_E_STATE, "need >= 2 device-kept draws per chain");
  HIPCHK(e, hipSetDevice(e->device));
  const int p = e->pmon;
  const int64_t L = mmb_gr_len(e);
  int32_t* dl = nullptr;
  double *ds = nullptr, *dout = nullptr;
  HIPCHK(e, hipMalloc(&dl, p * sizeof(int32_t)));
  HIPCHK(e, hipMalloc(&ds, p * sizeof(double)));
  HIPCHK(e, hipMalloc(&dout, L * sizeof(double)));
  HIPCHK(e, hipMemcpyAsync(dl, link, p * sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(ds, shift, p * sizeof(double), hipMemcpyHostToDevice, e->stream));
  hipError_t st = mmb_launch_gr_stats(p, e->n_kept, (int)e->K, e->d_draws, dl, ds, dout, e->stream);
  if (st != hipSuccess) {
    (void)hipFree(dl);
    (void)hipFree(ds);
    (void)hipFree(dout);
    return fail(e, MMB_E_HIP, "gr_stats: %s", hipGetErrorString(st));
  }
  HIPCHK(e, hipMemcpyAsync(out, dout, L * sizeof(double), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  (void)hipFree(dl);
  (void)hipFree(ds);
  (void)hipFree(dout);
  return 0;
}

// ---------------------------------------------------------------- posterior summaries
int mmb_chain_summary(mmb_engine* e, const double* shift, int64_t batch_size, int64_t chain_base, double* out) {
  if (!e || !shift || !out) return fail(e, MMB_E_ARG, "null argument");
  if (batch_size < 1) return fail(e, MMB_E_ARG, "batch size must be positive");
  if (chain_base < 0) return fail(e, MMB_E_ARG, "chain_base must be >= 0");
  if (e->n_kept < 1) return fail(e, MMB_E_STATE, "no device-kept draws (run with keep_device=1)");
  HIPCHK(e, hipSetDevice(e->device));
  const int p = e->pmon;
  const size_t nout = (size_t)e->K * p * MMB_SUMMARY_FIELDS;
  double *ds = nullptr, *dout = nullptr;
  HIPCHK(e, hipMalloc(&ds, p * sizeof(double)));
  HIPCHK(e, hipMalloc(&dout, nout * sizeof(double)));
  HIPCHK(e, hipMemcpyAsync(ds, shift, p * sizeof(double), hipMemcpyHostToDevice, e->stream));
  hipError_t st = mmb_launch_chain_summary(p, e->n_kept, (int)e->K, chain_base, batch_size, e->d_draws, ds,
                                           dout, e->stream);
  if (st == hipSuccess) st = hipMemcpyAsync(out, dout, nout * sizeof(double), hipMemcpyDeviceToHost, e->stream);
  if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
  (void)hipFree(ds);
  (void)hipFree(dout);
  if (st != hipSuccess) return fail(e, MMB_E_HIP, "chain_summary: %s", hipGetErrorString(st));
  return 0;
}

int mmb_order_hist(mmb_engine* e, int param, int ntargets, const uint64_t* prefix, int pass, uint64_t* counts) {
  if (!e || !prefix || !counts) return fail(e, MMB_E_ARG, "null argument");
  if (param < 0 || param >= e->pmon) return fail(e, MMB_E_ARG, "param %d out of range", param);
  if (ntargets < 1 || ntargets > MMB_ORDER_MAX_TARGETS) return fail(e, MMB_E_ARG, "1 <= ntargets <= %d",
                                                                      MMB_ORDER_MAX_TARGETS);
  if (pass < 0 || pass > 7) return fail(e, MMB_E_ARG, "pass must be 0..7");
  if (e->n_kept < 1) return fail(e, MMB_E_STATE, "no device-kept draws (run with keep_device=1)");
  HIPCHK(e, hipSetDevice(e->device));
  uint64_t* dp = nullptr;
  unsigned long long* dc = nullptr;
  HIPCHK(e, hipMalloc(&dp, ntargets * sizeof(uint64_t)));
  HIPCHK(e, hipMalloc(&dc, (size_t)ntargets * 256 * sizeof(unsigned long long)));
  hipError_t st = hipMemcpyAsync(dp, prefix, ntargets * sizeof(uint64_t), hipMemcpyHostToDevice, e->stream);
  if (st == hipSuccess)
    st = mmb_launch_order_hist(e->pmon, param, e->n_kept, (int)e->K, e->d_draws, ntargets, dp, pass, dc, e->stream);
  if (st == hipSuccess)
    st = hipMemcpyAsync(counts, dc, (size_t)ntargets * 256 * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream);
  if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
  (void)hipFree(dp);
  (void)hipFree(dc);
  if (st != hipSuccess) return fail(e, MMB_E_HIP, "order_hist: %s", hipGetErrorString(st));
  return 0;
}

// ---------------------------------------------------------------- timing
int mmb_sync(mmb_engine* e) {
  if (!e) return fail(e, MMB_E_ARG, "null argument");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return 0;
}

int mmb_kernel_time(const mmb_engine* e, double* total_ms, int64_t* launches, int64_t* units) {
  if (!e) return MMB_E_ARG;
  if (total_ms) *total_ms = e->kernel_ms;
  if (launches) *launches = e->launches;
  if (units) *units = e->units;
  return 0;
}

// Algorithmic HBM bytes per chain-update (B = 2*S_state + S_draw/thin is
// reported by bench.py; this returns 2*S_state with the minimal state: FP64 values,
// packed symmetric matrices, int32 counters, one byte per pivot index).
int mmb_state_bytes(const mmb_engine* e, double* bytes) {
  if (!e || !bytes) return MMB_E_ARG;
  double s = 8.0 * e->P;
  for (auto& h : e->blocks) {
    switch (h.spec.sampler) {
      case MMB_SAMPLER_AMWG: s += 8.0 * h.d * 2 + 4.0 * h.d * 0 + 4.0; break;  // sigma, accept, m
      case MMB_SAMPLER_AMM: s += 8.0 * (h.d + 2.0 * h.T) + 1.0 * h.d + 4.0; break;  // Mv, Mvv, L, piv, m
      case MMB_SAMPLER_NUTS: s += 8.0 * 7 + 4.0; break;
      case MMB_SAMPLER_HMC: s += 8.0 * 2; break;   // epsilon, L (read only)
      case MMB_SAMPLER_MALA: s += 8.0; break;
      default: break;
    }
  }
  *bytes = 2.0 * s;
  return 0;
}


int mmb_nuts_stats(mmb_engine* e, int64_t* out) {
  if (!e || !out) return fail(e, MMB_E_ARG, "null argument");
  unsigned long long v[3] = {0, 0, 0};
  if (e->d_nstat) {
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemcpyAsync(v, e->d_nstat, sizeof v, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  for (int i = 0; i < 3; ++i) out[i] = (int64_t)v[i];
  return 0;
}

int mmb_amwg_stats(mmb_engine* e, int64_t* out) {
  if (!e || !out) return fail(e, MMB_E_ARG, "null argument");
  unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (e->d_nstat) {
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemcpyAsync(v, e->d_nstat, sizeof v, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  out[0] = (int64_t)v[5];
  return 0;
}

int mmb_amm_stats(mmb_engine* e, int64_t* out) {
  if (!e || !out) return fail(e, MMB_E_ARG, "null argument");
  for (int i = 0; i < MMB_MAX_BLOCKS * MMB_AMM_STATS; ++i) out[i] = 0;
  if (e->K == 0) return 0;
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  std::vector<uint64_t> h;
  for (size_t b = 0; b < e->blocks.size(); ++b) {
    if (!e->blocks[b].astat) continue;
    int rc = d2h(e, h, e->blocks[b].astat, (size_t)e->K * MMB_AMM_STAT_STRIDE);
    if (rc) return rc;
    for (int64_t k = 0; k < e->K; ++k)
      for (int i = 0; i < MMB_AMM_STATS; ++i) out[b * MMB_AMM_STATS + i] += (int64_t)h[k * MMB_AMM_STAT_STRIDE + i];
  }
  return 0;
}

int mmb_chain_order(mmb_engine* e, int32_t* slot_to_chain) {
  if (!e || !slot_to_chain) return fail(e, MMB_E_ARG, "null argument");
  if (e->K == 0) return 0;
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (e->cperm_identity || !e->d_cperm) {
    for (int64_t k = 0; k < e->K; ++k) slot_to_chain[k] = (int32_t)k;
    return 0;
  }
  HIPCHK(e, hipMemcpy(slot_to_chain, e->d_cperm, (size_t)e->K * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}

int mmb_debug_pchol(int device, int64_t n, int d, const double* S, double* L, int32_t* pos, int32_t* info) {
  if (n < 1 || d < 1 || d > 30 || !S || !L || !pos || !info)
    return fail(nullptr, MMB_E_ARG, "mmb_debug_pchol: n >= 1, 1 <= d <= 30 and non-null buffers required");
  constexpr int TP = 480;
  hipError_t st = hipSetDevice(device);
  double *dS = nullptr, *dL = nullptr;
  int32_t *dpos = nullptr, *dinfo = nullptr;
  if (st == hipSuccess) st = hipMalloc(&dS, (size_t)n * TP * sizeof(double));
  if (st == hipSuccess) st = hipMalloc(&dL, (size_t)n * TP * sizeof(double));
  if (st == hipSuccess) st = hipMalloc(&dpos, (size_t)n * 32 * sizeof(int32_t));
  if (st == hipSuccess) st = hipMalloc(&dinfo, (size_t)n * 2 * sizeof(int32_t));
  if (st == hipSuccess) st = hipMemcpy(dS, S, (size_t)n * TP * sizeof(double), hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemset(dL, 0, (size_t)n * TP * sizeof(double));
  if (st == hipSuccess) st = mmb_launch_pchol_probe((int)n, d, dS, dL, dpos, dinfo, nullptr);
  if (st == hipSuccess) st = hipDeviceSynchronize();
  if (st == hipSuccess) st = hipMemcpy(L, dL, (size_t)n * TP * sizeof(double), hipMemcpyDeviceToHost);
  if (st == hipSuccess) st = hipMemcpy(pos, dpos, (size_t)n * 32 * sizeof(int32_t), hipMemcpyDeviceToHost);
  if (st == hipSuccess) st = hipMemcpy(info, dinfo, (size_t)n * 2 * sizeof(int32_t), hipMemcpyDeviceToHost);
  for (void* p : {(void*)dS, (void*)dL, (void*)dpos, (void*)dinfo})
    if (p) (void)hipFree(p);
  if (st != hipSuccess) return fail(nullptr, MMB_E_HIP, "mmb_debug_pchol: %s", hipGetErrorString(st));
  return 0;
}

int mmb_grad_evals(mmb_engine* e, int64_t* n) {
  if (!e || !n) return fail(e, MMB_E_ARG, "null argument");
  *n = 0;
  if (e->model != MMB_MODEL_LOGISTIC || !e->lg_ngrad) return 0;
  unsigned long long v = 0;
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipMemcpyAsync(&v, e->lg_ngrad, sizeof v, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  *n = (int64_t)v;
  return 0;
}

// ---------------------------------------------------------------- cross-GPU Gelman-Rubin (RCCL)
// The one collective of the path (gelmandiag.jl:11-25): each local engine reduces
// its kept draws to the mmb_gr_len sufficient statistics on device (gr.hip), then one SUM
// all-reduce over RCCL/xGMI, in place in a per-engine device buffer; the global [min, max]
// used for link() and the shift is one MAX all-reduce of (-min, max).
// the agreement slot's value outside an agreement: flag 2 = "this rank could not stage" (comm_agree)
static const double kAgreeFailed[4] = {2.0, 0.0, 0.0, 0.0};

struct mmb_comm {
  std::vector<mmb_engine*> eng;
  std::vector<ncclComm_t> comm;
  std::vector<double*> buf;  // per local engine: [L stats | 2p range | p shift | p link (int32) | 4 agree]
  int p = 0;
  int64_t L = 0;
  double agree[4] = {0.0, 0.0, 0.0, 0.0};  // comm_agree's contribution (outlives its async H2D copies)
};

#define NCCLCHK(e, x)                                                                 \
  do {                                                                                \
    ncclResult_t r_ = (x);                                                            \
    if (r_ != ncclSuccess) return fail((e), MMB_E_COMM, "%s: %s", #x, ncclGetErrorString(r_)); \
  } while (0)

__global__ void mmb_negate_mins(double* mm, int p) {
  const int j = (int)threadIdx.x;
  if (j < p) mm[2 * j] = -mm[2 * j];
}

int mmb_comm_id(uint8_t* id) {
  if (!id) return fail(nullptr, MMB_E_ARG, "null argument");
  ncclUniqueId u;
  NCCLCHK(nullptr, ncclGetUniqueId(&u));
  std::memcpy(id, u.internal, MMB_COMM_ID_BYTES);
  return 0;
}

void mmb_comm_destroy(mmb_comm* c) {
  if (!c) return;
  for (size_t i = 0; i < c->eng.size(); ++i) {
    (void)hipSetDevice(c->eng[i]->device);
    if (c->comm[i]) (void)ncclCommDestroy(c->comm[i]);
    if (c->buf[i]) (void)hipFree(c->buf[i]);
  }
  delete c;
}

int mmb_comm_init(mmb_engine** engines, int nlocal, int nranks, int rank0, const uint8_t* id, mmb_comm** out) {
  if (!engines || !out || nlocal < 1) return fail(nullptr, MMB_E_ARG, "null argument or nlocal < 1");
  *out = nullptr;
  mmb_engine* e0 = engines[0];
  if (!e0) return fail(nullptr, MMB_E_ARG, "null engine");
  if (nranks < nlocal || rank0 < 0 || rank0 + nlocal > nranks)
    return fail(e0, MMB_E_ARG, "ranks %d..%d outside 0..%d", rank0, rank0 + nlocal - 1, nranks - 1);
  if (nlocal < nranks && !id) return fail(e0, MMB_E_ARG, "ranks span processes: pass the mmb_comm_id bytes of rank 0");
  for (int i = 0; i < nlocal; ++i) {
    if (!engines[i]) return fail(e0, MMB_E_ARG, "null engine %d", i);
    if (engines[i]->pmon != e0->pmon) return fail(e0, MMB_E_ARG, "engines monitor different parameter counts");
    for (int k = 0; k < i; ++k)
      if (engines[k]->device == engines[i]->device) return fail(e0, MMB_E_ARG, "two local engines on device %d", engines[i]->device);
  }
  mmb_comm* c = new mmb_comm;
  c->eng.assign(engines, engines + nlocal);
  c->comm.assign(nlocal, nullptr);
  c->buf.assign(nlocal, nullptr);
  c->p = e0->pmon;
  c->L = mmb_gr_len(e0);
  const size_t nbuf = (size_t)c->L + 4 * (size_t)c->p + 4;
  for (int i = 0; i < nlocal; ++i) {
    // the agreement slot starts (and is left after every agreement) holding the failure flag, so
    // a rank that cannot stage its contribution still contributes "failed" (comm_agree)
    if (hipSetDevice(engines[i]->device) != hipSuccess || hipMalloc(&c->buf[i], nbuf * sizeof(double)) != hipSuccess ||
        hipMemcpy(c->buf[i] + (nbuf - 4), kAgreeFailed, sizeof kAgreeFailed, hipMemcpyHostToDevice) != hipSuccess) {
      mmb_comm_destroy(c);
      return fail(e0, MMB_E_HIP, "comm buffer allocation failed");
    }
  }
  ncclResult_t r;
  if (nlocal == nranks && !id) {
    std::vector<int> devs(nlocal);
    for (int i = 0; i < nlocal; ++i) devs[i] = engines[i]->device;
    r = ncclCommInitAll(c->comm.data(), nlocal, devs.data());
  } else {
    ncclUniqueId u;
    std::memcpy(u.internal, id, MMB_COMM_ID_BYTES);
    r = ncclGroupStart();
    for (int i = 0; r == ncclSuccess && i < nlocal; ++i) {
      (void)hipSetDevice(engines[i]->device);
      r = ncclCommInitRank(&c->comm[i], nranks, u, rank0 + i);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
  }
  if (r != ncclSuccess) {
    mmb_comm_destroy(c);
    return fail(e0, MMB_E_COMM, "RCCL communicator init (%d local of %d ranks): %s", nlocal, nranks,
                ncclGetErrorString(r));
  }
  *out = c;
  return 0;
}

static int comm_sync(mmb_comm* c) {
  for (mmb_engine* e : c->eng) {
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  return 0;
}

// One in-place all-reduce of n doubles at offset off of every local engine's buffer, grouped.
// ncclGroupEnd is called whatever happens inside the group, so a failed call never leaves the
// thread's RCCL group open for later collectives.
static ncclResult_t grouped_allreduce(mmb_comm* c, size_t off, size_t n, ncclRedOp_t op) {
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return r;
  for (size_t i = 0; r == ncclSuccess && i < c->eng.size(); ++i)
    r = ncclAllReduce(c->buf[i] + off, c->buf[i] + off, n, ncclDouble, op, c->comm[i], c->eng[i]->stream);
  const ncclResult_t r2 = ncclGroupEnd();
  return r != ncclSuccess ? r : r2;
}

// Agreement step before a data collective.  Every local engine contributes (flag, -n_kept,
// n_kept) to one MAX all-reduce, where flag = 1 if this process cannot take part (too few kept
// draws on some local engine) and 2 if it could not even stage its contribution: the slot holds
// 2 outside an agreement (set at comm init and re-armed after every readback), so an engine whose
// staging copy fails contributes the failure flag, never a stale "agree" of an earlier call.  A process whose precondition fails therefore still enters the
// collective, and every rank sees the same verdict: all fail together (MMB_E_STATE for too few
// draws, MMB_E_ARG when the ranks kept different numbers of draws, which would otherwise give
// a silently wrong PSRF) or all proceed with the common n_kept.
// A local HIP failure while staging the contribution does not skip the collective (the peers
// are already waiting in it): the process always joins the all-reduce and the sync, and reports
// its error afterwards (as mmb_gr_allreduce does for launch failures).
static int comm_agree(mmb_comm* c, int64_t need, int64_t* nkept) {
  mmb_engine* e0 = c->eng[0];
  const size_t off = (size_t)c->L + 4 * (size_t)c->p;
  int64_t lo = INT64_MAX, hi = -1;
  for (mmb_engine* e : c->eng) { lo = std::min(lo, e->n_kept); hi = std::max(hi, e->n_kept); }
  c->agree[0] = lo < need ? 1.0 : 0.0;
  c->agree[1] = -(double)lo;
  c->agree[2] = (double)hi;
  c->agree[3] = 0.0;
  int lrc = 0;
  // MMB_TEST_COMM_STAGE_FAIL=1 (tests only): skip the staging copy as if it had failed
  const char* tf = std::getenv("MMB_TEST_COMM_STAGE_FAIL");
  const bool inject = tf && std::atoi(tf) == 1;
  for (size_t i = 0; i < c->eng.size(); ++i) {
    hipError_t st = hipSetDevice(c->eng[i]->device);
    if (st == hipSuccess && inject) st = hipErrorUnknown;
    if (st == hipSuccess)
      st = hipMemcpyAsync(c->buf[i] + off, c->agree, sizeof(c->agree), hipMemcpyHostToDevice, c->eng[i]->stream);
    if (st != hipSuccess && !lrc) lrc = fail(e0, MMB_E_HIP, "agreement staging: %s", hipGetErrorString(st));
  }
  const ncclResult_t r = grouped_allreduce(c, off, 4, ncclMax);
  double all[4] = {2.0, 0.0, 0.0, 0.0};
  hipError_t st = hipSetDevice(e0->device);
  if (st == hipSuccess) st = hipMemcpyAsync(all, c->buf[0] + off, sizeof(all), hipMemcpyDeviceToHost, e0->stream);
  for (size_t i = 0; i < c->eng.size(); ++i)  // re-arm: the slot holds the failure flag again
    if (hipSetDevice(c->eng[i]->device) == hipSuccess)
      (void)hipMemcpyAsync(c->buf[i] + off, kAgreeFailed, sizeof kAgreeFailed, hipMemcpyHostToDevice, c->eng[i]->stream);
  const int rc = comm_sync(c);
  if (r != ncclSuccess) return fail(e0, MMB_E_COMM, "agreement all-reduce: %s", ncclGetErrorString(r));
  if (lrc)
    return fail(e0, MMB_E_HIP, "%s (the agreement all-reduce saw flag %.0f: every rank fails this collective)",
                g_last_error.c_str(), all[0]);
  if (st != hipSuccess) return fail(e0, MMB_E_HIP, "agreement readback: %s", hipGetErrorString(st));
  if (rc) return rc;
  if (all[0] >= 2.0)
    return fail(e0, MMB_E_COMM, "another rank could not stage its agreement contribution; collective skipped");
  if (all[0] != 0.0)
    return fail(e0, MMB_E_STATE, "need >= %lld device-kept draws per chain on every rank (this process: %lld)",
                (long long)need, (long long)lo);
  if (-all[1] != all[2])
    return fail(e0, MMB_E_ARG, "ranks kept different numbers of draws (%.0f .. %.0f)", -all[1], all[2]);
  *nkept = (int64_t)all[2];
  return 0;
}

int mmb_range_allreduce(mmb_comm* c, double* minmax) {
  if (!c || !minmax) return fail(nullptr, MMB_E_ARG, "null argument");
  mmb_engine* e0 = c->eng[0];
  const int p = c->p;
  int64_t nk = 0;
  int rc = comm_agree(c, 1, &nk);
  if (rc) return rc;
  for (size_t i = 0; i < c->eng.size(); ++i) {
    mmb_engine* e = c->eng[i];
    HIPCHK(e0, hipSetDevice(e->device));
    double* mm = c->buf[i] + c->L;
    hipError_t st = mmb_launch_gr_range(p, nk, (int)e->K, e->d_draws, mm, e->stream);
    if (st == hipSuccess) {
      hipLaunchKernelGGL(mmb_negate_mins, dim3(1), dim3(((p + 63) / 64) * 64), 0, e->stream, mm, p);
      st = hipGetLastError();
    }
    // a local launch failure after the agreement still joins the all-reduce below (its peers
    // are already committed to it); the error is reported afterwards
    if (st != hipSuccess) rc = fail(e0, MMB_E_HIP, "gr_range: %s", hipGetErrorString(st));
  }
  const ncclResult_t r = grouped_allreduce(c, (size_t)c->L, 2 * (size_t)p, ncclMax);
  if (r != ncclSuccess) return fail(e0, MMB_E_COMM, "range all-reduce: %s", ncclGetErrorString(r));
  if (rc) return rc;
  HIPCHK(e0, hipSetDevice(e0->device));
  HIPCHK(e0, hipMemcpyAsync(minmax, c->buf[0] + c->L, 2 * p * sizeof(double), hipMemcpyDeviceToHost, e0->stream));
  rc = comm_sync(c);
  if (rc) return rc;
  for (int j = 0; j < p; ++j) minmax[2 * j] = -minmax[2 * j];
  return 0;
}

int mmb_gr_allreduce(mmb_comm* c, const int32_t* link, const double* shift, double* out) {
  if (!c || !link || !shift || !out) return fail(nullptr, MMB_E_ARG, "null argument");
  mmb_engine* e0 = c->eng[0];
  const int p = c->p;
  int64_t nk = 0;
  int rc = comm_agree(c, 2, &nk);
  if (rc) return rc;
  for (size_t i = 0; i < c->eng.size(); ++i) {
    mmb_engine* e = c->eng[i];
    HIPCHK(e0, hipSetDevice(e->device));
    double* ds = c->buf[i] + c->L + 2 * p;
    int32_t* dl = (int32_t*)(ds + p);
    hipError_t st = hipMemcpyAsync(ds, shift, p * sizeof(double), hipMemcpyHostToDevice, e->stream);
    if (st == hipSuccess) st = hipMemcpyAsync(dl, link, p * sizeof(int32_t), hipMemcpyHostToDevice, e->stream);
    if (st == hipSuccess) st = mmb_launch_gr_stats(p, nk, (int)e->K, e->d_draws, dl, ds, c->buf[i], e->stream);
    if (st != hipSuccess) rc = fail(e0, MMB_E_HIP, "gr_stats: %s", hipGetErrorString(st));
  }
  const ncclResult_t r = grouped_allreduce(c, 0, (size_t)c->L, ncclSum);
  if (r != ncclSuccess) return fail(e0, MMB_E_COMM, "Gelman-Rubin all-reduce: %s", ncclGetErrorString(r));
  if (rc) { (void)comm_sync(c); return rc; }
  HIPCHK(e0, hipSetDevice(e0->device));
  HIPCHK(e0, hipMemcpyAsync(out, c->buf[0], c->L * sizeof(double), hipMemcpyDeviceToHost, e0->stream));
  // the host copies of link/shift must outlive the async H2D copies: wait before returning
  return comm_sync(c);
}
