// ir_jit.cpp — specialisation of the node-IR sweep kernel for one lowered model (SURVEY.md §8f
// row 2).  The interpreter of ir.h pays, per expression op, a scalar code
// fetch, a decode, a compare-and-branch chain and an LDS stack spill; the per-lane pool gathers
// of its leaves sit on the same dependency chain.  At mmb_create_ir the engine instead writes
// the model as HIP source -- every node's logpdf_sub loop (dependent.jl:207-213 ->
// distributionstruct.jl:136-168) with its parameter expressions as straight-line code, every
// block's logpdf! term list (simulation.jl:77-90) unrolled with its early exit -- and compiles
// it with hipRTC together with the same sweep / sampler headers as the static kernels.
//
// Bit-identity with the interpreter (and so with the oracle, which restates the interpreter):
// each generated statement is one of the interpreter's IEEE operations on the same operands in
// the same order -- a stack op becomes a named temporary, a binary op `l op r` with l the
// earlier push -- compiled with -ffp-contract=off like the static kernels; expression constants
// are written as exact hexadecimal literals (data stays in the pool: the source depends on the
// model's structure only); lane partials and the 32-lane butterfly are the interpreter's.
//
// Compiled code objects are cached by a hash of the full source (the generated model, the
// embedded headers, the options, the hipRTC version): MMB_JIT_CACHE, else <library dir>/jit.
#include "ir_jit.h"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "jit_headers.inc"  // mmb_jit_headers[] / mmb_jit_header_names[] (build.py: the csrc headers)

namespace {

std::string lit(double v) {
  if (v != v) return "__builtin_nan(\"\")";
  if (v == __builtin_inf()) return "__builtin_inf()";
  if (v == -__builtin_inf()) return "(-__builtin_inf())";
  char b[64];
  snprintf(b, sizeof b, "%a", v);
  return std::string("(") + b + ")";
}

// Emit the statements of expression `pc` (validated stack code, ends in END) evaluated at
// element index `idx`; returns the temporary holding the value.  sub: state slots read from the
// candidate values c[a] instead of vals (a Slice block's coordinates; run-time slots through the
// generated reader rd(k)).
std::string gen_expr(const mmb_ir_model& ir, int pc, const std::string& idx, std::ostringstream& o, int& tmp,
                     const std::vector<int>* sub = nullptr) {
  auto sval = [&](int slot) -> std::string {
    if (sub)
      for (size_t a = 0; a < sub->size(); ++a)
        if ((*sub)[a] == slot) return "c[" + std::to_string(a) + "]";
    return "vals[" + std::to_string(slot) + "]";
  };
  std::vector<std::string> st;
  auto fresh = [&]() { return "t" + std::to_string(tmp++); };
  for (;; ++pc) {
    const uint32_t w = (uint32_t)ir.code[pc];
    const int op = (int)(w >> 24), arg = (int)(w & 0xffffffu);
    if (op == MMB_IR_OP_END) break;
    const std::string t = fresh();
    switch (op) {
      case MMB_IR_OP_CONST: o << "    const double " << t << " = " << lit(ir.consts[arg]) << ";\n"; break;
      case MMB_IR_OP_VAL: o << "    const double " << t << " = " << sval(arg) << ";\n"; break;
      case MMB_IR_OP_VALI:
        if (sub) o << "    const double " << t << " = rd(" << arg << " + " << idx << ");\n";
        else o << "    const double " << t << " = vals[" << arg << " + " << idx << "];\n";
        break;
      case MMB_IR_OP_VALG: {  // gather: the pool offset of the indices is the next word
        const int woff = ir.code[++pc];
        if (sub) o << "    const double " << t << " = rd(" << arg << " + (int)A.ir_pool[" << woff << " + " << idx << "]);\n";
        else o << "    const double " << t << " = vals[" << arg << " + (int)A.ir_pool[" << woff << " + " << idx << "]];\n";
        break;
      }
      case MMB_IR_OP_DATA: o << "    const double " << t << " = A.ir_pool[" << arg << " + " << idx << "];\n"; break;
      case MMB_IR_OP_DATAS: o << "    const double " << t << " = mmb_jit_uload(A.ir_pool, " << arg << ");\n"; break;
      case MMB_IR_OP_ADD: case MMB_IR_OP_SUB: case MMB_IR_OP_MUL: case MMB_IR_OP_DIV: {
        const std::string r = st.back(); st.pop_back();
        const std::string l = st.back(); st.pop_back();
        const char* c = op == MMB_IR_OP_ADD ? " + " : op == MMB_IR_OP_SUB ? " - " : op == MMB_IR_OP_MUL ? " * " : " / ";
        o << "    const double " << t << " = " << l << c << r << ";\n";
        break;
      }
      default: {  // unary
        const std::string a = st.back(); st.pop_back();
        o << "    const double " << t << " = mmb_ir_unary(" << op << ", " << a << ");\n";
        break;
      }
    }
    st.push_back(t);
  }
  return st.back();
}

// Whether expression pc depends on the element index (indexed / gathered state, indexed data)
bool expr_indexed(const mmb_ir_model& ir, int pc) {
  for (;; ++pc) {
    const uint32_t w = (uint32_t)ir.code[pc];
    const int op = (int)(w >> 24);
    if (op == MMB_IR_OP_END) return false;
    if (op == MMB_IR_OP_VALI || op == MMB_IR_OP_VALG || op == MMB_IR_OP_DATA) return true;
    if (op == MMB_IR_OP_VALG) ++pc;
  }
}

// logpdf(node[, transform]) of node n as the interpreter's node_lp (ir.h), group-uniform
void gen_node(const mmb_ir_model& ir, int n, std::ostringstream& o) {
  const mmb_ir_node& N = ir.nodes[n];
  int tmp = 0;
  o << "__device__ __forceinline__ double mmb_jn_" << n
    << "(const SweepArgs& A, const double* vals, const Grp<32>& g, int tr) {\n";
  o << "  (void)tr;\n  const int lane = g.lane;\n";
  const std::string src = N.fixed ? "(A.ir_pool + " + std::to_string(N.off) + ")" : "(vals + " + std::to_string(N.off) + ")";
  if (N.family == MMB_IR_ISONORMAL) {  // MvNormal(mu, sigma): PDMats ScalMat, insupport = all finite
    o << "  double sig;\n  {\n    const int i = 0;\n    (void)i;\n";
    const std::string s = gen_expr(ir, N.expr[1], "i", o, tmp);
    o << "    sig = " << s << ";\n  }\n";
    o << "  double ss = 0.0, bad = 0.0;\n";
    o << "  for (int i = lane; i < " << N.len << "; i += 32) {\n";
    o << "    const double x = " << src << "[i];\n";
    const std::string m = gen_expr(ir, N.expr[0], "i", o, tmp);
    o << "    const double r = x - " << m << ";\n";
    o << "    ss = ss + r * r;\n    bad = isfinite(x) ? bad : 1.0;\n  }\n";
    o << "  g.sum2(ss, bad);\n";
    o << "  return bad != 0.0 ? -__builtin_inf() : d_iso(" << N.len << ", sig, ss);\n}\n";
    return;
  }
  if (N.len == 1) {
    // one element: every lane forms it (no lane partials, no butterfly).  The butterfly over lane
    // 0's term and 31 zeros returns the term itself except that -0 becomes +0, and the block's
    // running lp -- which starts at +0 and so is never -0 -- adds either to the same value
    o << "  (void)lane;\n  const int i = 0;\n";
    std::string a = "0.0", b = "0.0", ct = "0.0";
    if (N.expr[0] >= 0) a = gen_expr(ir, N.expr[0], "i", o, tmp);
    if (N.expr[1] >= 0) b = gen_expr(ir, N.expr[1], "i", o, tmp);
    if (N.cterm >= 0) ct = "A.ir_pool[" + std::to_string(N.cterm) + " + i]";
    o << "  return 0.0 + mmb_ir_lp(" << N.family << ", " << src << "[i], " << a << ", " << b << ", " << ct
      << ", tr, " << lit(N.lo) << ", " << lit(N.hi) << ");\n}\n";
    return;
  }
  if (N.family == MMB_IR_NORMAL && N.expr[1] >= 0 && !expr_indexed(ir, N.expr[1])) {
    // sigma the same for every element: it and its log formed once (mmb_ir_normal_lb)
    o << "  double sg, lsg;\n  {\n    const int i = 0;\n    (void)i;\n";
    const std::string b = gen_expr(ir, N.expr[1], "i", o, tmp);
    o << "    sg = " << b << ";\n    lsg = mmb_log(sg);\n  }\n";
    o << "  double acc = 0.0;\n";
    o << "  for (int i = lane; i < " << N.len << "; i += 32) {\n";
    const std::string a = N.expr[0] >= 0 ? gen_expr(ir, N.expr[0], "i", o, tmp) : "0.0";
    o << "    acc = acc + mmb_ir_normal_lb(" << src << "[i], " << a << ", sg, lsg);\n  }\n";
    o << "  return g.sum(acc);\n}\n";
    return;
  }
  o << "  double acc = 0.0;\n";
  o << "  for (int i = lane; i < " << N.len << "; i += 32) {\n";
  std::string a = "0.0", b = "0.0", ct = "0.0";
  if (N.expr[0] >= 0) a = gen_expr(ir, N.expr[0], "i", o, tmp);
  if (N.expr[1] >= 0) b = gen_expr(ir, N.expr[1], "i", o, tmp);
  if (N.cterm >= 0) ct = "A.ir_pool[" + std::to_string(N.cterm) + " + i]";
  o << "    acc = acc + mmb_ir_lp(" << N.family << ", " << src << "[i], " << a << ", " << b << ", " << ct
    << ", tr, " << lit(N.lo) << ", " << lit(N.hi) << ");\n  }\n";
  o << "  return g.sum(acc);\n}\n";
}

// One element's term of node n's logpdf_sub at element i, exactly as gen_node's loop forms it (the
// lane-parallel AMWG of ir.h amwg_dm sums differences of these): mmb_ir_lp(...) for the element
// families, r * r for an MvNormal (NaN when the value is not finite: its insupport test).
void gen_elem(const mmb_ir_model& ir, int n, std::ostringstream& o) {
  const mmb_ir_node& N = ir.nodes[n];
  int tmp = 0;
  o << "__device__ __forceinline__ double mmb_je_" << n << "(const SweepArgs& A, const double* vals, int i, int tr) {\n";
  o << "  (void)tr; (void)A;\n";
  const std::string src = N.fixed ? "(A.ir_pool + " + std::to_string(N.off) + ")" : "(vals + " + std::to_string(N.off) + ")";
  if (N.family == MMB_IR_ISONORMAL) {
    o << "  const double x = " << src << "[i];\n";
    const std::string m = gen_expr(ir, N.expr[0], "i", o, tmp);
    o << "  const double r = x - " << m << ";\n";
    o << "  return isfinite(x) ? r * r : __builtin_nan(\"\");\n}\n";
    return;
  }
  std::string a = "0.0", b = "0.0", ct = "0.0";
  if (N.expr[0] >= 0) a = gen_expr(ir, N.expr[0], "i", o, tmp);
  if (N.expr[1] >= 0) b = gen_expr(ir, N.expr[1], "i", o, tmp);
  if (N.cterm >= 0) ct = "A.ir_pool[" + std::to_string(N.cterm) + " + i]";
  o << "  return mmb_ir_lp(" << N.family << ", " << src << "[i], " << a << ", " << b << ", " << ct << ", tr, "
    << lit(N.lo) << ", " << lit(N.hi) << ");\n}\n";
}

// Weight of node n's element terms in the block's logpdf! and the magnitude of its constant part:
// 1 and 0 for the element families; for an MvNormal, d_iso's -0.5 / sigma^2 and 0.5 |k log2pi +
// k log sigma^2| (sigma at element 0, as gen_node evaluates it).
void gen_termw(const mmb_ir_model& ir, int n, std::ostringstream& o) {
  const mmb_ir_node& N = ir.nodes[n];
  int tmp = 0;
  o << "__device__ __forceinline__ void mmb_jw_" << n << "(const SweepArgs& A, const double* vals, double* w, double* c) {\n";
  o << "  (void)A; (void)vals;\n";
  if (N.family != MMB_IR_ISONORMAL) {
    o << "  *w = 1.0;\n  *c = 0.0;\n}\n";
    return;
  }
  o << "  const int i = 0;\n  (void)i;\n";
  const std::string s = gen_expr(ir, N.expr[1], "i", o, tmp);
  o << "  const double value = " << s << " * " << s << ";\n";
  o << "  const double invv = 1.0 / value;\n";
  o << "  *w = -0.5 * invv;\n";
  o << "  *c = 0.5 * fabs(" << N.len << " * MMB_LOG2PI + " << N.len << " * mmb_log(value));\n}\n";
}

// Whether expression pc reads any of `slots` (a Slice block's coordinates): a VAL of one, or an
// indexed / gathered read of a node whose slot range holds one (an unknown base: yes)
bool expr_reads(const mmb_ir_model& ir, int pc, const std::vector<int>& slots) {
  auto in_node = [&](int base) {
    for (int n = 0; n < ir.nnodes; ++n) {
      const mmb_ir_node& N = ir.nodes[n];
      if (N.fixed || N.off != base) continue;
      for (int k : slots)
        if (k >= base && k < base + N.len) return true;
      return false;
    }
    return true;
  };
  for (;; ++pc) {
    const uint32_t w = (uint32_t)ir.code[pc];
    const int op = (int)(w >> 24), arg = (int)(w & 0xffffffu);
    if (op == MMB_IR_OP_END) return false;
    if (op == MMB_IR_OP_VAL && std::find(slots.begin(), slots.end(), arg) != slots.end()) return true;
    if ((op == MMB_IR_OP_VALI || op == MMB_IR_OP_VALG) && in_node(arg)) return true;
    if (op == MMB_IR_OP_VALG) ++pc;
  }
}

// The MvNormal terms of Slice block b whose elements read none of the block's coordinates (only
// their sigma does, e.g. rats' y term in the s2_c block): their sum of squares is the same for
// every candidate, so mmb_jp_<b> forms it once per update with logf's own loop and 32-lane sum
// (gen_node), and mmb_jc_<b> only evaluates d_iso at the candidate's sigma -- the same value as
// the candidate-side loop, whose tree is logf's.
std::vector<int> slice_shared_terms(const mmb_model_spec& spec, const mmb_ir_model& ir, int b,
                                    const std::vector<int>& slots) {
  const mmb_block_spec& s = spec.blocks[b];
  const mmb_ir_block& IB = ir.blocks[b];
  std::vector<int> out;
  for (int t = 0; t < IB.nterms; ++t) {
    const int n = IB.term[t];
    const mmb_ir_node& N = ir.nodes[n];
    if (N.family != MMB_IR_ISONORMAL) continue;
    bool inblk = false;
    for (int a = 0; a < s.nnodes; ++a) inblk = inblk || s.nodes[a] == n;
    if (inblk || expr_reads(ir, N.expr[0], slots)) continue;
    out.push_back(t);
  }
  return out;
}

void gen_slice_prep(const mmb_model_spec& spec, const mmb_ir_model& ir, int b, const std::vector<int>& shared,
                    std::ostringstream& o) {
  (void)spec;
  const mmb_ir_block& IB = ir.blocks[b];
  o << "__device__ __forceinline__ void mmb_jp_" << b
    << "(const SweepArgs& A, const double* vals, const Grp<32>& g, double* pre) {\n";
  o << "  const int lane = g.lane;\n  (void)lane;\n";
  int tmp = 0;
  for (size_t j = 0; j < shared.size(); ++j) {
    const int n = IB.term[shared[j]];
    const mmb_ir_node& N = ir.nodes[n];
    const std::string src = N.fixed ? "(A.ir_pool + " + std::to_string(N.off) + ")" : "(vals + " + std::to_string(N.off) + ")";
    o << "  {  // term " << shared[j] << ": node " << n << "\n";
    o << "    double ss = 0.0, bad = 0.0;\n";
    o << "    for (int i = lane; i < " << N.len << "; i += 32) {\n";
    o << "      const double x = " << src << "[i];\n";
    const std::string m = gen_expr(ir, N.expr[0], "i", o, tmp);
    o << "      const double r = x - " << m << ";\n";
    o << "      ss = ss + r * r;\n      bad = isfinite(x) ? bad : 1.0;\n    }\n";
    o << "    g.sum2(ss, bad);\n";
    o << "    pre[" << 2 * j << "] = ss;\n    pre[" << 2 * j + 1 << "] = bad;\n  }\n";
  }
  o << "}\n";
}

// logpdf!(m, x, block) of Slice block b at one candidate per group of 32 / VL lanes (samplers.h
// slice_uni_cand / slice_multi_cand; ir.h slice_cand_logf): the block's coordinates are read from
// c[] (state values, invlinked) instead of the chain state.  Lane r of the group stands for lanes
// VL r .. VL r + VL - 1 of the 32-lane layout: it forms their VL lane partials (elements i = lane,
// lane + 32, .. in order, as gen_node's loop) and combines them as the first log2(VL) levels of the
// 32-lane butterfly -- (p0 + p1), or ((p0 + p1) + (p2 + p3)) for VL = 4; the remaining levels are
// Grp<32>::other_d<0..> across the group (after the local levels every lane's virtual lanes agree,
// so each later partner lane of Grp<32>::sum's tree is reached by the next stage's partner of the
// real lane).  The same tree over the same terms: bit-identical to logf.
std::vector<int> block_slots(const mmb_model_spec& spec, const mmb_ir_model& ir, int b) {
  const mmb_block_spec& s = spec.blocks[b];
  std::vector<int> slots;
  for (int a = 0; a < s.nnodes; ++a) {
    const mmb_ir_node& N = ir.nodes[s.nodes[a]];
    for (int q = 0; q < N.len; ++q) slots.push_back(N.off + q);
  }
  return slots;
}

void gen_slice_cand(const mmb_model_spec& spec, const mmb_ir_model& ir, int b, const std::vector<int>& shared,
                    int VL, std::ostringstream& o) {
  const mmb_block_spec& s = spec.blocks[b];
  const mmb_ir_block& IB = ir.blocks[b];
  const std::vector<int> slots = block_slots(spec, ir, b);
  o << "__device__ __forceinline__ double mmb_jc_" << b << "(const SweepArgs& A, const double* vals, const double* c, int r,\n"
       "                                        int transform, const double* pre) {\n";
  o << "  (void)transform; (void)pre;\n";
  o << "  auto rd = [&](int k) -> double {\n    return ";
  for (size_t a = 0; a < slots.size(); ++a) o << "k == " << slots[a] << " ? c[" << a << "] : ";
  o << "vals[k];\n  };\n  (void)rd;\n";
  o << "  double lp = 0.0;\n";
  int tmp = 0;
  for (int t = 0; t < IB.nterms; ++t) {
    const int n = IB.term[t];
    const mmb_ir_node& N = ir.nodes[n];
    bool inblk = false;
    for (int a = 0; a < s.nnodes; ++a) inblk = inblk || s.nodes[a] == n;
    const std::string tr = IB.trans[t] ? "transform" : "0";
    auto xval = [&](const std::string& i) {
      if (N.fixed) return "A.ir_pool[" + std::to_string(N.off) + " + " + i + "]";
      if (inblk) return "rd(" + std::to_string(N.off) + " + " + i + ")";
      return "vals[" + std::to_string(N.off) + " + " + i + "]";
    };
    o << "  {  // term " << t << ": node " << n << "\n";
    const auto sh = std::find(shared.begin(), shared.end(), t);
    if (sh != shared.end()) {  // elements independent of the candidate: mmb_jp_<b>'s sums
      const int j = (int)(sh - shared.begin());
      o << "    double sig;\n    {\n    const int i = 0;\n    (void)i;\n";
      const std::string sg = gen_expr(ir, N.expr[1], "i", o, tmp, &slots);
      o << "    sig = " << sg << ";\n    }\n";
      o << "    lp += pre[" << 2 * j + 1 << "] != 0.0 ? -__builtin_inf() : d_iso(" << N.len << ", sig, pre[" << 2 * j << "]);\n";
    } else if (N.family == MMB_IR_ISONORMAL) {
      o << "    double sig;\n    {\n    const int i = 0;\n    (void)i;\n";
      const std::string sg = gen_expr(ir, N.expr[1], "i", o, tmp, &slots);
      o << "    sig = " << sg << ";\n    }\n";
      o << "    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0, bd = 0.0;\n";
      o << "#pragma nounroll\n    for (int v = 0; v < " << VL << "; ++v) {\n      double ss = 0.0;\n";
      o << "      for (int i = " << VL << " * r + v; i < " << N.len << "; i += 32) {\n";
      o << "        const double x = " << xval("i") << ";\n";
      const std::string m = gen_expr(ir, N.expr[0], "i", o, tmp, &slots);
      o << "        const double rr = x - " << m << ";\n        ss = ss + rr * rr;\n";
      o << "        bd = isfinite(x) ? bd : 1.0;\n      }\n";
      o << "      p0 = v == 0 ? ss : p0;\n      p1 = v == 1 ? ss : p1;\n      p2 = v == 2 ? ss : p2;\n      p3 = v == 3 ? ss : p3;\n    }\n";
      o << (VL == 4 ? "    double sv = (p0 + p1) + (p2 + p3);\n" : "    double sv = p0 + p1;\n");
      for (int k = 0; k < 5 - (VL == 4 ? 2 : 1); ++k)
        o << "    sv += Grp<32>::other_d<" << k << ">(sv); bd += Grp<32>::other_d<" << k << ">(bd);\n";
      o << "    lp += bd != 0.0 ? -__builtin_inf() : d_iso(" << N.len << ", sig, sv);\n";
    } else if (N.len == 1) {  // one element: on every lane, as gen_node
      o << "    {\n    const int i = 0;\n";
      std::string a = "0.0", bb = "0.0", ct = "0.0";
      if (N.expr[0] >= 0) a = gen_expr(ir, N.expr[0], "i", o, tmp, &slots);
      if (N.expr[1] >= 0) bb = gen_expr(ir, N.expr[1], "i", o, tmp, &slots);
      if (N.cterm >= 0) ct = "A.ir_pool[" + std::to_string(N.cterm) + " + i]";
      o << "    lp += 0.0 + mmb_ir_lp(" << N.family << ", " << xval("i") << ", " << a << ", " << bb << ", " << ct
        << ", " << tr << ", " << lit(N.lo) << ", " << lit(N.hi) << ");\n    }\n";
    } else {
      const bool hoist = N.family == MMB_IR_NORMAL && N.expr[1] >= 0 && !expr_indexed(ir, N.expr[1]);
      if (hoist) {  // sigma and its log once per lane (as gen_node)
        o << "    double sg, lsg;\n    {\n    const int i = 0;\n    (void)i;\n";
        const std::string bs = gen_expr(ir, N.expr[1], "i", o, tmp, &slots);
        o << "    sg = " << bs << ";\n    lsg = mmb_log(sg);\n    }\n";
      }
      o << "    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;\n";
      o << "#pragma nounroll\n    for (int v = 0; v < " << VL << "; ++v) {\n      double acc = 0.0;\n";
      o << "      for (int i = " << VL << " * r + v; i < " << N.len << "; i += 32) {\n";
      std::string a = "0.0", bb = "0.0", ct = "0.0";
      if (N.expr[0] >= 0) a = gen_expr(ir, N.expr[0], "i", o, tmp, &slots);
      if (hoist) {
        o << "        acc = acc + mmb_ir_normal_lb(" << xval("i") << ", " << a << ", sg, lsg);\n      }\n";
      } else {
        if (N.expr[1] >= 0) bb = gen_expr(ir, N.expr[1], "i", o, tmp, &slots);
        if (N.cterm >= 0) ct = "A.ir_pool[" + std::to_string(N.cterm) + " + i]";
        o << "        acc = acc + mmb_ir_lp(" << N.family << ", " << xval("i") << ", " << a << ", " << bb << ", " << ct
          << ", " << tr << ", " << lit(N.lo) << ", " << lit(N.hi) << ");\n      }\n";
      }
      o << "      p0 = v == 0 ? acc : p0;\n      p1 = v == 1 ? acc : p1;\n      p2 = v == 2 ? acc : p2;\n      p3 = v == 3 ? acc : p3;\n    }\n";
      o << (VL == 4 ? "    double sv = (p0 + p1) + (p2 + p3);\n" : "    double sv = p0 + p1;\n");
      for (int k = 0; k < 5 - (VL == 4 ? 2 : 1); ++k) o << "    sv += Grp<32>::other_d<" << k << ">(sv);\n";
      o << "    lp += sv;\n";
    }
    o << "    if (!isfinite(lp)) return lp;\n  }\n";
  }
  o << "  return lp;\n}\n";
}

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
  const unsigned char* c = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) { h ^= c[i]; h *= 1099511628211ull; }
  return h;
}

std::string lib_dir() {
  Dl_info info;
  if (dladdr((void*)&fnv1a, &info) && info.dli_fname) {
    std::string f(info.dli_fname);
    const size_t k = f.rfind('/');
    if (k != std::string::npos) return f.substr(0, k);
  }
  return ".";
}

bool read_file(const std::string& path, std::vector<char>& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return !out.empty();
}

}  // namespace

std::string mmb_ir_jit_source(const mmb_model_spec& spec, const mmb_ir_model& ir, unsigned kinds, int dmax) {
  std::ostringstream o;
  o << "// node-IR sweep kernel specialised for one model (generated by ir_jit.cpp)\n";
  // occupancy target of the specialised kernel (MMB_IR_JIT_WAVES, default 4 waves per SIMD: the
  // straight-line model code fits 128 VGPRs where the interpreter needed 2 waves' budget)
  int waves = 4;
  if (const char* w = std::getenv("MMB_IR_JIT_WAVES")) waves = std::max(1, std::min(8, std::atoi(w)));
  o << "#define MMB_IR_JIT 1\n#define MMB_IR_DMAX " << dmax << "\n#define MMB_IR_WAVES " << waves << "\n";
  {  // logf inlined at its call sites: a call makes the caller save and restore its SGPRs around
     // it (rats via the IR: 689 -> 509 SGPR spill slots, 6.1e7 -> 7.4e7 chain-updates/s A/B);
     // MMB_IR_LOGF_INLINE=0 keeps the call
    const char* e = std::getenv("MMB_IR_LOGF_INLINE");
    if (!(e && std::atoi(e) == 0)) o << "#define MMB_IR_LOGF_ATTR __forceinline__\n";
  }
  o << "#include \"device.h\"\n\n";
  // a uniform pool value (scalar load): data may change between models of the same structure,
  // so the source -- and the cached code object -- depends on the model's structure only
  o << "__device__ __forceinline__ double mmb_jit_uload(const double* p, int k) {\n"
       "  return *(const double*)&((const __attribute__((address_space(4))) double*)p)[k];\n}\n\n";
  std::vector<char> used(ir.nnodes, 0);
  for (int b = 0; b < spec.nblocks; ++b)
    for (int t = 0; t < ir.blocks[b].nterms; ++t) used[ir.blocks[b].term[t]] = 1;
  for (int n = 0; n < ir.nnodes; ++n)
    if (used[n]) gen_node(ir, n, o);
  // logpdf!(m, x, block, transform): params \ targets, then targets; early exit (simulation.jl:77-90)
  o << "__device__ __forceinline__ double mmb_jit_block_lp(const SweepArgs& A, int blk, const double* vals,\n"
       "                                                   const Grp<32>& g, int transform) {\n"
       "  (void)transform;\n  double lp = 0.0;\n  switch (blk) {\n";
  for (int b = 0; b < spec.nblocks; ++b) {
    const mmb_ir_block& IB = ir.blocks[b];
    o << "    case " << b << ":\n";
    for (int t = 0; t < IB.nterms; ++t) {
      o << "      lp += mmb_jn_" << IB.term[t] << "(A, vals, g, " << (IB.trans[t] ? "transform" : "0") << ");\n";
      o << "      if (!isfinite(lp)) break;\n";
    }
    o << "      break;\n";
  }
  o << "    default: break;\n  }\n  return lp;\n}\n";
  if (kinds & (1u << MMB_SAMPLER_AMWG)) {
    // element terms and term weights of the AMWG blocks' logpdf! (lane-parallel decisions, ir.h
    // amwg_dm; used only on blocks the engine finds separable, engine.cpp ir_sep_table)
    std::vector<char> en(ir.nnodes, 0);
    for (int b = 0; b < spec.nblocks; ++b)
      if (spec.blocks[b].sampler == MMB_SAMPLER_AMWG)
        for (int t = 0; t < ir.blocks[b].nterms; ++t) en[ir.blocks[b].term[t]] = 1;
    for (int n = 0; n < ir.nnodes; ++n)
      if (en[n]) {
        gen_elem(ir, n, o);
        gen_termw(ir, n, o);
      }
    o << "#define MMB_IR_SEP 1\n";
    o << "__device__ __forceinline__ double mmb_jit_elem(const SweepArgs& A, int blk, int t, int i, const double* vals,\n"
         "                                               int transform) {\n"
         "  (void)transform;\n  switch (blk) {\n";
    for (int b = 0; b < spec.nblocks; ++b) {
      if (spec.blocks[b].sampler != MMB_SAMPLER_AMWG) continue;
      const mmb_ir_block& IB = ir.blocks[b];
      o << "    case " << b << ":\n      switch (t) {\n";
      for (int t = 0; t < IB.nterms; ++t)
        o << "        case " << t << ": return mmb_je_" << IB.term[t] << "(A, vals, i, "
          << (IB.trans[t] ? "transform" : "0") << ");\n";
      o << "        default: return 0.0;\n      }\n";
    }
    o << "    default: return 0.0;\n  }\n}\n";
    o << "__device__ __forceinline__ void mmb_jit_termw(const SweepArgs& A, int blk, int t, const double* vals,\n"
         "                                              double* w, double* c) {\n"
         "  *w = 1.0;\n  *c = 0.0;\n  switch (blk) {\n";
    for (int b = 0; b < spec.nblocks; ++b) {
      if (spec.blocks[b].sampler != MMB_SAMPLER_AMWG) continue;
      const mmb_ir_block& IB = ir.blocks[b];
      o << "    case " << b << ":\n      switch (t) {\n";
      for (int t = 0; t < IB.nterms; ++t)
        o << "        case " << t << ": mmb_jw_" << IB.term[t] << "(A, vals, w, c); return;\n";
      o << "        default: return;\n      }\n";
    }
    o << "    default: return;\n  }\n}\n";
  }
  {  // Slice blocks of up to four coordinates: candidates evaluated four at a time (ir.h)
    bool any = false;
    int npre = 0;
    std::vector<int> pre_blocks;  // Slice candidate blocks with shared MvNormal sums
    // candidates per round = virtual lanes per lane: 2 (sixteen lanes per candidate; default) or 4
    // (eight; MMB_IR_SLICE_NC=4).  rats via the IR: 7.52e7 (2) vs 7.15e7 (4) chain-updates/s A/B --
    // the scalar blocks accept within a candidate or two, so wider rounds mostly add work
    int nc = 2;
    if (const char* e = std::getenv("MMB_IR_SLICE_NC")) nc = std::atoi(e) == 4 ? 4 : 2;
    for (int b = 0; b < spec.nblocks; ++b) {
      if (spec.blocks[b].sampler != MMB_SAMPLER_SLICE) continue;
      int d = 0;
      for (int a = 0; a < spec.blocks[b].nnodes; ++a) d += ir.nodes[spec.blocks[b].nodes[a]].len;
      if (d > 4) continue;
      const std::vector<int> shared = slice_shared_terms(spec, ir, b, block_slots(spec, ir, b));
      if (!shared.empty()) {
        gen_slice_prep(spec, ir, b, shared, o);
        pre_blocks.push_back(b);
      }
      npre = std::max(npre, (int)shared.size());
      gen_slice_cand(spec, ir, b, shared, nc, o);
      any = true;
    }
    if (any) {
      o << "#define MMB_IR_SLICEC 1\n#define MMB_IR_SPRE " << std::max(npre, 1) << "\n#define MMB_IR_SLICE_NC " << nc << "\n";
      o << "__device__ __forceinline__ void mmb_jit_slice_prep(const SweepArgs& A, int blk, const double* vals,\n"
           "                                                   const Grp<32>& g, double* pre) {\n"
           "  (void)A; (void)vals; (void)g; (void)pre;\n  switch (blk) {\n";
      for (int b = 0; b < spec.nblocks; ++b) {
        if (spec.blocks[b].sampler != MMB_SAMPLER_SLICE) continue;
        int d = 0;
        for (int a = 0; a < spec.blocks[b].nnodes; ++a) d += ir.nodes[spec.blocks[b].nodes[a]].len;
        if (d > 4 || slice_shared_terms(spec, ir, b, block_slots(spec, ir, b)).empty()) continue;
        o << "    case " << b << ": mmb_jp_" << b << "(A, vals, g, pre); return;\n";
      }
      o << "    default: return;\n  }\n}\n";
      o << "__device__ __forceinline__ bool mmb_jit_slice_has_pre(int blk) {\n  switch (blk) {\n";
      for (int b : pre_blocks) o << "    case " << b << ": return true;\n";
      o << "    default: return false;\n  }\n}\n";
      // logpdf!(m, x, block) as mmb_jit_block_lp, the shared MvNormal terms from the prep's sums
      o << "__device__ __forceinline__ double mmb_jit_block_lp_pre(const SweepArgs& A, int blk, const double* vals,\n"
           "                                                       const Grp<32>& g, int transform, const double* pre) {\n"
           "  (void)transform;\n  double lp = 0.0;\n  switch (blk) {\n";
      for (int b : pre_blocks) {
        const mmb_ir_block& IB = ir.blocks[b];
        const std::vector<int> shared = slice_shared_terms(spec, ir, b, block_slots(spec, ir, b));
        o << "    case " << b << ":\n";
        for (int t = 0; t < IB.nterms; ++t) {
          const auto sh = std::find(shared.begin(), shared.end(), t);
          if (sh == shared.end()) {
            o << "      lp += mmb_jn_" << IB.term[t] << "(A, vals, g, " << (IB.trans[t] ? "transform" : "0") << ");\n";
          } else {  // gen_node's MvNormal with the prep's (ss, bad)
            const int j = (int)(sh - shared.begin());
            const mmb_ir_node& N = ir.nodes[IB.term[t]];
            int tmp = 0;
            o << "      {\n      double sig;\n      {\n      const int i = 0;\n      (void)i;\n";
            const std::string sg = gen_expr(ir, N.expr[1], "i", o, tmp);
            o << "      sig = " << sg << ";\n      }\n";
            o << "      lp += pre[" << 2 * j + 1 << "] != 0.0 ? -__builtin_inf() : d_iso(" << N.len << ", sig, pre["
              << 2 * j << "]);\n      }\n";
          }
          o << "      if (!isfinite(lp)) break;\n";
        }
        o << "      break;\n";
      }
      o << "    default: break;\n  }\n  return lp;\n}\n";
      o << "__device__ __forceinline__ double mmb_jit_slice_cand(const SweepArgs& A, int blk, const double* vals,\n"
           "                                                     const double* c, int r, int transform,\n"
           "                                                     const double* pre) {\n"
           "  switch (blk) {\n";
      for (int b = 0; b < spec.nblocks; ++b) {
        if (spec.blocks[b].sampler != MMB_SAMPLER_SLICE) continue;
        int d = 0;
        for (int a = 0; a < spec.blocks[b].nnodes; ++a) d += ir.nodes[spec.blocks[b].nodes[a]].len;
        if (d > 4) continue;
        o << "    case " << b << ": return mmb_jc_" << b << "(A, vals, c, r, transform, pre);\n";
      }
      o << "    default: return __builtin_nan(\"\");\n  }\n}\n";
    }
  }
  // monitored Logical nodes (write_draws)
  o << "__device__ __forceinline__ double mmb_jit_logical(const SweepArgs& A, int n, int i, const double* vals) {\n"
       "  (void)A; (void)i; (void)vals;\n  switch (n) {\n";
  for (int q = 0; q < ir.nmon; ++q) {
    const int n = ir.mon[q];
    if (ir.nodes[n].family != MMB_IR_LOGICAL) continue;
    bool dup = false;
    for (int q2 = 0; q2 < q; ++q2) dup = dup || ir.mon[q2] == n;
    if (dup) continue;
    int tmp = 0;
    o << "    case " << n << ": {\n";
    const std::string r = gen_expr(ir, ir.nodes[n].expr[0], "i", o, tmp);
    o << "    return " << r << ";\n    }\n";
  }
  o << "    default: return 0.0;\n  }\n}\n\n#include \"sweep.h\"\n\n";
  o << "extern \"C\" __global__ __launch_bounds__(256, MMB_IR_WAVES) void mmb_ir_jit_kernel(const SweepArgs A) {\n"
       "  sweep_body<MMB_MODEL_IR, " << kinds << "u>(A);\n}\n";
  return o.str();
}

// the target of the specialised kernels is the library's own (build.py passes PYTORCH_ROCM_ARCH as
// MMB_ARCH), so they run wherever the static kernels do; it is part of the cache key via kOpts
#ifndef MMB_ARCH
#define MMB_ARCH "gfx950"
#endif
static const char* const kOpts[] = {"-O3", "--offload-arch=" MMB_ARCH, "-std=c++17", "-ffp-contract=off",
                                    "-mllvm", "-pragma-unroll-threshold=100000"};

int mmb_ir_jit_obtain(const std::string& src, std::vector<char>* code, std::string* info) {
  int maj = 0, mnr = 0;
  if (hiprtcVersion(&maj, &mnr) != HIPRTC_SUCCESS) { *info = "hipRTC unavailable"; return -1; }
  uint64_t h = 1469598103934665603ull;
  h = fnv1a(h, src.data(), src.size());
  for (int k = 0; k < mmb_jit_nheaders; ++k) {
    h = fnv1a(h, mmb_jit_header_names[k], strlen(mmb_jit_header_names[k]));
    h = fnv1a(h, mmb_jit_headers[k], strlen(mmb_jit_headers[k]));
  }
  for (const char* op : kOpts) h = fnv1a(h, op, strlen(op));
  h = fnv1a(h, &maj, sizeof maj);
  h = fnv1a(h, &mnr, sizeof mnr);
  char name[64];
  snprintf(name, sizeof name, "irjit_%016llx.co", (unsigned long long)h);
  if (const char* dump = std::getenv("MMB_JIT_DUMP")) {  // (inspection: the generated source)
    std::ofstream f(dump);
    if (f) f << src;
  }
  const char* env = std::getenv("MMB_JIT_CACHE");
  const std::string dir = env && *env ? std::string(env) : lib_dir() + "/jit";
  const std::string path = dir + "/" + name;
  if (read_file(path, *code)) {
    *info = std::string("cache hit ") + path;
    return 0;
  }
  const auto t0 = std::chrono::steady_clock::now();
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "mmb_ir_jit.hip", mmb_jit_nheaders, mmb_jit_headers,
                          mmb_jit_header_names) != HIPRTC_SUCCESS) {
    *info = "hiprtcCreateProgram failed";
    return -1;
  }
  const hiprtcResult r = hiprtcCompileProgram(prog, (int)(sizeof kOpts / sizeof kOpts[0]), kOpts);
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    *info = std::string("hipRTC compile failed: ") + hiprtcGetErrorString(r) + "\n" + log.substr(0, 4000);
    return -1;
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code->resize(n);
  hiprtcGetCode(prog, code->data());
  hiprtcDestroyProgram(&prog);
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  char msg[96];
  snprintf(msg, sizeof msg, "compiled in %.1f s", s);
  *info = msg;
  // best-effort cache write (atomic rename): a read-only tree only costs the next compile
  mkdir(dir.c_str(), 0755);
  const std::string tmp = path + ".tmp." + std::to_string((long)getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    if (f) f.write(code->data(), (std::streamsize)code->size());
  }
  if (rename(tmp.c_str(), path.c_str()) == 0) *info += std::string(", cached ") + path;
  else unlink(tmp.c_str());
  return 0;
}
