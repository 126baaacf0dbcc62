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
// element index `idx`; returns the temporary holding the value.
std::string gen_expr(const mmb_ir_model& ir, int pc, const std::string& idx, std::ostringstream& o, int& tmp) {
  std::vector<std::string> st;
  auto fresh = [&]() { return "t" + std::to_string(tmp++); };
  for (;; ++pc) {
    const uint32_t w = (uint32_t)ir.code[pc];
    const int op = (int)(w >> 24), arg = (int)(w & 0xffffffu);
    if (op == MMB_IR_OP_END) break;
    const std::string t = fresh();
    switch (op) {
      case MMB_IR_OP_CONST: o << "    const double " << t << " = " << lit(ir.consts[arg]) << ";\n"; break;
      case MMB_IR_OP_VAL: o << "    const double " << t << " = vals[" << arg << "];\n"; break;
      case MMB_IR_OP_VALI: o << "    const double " << t << " = vals[" << arg << " + " << idx << "];\n"; break;
      case MMB_IR_OP_VALG: {  // gather: the pool offset of the indices is the next word
        const int woff = ir.code[++pc];
        o << "    const double " << t << " = vals[" << arg << " + (int)A.ir_pool[" << woff << " + " << idx << "]];\n";
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
  o << "#define MMB_IR_JIT 1\n#define MMB_IR_DMAX " << dmax << "\n#include \"device.h\"\n\n";
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
