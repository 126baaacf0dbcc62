// device.h — shared device-side definitions for the sweep kernels.
//
// Execution model: one chain is advanced by a *group* of G
// lanes of a wave64 (G = 32 for rats: lane i <-> rat i / block element i, two
// chains per wave; G = 1 for line: one chain per lane).  Element e of a block's
// unlisted vector lives in lane e % G, register slot e / G (R slots per lane).
// Group-uniform control flow only; group reductions are xor-butterflies inside
// the G-aligned lane group, so every lane of a group ends with the same value.
#pragma once
#if !defined(__HIPCC_RTC__)  // hipRTC (the node-IR JIT, engine.cpp) brings its own runtime header
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "../../include/mamba_hip.h"
#include "mmb_math.h"
#include "ir_math.h"

#define MMB_MAXB MMB_MAX_BLOCKS

// lane's bit of a wave mask.  hipRTC's compiler (the one torch bundles) lacks the wave64 builtin;
// there the bit is extracted by the lane id (node-IR specialised kernels only).
__device__ __forceinline__ bool mmb_inverse_ballot(uint64_t m) {
#if defined(__HIPCC_RTC__)
  return ((m >> (threadIdx.x & 63)) & 1ull) != 0ull;
#else
  return __builtin_amdgcn_inverse_ballot_w64(m);
#endif
}

// compile-time bool tag (a std::integral_constant without <type_traits>, which hipRTC lacks)
template <bool B>
struct mmb_bc {
  static constexpr bool value = B;
  constexpr operator bool() const { return B; }
};

// Correctly rounded sqrt(x) and 1/y for operands well inside the normal range, without the
// range handling of the generic sequences.  For x in [2^-700, 2^700] these are the very
// instruction sequences the compiler emits for sqrt() / 1.0 / y (ocml: rsq + Goldschmidt +
// two corrections; fdiv: rcp + two Newton steps + one correction) with the no-op parts
// dropped: no 2^256 input scaling (x >= 2^-767), v_div_scale / v_div_fmas leave operands
// unscaled (exponents within 768 of 1.0) and v_div_fixup passes finite non-zero quotients
// through.  So they return the IEEE results bit for bit (the oracle uses C sqrt and /).
// Callers check the range and take sqrt() / division otherwise.
__device__ __forceinline__ bool mmb_fast_range(double x) { return x >= 0x1p-700 && x <= 0x1p700; }
__device__ __forceinline__ double mmb_sqrt_inrange(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
}
__device__ __forceinline__ double mmb_rcp_inrange(double y) {
  double r = __builtin_amdgcn_rcp(y);
  double e = fma(-y, r, 1.0);
  r = fma(r, e, r);
  e = fma(-y, r, 1.0);
  r = fma(r, e, r);
  e = fma(-y, r, 1.0);
  return fma(e, r, r);
}
// Both for the pivoted Cholesky: s = sqrt(x), r = 1.0 / s.  (A shorter reciprocal seeded by
// the square root's Goldschmidt half-reciprocal, one Newton step and the final correction,
// matched on 2^32 random samples but returned wrong last bits near binade boundaries --
// x within 8 ulps of a power of two, sqrt(x) with an all-ones significand -- in the directed
// set of tools/sqrt_rcp_check.hip; the rcp-seeded sequence matches there as well.)
__device__ __forceinline__ void mmb_sqrt_rcp_inrange(double x, double* s, double* rcp) {
  *s = mmb_sqrt_inrange(x);
  *rcp = mmb_rcp_inrange(*s);
}

// AMM factorization counters per chain (mmb_amm_stats fields; 64-bit: a chain adds up to d = 30 to
// the rank and step sums per update, which would wrap 32 bits after ~1.4e8 updates; padded to 64 bytes)
#define MMB_AMM_STAT_STRIDE 8

// Per-block descriptor passed in kernel arguments (constant memory, uniform access).
struct DBlock {
  int32_t kind, nn, d, transform, form, adapt, batchsize, sigl_diag;
  int32_t nodes[4];
  int32_t emap[4];       // line/rats scalar blocks: element -> value index / node id
  double target, beta, scale;
  double width0;         // Slice: scalar width
  const double* width;   // Slice: widths[d] (device) or null when scalar
  const double* sigl;    // AMM, HMC/MALA: chol(Sigma) lower, row-major d x d (device); HMC/MALA: null = I
  // tune state (device, chain-major)
  double* t_sigma;       // AMWG  [K][DP]
  double* t_accept;      // AMWG  [K][DP]
  int32_t* t_m;          // AMWG/AMM/NUTS m [K]
  int32_t* t_flags;      // [K] bit0 adapt, bit1 AMM alias, bit2 AMM factor valid, bit3 NUTS init
  double* t_Mv;          // AMM   [K][DP]
  double* t_Mvv;         // AMM   [K][TP] packed lower, row-major (slot(i,k) = i(i+1)/2 + k)
  double* t_Ls;          // AMM   [K][TP] factor, in-place slot storage
  uint8_t* t_piv;        // AMM   [K][DP] pivot order
  double* t_xnext;       // AMM   [K][DP] next iteration's proposal minus v (samplers.h amm: formed
                         //       with the factor still in registers), valid when t_xtag[c] matches
  int64_t* t_xtag;       // AMM   [K] (xepoch << 32) | iteration the carried proposal is for
  uint64_t* t_astat;     // AMM   [K][MMB_AMM_STAT_STRIDE] factorization counters (mmb_amm_stats), diagnostics
  double* t_nuts;        // NUTS  [K][8] eps, epsbar, Hbar, mu, alpha, nalpha, -, -
  double* t_nfr;         // NUTS  [K][NutsFrames<DV>::DBL] tree frames (scratch, nuts.h)
  double* t_hmc;         // HMC/MALA [K][2] epsilon, L (HMCTune / MALATune, hmc.jl:5-28)
  int32_t ir_blk;        // node IR: index into SweepArgs::ir_blocks
  int32_t fdgrad;        // NUTS/HMC/MALA on line: 1 = Calculus forward differences (mmb_gradient)
  const int32_t* sep;    // node-IR AMWG block whose logpdf! separates by coordinate (engine.cpp ir_sep_table):
                         // [d + 2 offsets][entries (term << 24 | element)], entries of coordinate j at
                         // off[j] .. off[j+1], elements on no coordinate at off[d] .. off[d+1]; null: none
  double sep_eps;        // its lane-parallel decision's relative rounding band (ir.h amwg_dm)
};

struct SweepArgs {
  int32_t K;             // chains in this shard
  uint32_t chain_offset; // global id of chain 0
  uint64_t seed;
  int64_t iter0;         // window starts at iter0+1
  int32_t n_iters;
  int32_t nb;
  int64_t burnin, thin, model_burnin;
  int64_t kept_base;     // kept rows before this launch (within the mmb_run window)
  int64_t kept_origin;   // kept count at the window start (rows are relative to the window)
  double* vals;          // model-specific device layout
  int64_t xepoch;        // bumped by every host write of chain state (invalidates carried proposals)
  unsigned long long* nuts_stat;  // NUTS {updates, depth-cap hits, depth sum} (nuts.h Env::stat),
                                  // [3] Slice updates stopped at MMB_SLICE_MAX_SHRINK,
                                  // [5] AMWG block updates that took the sequential path
  double* draws;         // [n_kept][pmon][K] or null
  const double* data0;   // model data (rats: y[150]; line: x[5], y[5] packed as 10)
  double ig_c;           // 0.001 log(0.001) - lgamma(0.001)
  double xbar;           // rats
  double xm[5];          // rats: x - xbar
  double lx[5], ly[5];   // line data
  const DBlock* blocks;  // device array [nb] (uniform, scalar-cache loads)
  // node IR (MMB_MODEL_IR, ir.h): tables, state row length, LDS layout per chain
  const mmb_ir_node* ir_nodes;
  const int32_t* ir_code;
  const double* ir_const;
  const double* ir_pool;
  const mmb_ir_block* ir_blocks;
  const int32_t* ir_mon;
  int32_t ir_nmon, ir_pmon;
  int32_t ir_vs;         // doubles per chain row of `vals` (P rounded up to 32)
  int32_t ir_amm;        // AMM scratch doubles at the start of a chain's LDS (0 without AMM)
  int32_t ir_lds;        // LDS doubles per chain
  const int32_t* cperm;  // lane-group slot -> chain (null: identity), sweep.hip order_chains_kernel
  int32_t amwg_exact;    // MMB_AMWG_EXACT: 1 = AMWG takes amwg_sub!'s sequential loop (samplers.h amwg),
                         // 2 = AMWG certainty band widened 2^30 times (tests: frequent fallback)
  int32_t slice_exact;   // MMB_SLICE_EXACT=1: Slice evaluates one shrink candidate at a time (slice_uni /
                         // slice_multi) instead of four per round
  int32_t amwg_probe;    // MMB_AMWG_PROBE=1 (tests only): near-threshold AMWG accept uniforms
                         // (mmb_math.h mmb_amwg_probe_factor)
};

// Wavefront pairing (sweep.hip order_chains_kernel): classes from the first MMB_ORDER_BLOCKS AMM
// blocks' factor-valid flags
#define MMB_ORDER_BLOCKS 3
struct OrderArgs {
  const int32_t* flags[MMB_ORDER_BLOCKS];  // AMM blocks' t_flags, [K] each
  int32_t nblk;
  int32_t K;
  int32_t cpw;                             // chains per workgroup of the sweep kernel
  int32_t mode;                            // 0 ascending class order, 1 descending, 2 balanced workgroups
  int32_t* perm;                           // out: slot -> chain
};

// Block descriptors are read-only for a launch: read them through the constant address
// space so uniform accesses become scalar loads (s_load, scalar cache).
__device__ __forceinline__ const DBlock& mmb_block(const DBlock* p, int b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const DBlock*)&((const __attribute__((address_space(4))) DBlock*)p)[b];
#else
  return p[b];
#endif
}

MMB_HD int mmb_tri(int i) { return (i * (i + 1)) >> 1; }
MMB_HD int mmb_slot(int i, int k) { return i >= k ? mmb_tri(i) + k : mmb_tri(k) + i; }

// wave-scope compiler/memory ordering between a lane's LDS write and another lane's read
__device__ __forceinline__ void grp_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- cross-lane primitives for 32-lane groups: DPP / permlane (no LDS round trip) ----
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  // quad_perm / row_mirror / row_half_mirror read a valid lane for every lane, so no
  // "old" operand is needed (bound_ctrl): no extra v_mov per DPP move
  return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  uint64_t u = mmb_d2u(x);
  int lo = dpp_i<CTRL>((int)(uint32_t)u), hi = dpp_i<CTRL>((int)(uint32_t)(u >> 32));
  return mmb_u2d((uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32));
}
// value of lane ^ 16 (rows 0<->1 and 2<->3 of the wave)
__device__ __forceinline__ int swap16_i(int x) {
  auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
  return (int)((threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ double swap16_d(double x) {
  uint64_t u = mmb_d2u(x);
  int lo = swap16_i((int)(uint32_t)u), hi = swap16_i((int)(uint32_t)(u >> 32));
  return mmb_u2d((uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32));
}
// acc = fma(b, x of lane n of this lane's 16-lane row, acc): one v_fmac_f64 with a 64-bit DPP
// row_newbcast source (gfx950 DPP64), i.e. a row broadcast without an LDS read per lane.  A source
// lane disabled in EXEC would read as "no write", so callers keep every lane of the row active.
// The compiler's hazard recognizer does not look inside inline asm, so the first use of a
// source value (first = true) starts with the two wait states a DPP read needs after a VALU
// write of its source; later uses of the same value follow DPP instructions only.
template <int N, bool FIRST>
__device__ __forceinline__ void fmac_rowbc(double& acc, double x, double b) {
  if constexpr (FIRST)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(x), "v"(b), "n"(N));
  else
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(x), "v"(b), "n"(N));
}
__device__ __forceinline__ void fmac_rowbc_nf(double& acc, double x, double b, int n, bool first);
// n = k % 16 of a dot product over k ascending: the uses at k = 0 and k = 16 are first uses
__device__ __forceinline__ void fmac_rowbc_n(double& acc, double x, double b, int n) {
  switch (n) {  // n is a constant after unrolling: one case survives
#define MMB_RBC(i) case i: fmac_rowbc<i, i == 0>(acc, x, b); break;
    MMB_RBC(0) MMB_RBC(1) MMB_RBC(2) MMB_RBC(3) MMB_RBC(4) MMB_RBC(5) MMB_RBC(6) MMB_RBC(7)
    MMB_RBC(8) MMB_RBC(9) MMB_RBC(10) MMB_RBC(11) MMB_RBC(12) MMB_RBC(13) MMB_RBC(14) MMB_RBC(15)
#undef MMB_RBC
  }
}

// as fmac_rowbc_n for a source last written by an LDS read, not by a VALU instruction: the DPP
// read-after-VALU-write hazard does not apply and no use needs wait states (tests/test_isa.py
// checks the built code for VALU writes of every DPP source)
__device__ __forceinline__ void fmac_rowbc_ld(double& acc, double x, double b, int n) {
#ifdef MMB_EXP_DPPNOP
  fmac_rowbc_n(acc, x, b, n);
#else
  fmac_rowbc_nf(acc, x, b, n, false);
#endif
}

// as fmac_rowbc_n with the first use of the source at an explicit step (a dot product whose
// first products are formed otherwise)
__device__ __forceinline__ void fmac_rowbc_nf(double& acc, double x, double b, int n, bool first) {
  if (first) {
    switch (n) {
#define MMB_RBC(i) case i: fmac_rowbc<i, true>(acc, x, b); break;
      MMB_RBC(0) MMB_RBC(1) MMB_RBC(2) MMB_RBC(3) MMB_RBC(4) MMB_RBC(5) MMB_RBC(6) MMB_RBC(7)
      MMB_RBC(8) MMB_RBC(9) MMB_RBC(10) MMB_RBC(11) MMB_RBC(12) MMB_RBC(13) MMB_RBC(14) MMB_RBC(15)
#undef MMB_RBC
    }
  } else {
    switch (n) {
#define MMB_RBC(i) case i: fmac_rowbc<i, false>(acc, x, b); break;
      MMB_RBC(0) MMB_RBC(1) MMB_RBC(2) MMB_RBC(3) MMB_RBC(4) MMB_RBC(5) MMB_RBC(6) MMB_RBC(7)
      MMB_RBC(8) MMB_RBC(9) MMB_RBC(10) MMB_RBC(11) MMB_RBC(12) MMB_RBC(13) MMB_RBC(14) MMB_RBC(15)
#undef MMB_RBC
    }
  }
}

// stage s of the 32-lane all-reduce: partner lanes xor1, xor2 (quad_perm), 7-i (row_half_mirror),
// 15-i (row_mirror), i^16 (permlane16_swap).  After stage s every lane of the 2^(s+1) subgroup
// holds the same (commutative) combination.
#define MMB_DPP_XOR1 0xB1
#define MMB_DPP_XOR2 0x4E
#define MMB_DPP_HMIRROR 0x141
#define MMB_DPP_MIRROR 0x140

template <int G>
struct Grp {
  int lane;
  __device__ __forceinline__ Grp() : lane((int)(threadIdx.x & (G - 1))) {}
  template <int S>
  __device__ __forceinline__ static double other_d(double x) {
    if (S == 0) return dpp_d<MMB_DPP_XOR1>(x);
    if (S == 1) return dpp_d<MMB_DPP_XOR2>(x);
    if (S == 2) return dpp_d<MMB_DPP_HMIRROR>(x);
    if (S == 3) return dpp_d<MMB_DPP_MIRROR>(x);
    return swap16_d(x);
  }
  template <int S>
  __device__ __forceinline__ static int other_i(int x) {
    if (S == 0) return dpp_i<MMB_DPP_XOR1>(x);
    if (S == 1) return dpp_i<MMB_DPP_XOR2>(x);
    if (S == 2) return dpp_i<MMB_DPP_HMIRROR>(x);
    if (S == 3) return dpp_i<MMB_DPP_MIRROR>(x);
    return swap16_i(x);
  }
  __device__ __forceinline__ double sum(double x) const {
    if (G == 32) {
      x += other_d<0>(x); x += other_d<1>(x); x += other_d<2>(x); x += other_d<3>(x);
      x += other_d<4>(x);
      return x;
    }
    if (G == 16) {  // one DPP row: four stages, no permlane
      x += other_d<0>(x); x += other_d<1>(x); x += other_d<2>(x); x += other_d<3>(x);
      return x;
    }
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
  }
  __device__ __forceinline__ void sum2(double& x, double& y) const {
    if (G == 32) {
      x += other_d<0>(x); y += other_d<0>(y);
      x += other_d<1>(x); y += other_d<1>(y);
      x += other_d<2>(x); y += other_d<2>(y);
      x += other_d<3>(x); y += other_d<3>(y);
      x += other_d<4>(x); y += other_d<4>(y);
      return;
    }
    if (G == 16) {
      x += other_d<0>(x); y += other_d<0>(y);
      x += other_d<1>(x); y += other_d<1>(y);
      x += other_d<2>(x); y += other_d<2>(y);
      x += other_d<3>(x); y += other_d<3>(y);
      return;
    }
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
      double a = __shfl_xor(x, m, 64);
      double b = __shfl_xor(y, m, 64);
      x += a;
      y += b;
    }
  }
  // four independent sums, stage by stage (each as sum() would form it)
  __device__ __forceinline__ void sum4(double& x, double& y, double& z, double& w) const {
    if (G == 32) {
      x += other_d<0>(x); y += other_d<0>(y); z += other_d<0>(z); w += other_d<0>(w);
      x += other_d<1>(x); y += other_d<1>(y); z += other_d<1>(z); w += other_d<1>(w);
      x += other_d<2>(x); y += other_d<2>(y); z += other_d<2>(z); w += other_d<2>(w);
      x += other_d<3>(x); y += other_d<3>(y); z += other_d<3>(z); w += other_d<3>(w);
      x += other_d<4>(x); y += other_d<4>(y); z += other_d<4>(z); w += other_d<4>(w);
      return;
    }
    sum2(x, y);
    sum2(z, w);
  }
  __device__ __forceinline__ double bcast(double x, int src) const {
    if (G == 1) return x;
    int base = (int)(threadIdx.x & 63) & ~(G - 1);
    return __shfl(x, base + src, 64);
  }
  __device__ __forceinline__ int bcast_i(int x, int src) const {
    if (G == 1) return x;
    int base = (int)(threadIdx.x & 63) & ~(G - 1);
    return __shfl(x, base + src, 64);
  }
  template <int S>
  __device__ __forceinline__ static void amax_stage(double& key, int& pi) {
    double ok = other_d<S>(key);
    int op = other_i<S>(pi);
    bool take = (ok > key) || (ok == key && op < pi);
    key = take ? ok : key;
    pi = take ? op : pi;
  }
  // Lexicographic argmax: larger key wins, ties -> smaller position.  pi = pos << 16 | idx
  // (pos, idx < 2^15), so comparing pi compares positions.
  __device__ __forceinline__ void argmax(double& key, int& pi) const {
    if (G == 32) {
      amax_stage<0>(key, pi); amax_stage<1>(key, pi); amax_stage<2>(key, pi);
      amax_stage<3>(key, pi); amax_stage<4>(key, pi);
      return;
    }
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {
      double ok = __shfl_xor(key, m, 64);
      int op = __shfl_xor(pi, m, 64);
      bool take = (ok > key) || (ok == key && op < pi);
      key = take ? ok : key;
      pi = take ? op : pi;
    }
  }
};

// Phase timing (profiling builds only, -DMMB_PHASE_PROF): per-phase s_memtime cycles summed
// over lane groups into mmb_prof[]; engine.cpp prints them at mmb_destroy.
#ifdef MMB_PHASE_PROF
extern __device__ unsigned long long mmb_prof[32];
// per-wave accumulators in LDS (lane 0 of each wave), flushed once per kernel
__device__ __forceinline__ unsigned long long* mmb_prof_lds() {
  __shared__ unsigned long long p[4][16];
  return p[threadIdx.x >> 6];
}
#define MMB_PROF_START uint64_t _mmb_t0 = __builtin_amdgcn_s_memtime();
#define MMB_PROF_MARK(i, lane)                                              \
  {                                                                         \
    uint64_t _mmb_t1 = __builtin_amdgcn_s_memtime();                        \
    if ((threadIdx.x & 63) == 0) mmb_prof_lds()[(i)] += _mmb_t1 - _mmb_t0;  \
    _mmb_t0 = _mmb_t1;                                                      \
  }
#else
#define MMB_PROF_START
#define MMB_PROF_MARK(i, lane)
#endif

// Julia min(a, b): NaN propagates
__device__ __forceinline__ double jmin(double a, double b) {
  if (isnan(a)) return a;
  if (isnan(b)) return b;
  return b < a ? b : a;
}

// StatsFuns normlogpdf(mu, sig, x) with insupport(Normal, x)
__device__ __forceinline__ double d_normlogpdf(double mu, double sig, double logsig, double x) {
  if (isnan(x)) return -__builtin_inf();
  double z = (x - mu) / sig;
  return -(z * z + MMB_LOG2PI) / 2.0 - logsig;
}
// InverseGamma(0.001, 0.001) with insupport 0 <= x <= Inf, + log(x) Jacobian when transformed
__device__ __forceinline__ double d_iglogpdf(double igc, double x, int transform) {
  if (!(0.0 <= x && x <= __builtin_inf())) return -__builtin_inf();
  double lx = mmb_log(x);
  double lp = igc - (0.001 + 1.0) * lx - 0.001 / x;
  return transform ? lp + lx : lp;
}
// IsoNormal via PDMats ScalMat: -0.5*(k*log2pi + k*log(sig^2) + ssq/sig^2)
__device__ __forceinline__ double d_iso(int k, double sig, double ssq) {
  double value = sig * sig;
  double invv = 1.0 / value;
  return -0.5 * ((k * MMB_LOG2PI + k * mmb_log(value)) + ssq * invv);
}
