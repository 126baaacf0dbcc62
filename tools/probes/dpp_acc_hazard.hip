// Probe: does a v_fmac_f64_dpp need wait states after a VALU write of its ACCUMULATOR (src2 /
// vdst), as opposed to its DPP source (src0)?  LLVM's hazard recognizer treats every VGPR use of
// a DPP instruction as a DPP read and pads the factorization's two-accumulator dot product with an
// s_nop 0 after each pair of fmacs.  Here one asm block holds chains with the accumulator
// rewritten by the instruction right before its next read (alternating: one instruction between;
// back to back: none), run by one wave alone on the chip (nothing to interleave), against a
// control with five wait states before every fmac and against the same fmas formed on the host.
//   hipcc --offload-arch=gfx950 -O3 dpp_acc_hazard.hip -o probe && ./probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

#define FM0(acc, n) "v_fmac_f64_dpp " acc ", %4, %5 row_newbcast:" #n " row_mask:0xf bank_mask:0xf\n\t"
#define FMP(acc, n) "s_nop 4\n\tv_fmac_f64_dpp " acc ", %4, %5 row_newbcast:" #n " row_mask:0xf bank_mask:0xf\n\t"

#define PROBE_BODY(FM)                                                                           \
  const int t = threadIdx.x;                                                                     \
  double x = in[t], b = in[64 + t];                                                              \
  double a0 = 1.0, a1 = 2.0, a2 = 3.0, a3 = 4.0;                                                 \
  for (int r = 0; r < reps; ++r) {                                                               \
    asm volatile("s_nop 4\n\t" FM("%0", 1) FM("%1", 2) FM("%0", 3) FM("%1", 4) FM("%0", 5)       \
                 FM("%1", 6) FM("%0", 7) FM("%1", 8)                                             \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(b));                     \
    asm volatile("s_nop 4\n\t" FM("%2", 9) FM("%2", 10) FM("%2", 11) FM("%3", 12) FM("%3", 13)   \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(b));                     \
    x = __builtin_fma(x, 0.999, 1e-3);                                                           \
    b = __builtin_fma(b, 0.998, 2e-3);                                                           \
  }                                                                                              \
  out[t] = a0; out[64 + t] = a1; out[128 + t] = a2; out[192 + t] = a3;

__global__ void probe_bare(double* out, const double* in, int reps) { PROBE_BODY(FM0) }
__global__ void probe_padded(double* out, const double* in, int reps) { PROBE_BODY(FMP) }

static double bc(const double* v, int lane, int n) { return v[(lane & ~15) + n]; }

static int check(const char* e) {
  if (e) { fprintf(stderr, "%s\n", e); return 1; }
  return 0;
}

int main() {
  const int reps = 200;
  double h_in[128], bare[256], padded[256], ref[256];
  for (int i = 0; i < 128; ++i) h_in[i] = 1.0 + 1e-3 * ((i * 37) % 101) - 0.05;
  double *d_in, *d_out;
  if (hipMalloc(&d_in, sizeof h_in) != hipSuccess || hipMalloc(&d_out, sizeof bare) != hipSuccess)
    return check("hipMalloc failed");
  if (hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice) != hipSuccess) return check("copy in");
  hipLaunchKernelGGL(probe_bare, dim3(1), dim3(64), 0, 0, d_out, d_in, reps);
  if (hipMemcpy(bare, d_out, sizeof bare, hipMemcpyDeviceToHost) != hipSuccess) return check("copy out");
  hipLaunchKernelGGL(probe_padded, dim3(1), dim3(64), 0, 0, d_out, d_in, reps);
  if (hipMemcpy(padded, d_out, sizeof padded, hipMemcpyDeviceToHost) != hipSuccess) return check("copy out");
  double x[64], b[64], a[4][64];
  for (int t = 0; t < 64; ++t) {
    x[t] = h_in[t]; b[t] = h_in[64 + t];
    a[0][t] = 1; a[1][t] = 2; a[2][t] = 3; a[3][t] = 4;
  }
  for (int r = 0; r < reps; ++r) {
    for (int t = 0; t < 64; ++t) {
      for (int n = 1; n <= 8; ++n) a[(n - 1) & 1][t] = std::fma(bc(x, t, n), b[t], a[(n - 1) & 1][t]);
      for (int n = 9; n <= 11; ++n) a[2][t] = std::fma(bc(x, t, n), b[t], a[2][t]);
      for (int n = 12; n <= 13; ++n) a[3][t] = std::fma(bc(x, t, n), b[t], a[3][t]);
    }
    for (int t = 0; t < 64; ++t) { x[t] = std::fma(x[t], 0.999, 1e-3); b[t] = std::fma(b[t], 0.998, 2e-3); }
  }
  for (int k = 0; k < 4; ++k) for (int t = 0; t < 64; ++t) ref[64 * k + t] = a[k][t];
  int bad[4] = {0, 0, 0, 0}, badp = 0;
  double maxrel = 0.0;
  for (int i = 0; i < 256; ++i) {
    if (bare[i] != ref[i]) bad[i / 64]++;
    if (padded[i] != ref[i]) badp++;
    maxrel = std::fmax(maxrel, std::fabs(bare[i] - ref[i]) / std::fabs(ref[i]));
  }
  printf("{\"probe\": \"dpp_acc_hazard\", \"reps\": %d, \"padded_mismatch\": %d, "
         "\"bare_mismatch_alternating\": [%d, %d], \"bare_mismatch_back_to_back\": [%d, %d], "
         "\"bare_max_rel_diff\": %.3g}\n",
         reps, badp, bad[0], bad[1], bad[2], bad[3], maxrel);
  return (badp | bad[0] | bad[1] | bad[2] | bad[3]) ? 1 : 0;
}
