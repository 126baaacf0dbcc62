// logistic.h — device state of the batched-gradient engine (BASELINE config 4: NUTS; also HMC, MALA).
//
// Model (build-defined after doc/examples/surgical.jl:14-24):
//   y[n] ~ Bernoulli(invlogit(X[n,:] beta)),  beta ~ MvNormal(p, prior_sd),  scheme [NUTS(:beta)].
// One wave per chain runs the NUTS machine of nuts.h (lane e <-> beta[e], p <= 64) in
// lg_ctl_kernel until every chain either needs logf/grad at its leapfrog position or has
// finished the window; lg_grad_kernel then evaluates all requested gradients at once as
// two f64 MFMA GEMMs, X * B and X' * R, with the residual nonlinearity fused in between.
#pragma once
#include <stdint.h>

#include "mmb_math.h"

#define MMB_LG_NVEC 12  // machine vectors kept per chain besides v (nuts.h NutsM order)
#define MMB_LG_NSC 16
#define MMB_LG_NIV 16
#define MMB_LG_SPLIT_MAX 4  // independent chain parts of a window, one stream each (engine.cpp run_logistic)

struct LgArgs {
  int32_t kind;            // mmb_sampler_kind of the single block: NUTS, HMC or MALA
  int32_t K, p, N, rps;    // chains, coefficients, rows, rows per sub-range (mmb_lg_rps)
  int32_t Np;              // padded rows = MMB_LG_NG * MMB_LG_NS * rps
  uint32_t chain_offset;
  uint64_t seed;
  int64_t iter0, it_end;   // window = iter0+1 .. it_end
  int64_t burnin, thin, model_burnin, kept_origin;
  double prior_sd, target;
  const double* X;         // [Np][64] row-major, zero padded (rows and columns)
  const double* y;         // [N_pad]
  double* vals;            // [K][64] beta (the NUTS variate v)
  double* vec;             // [K][MMB_LG_NVEC][64]
  double* sc;              // [K][MMB_LG_NSC]
  int32_t* iv;             // [K][MMB_LG_NIV]
  int64_t* itc;            // [K] last completed iteration
  double* frames;          // [K][NutsFrames<64>::DBL]
  double* tune;            // NUTS [K][8] eps, epsbar, Hbar, mu, alpha, nalpha | HMC/MALA [K][2] epsilon, L
  const double* sigl;      // HMC/MALA chol(Sigma) lower row-major p x p, or null (I)
  int32_t* tm;             // [K] m
  int32_t* tflags;         // [K]
  double* draws;           // [n_kept][p][Kd] or null (this launch's chains from column 0)
  int32_t Kd;              // draws column stride: the engine's chains (a window may run its chains
                           // as independent halves, engine.cpp run_logistic)
  // gradient exchange between the two kernels
  double* pos;             // [K][64] positions of the chains that requested a gradient (slot order)
  double* gpart;           // [MMB_LG_NG * MMB_LG_NS][K][64] sub-range partials (one workgroup each)
  double* lpart;           // [MMB_LG_NG * MMB_LG_NS][K]
  int32_t* count;          // [2] requests in the current step (ping-pong by step parity)
  int32_t* s2c;            // [2][K] requesting chain of each slot (ping-pong): the next control
                           //        kernel visits exactly these chains (every running chain
                           //        requests one gradient per step)
  unsigned long long* ngrad;  // total gradient evaluations of the window
  unsigned long long* nstat;  // NUTS {updates, depth-cap hits, depth sum} (nuts.h Env::stat)
  // gradient scheme: fd = 0 the analytic gradient (one column per request), fd = 1 Calculus
  // forward differences (simulation.jl:47-51, the reference's default dtype=:forward): nv = p + 1
  // logpdf! columns per request -- the position and each coordinate moved by its epsilon -- as
  // virtual columns slot * nv + k of the gradient kernel (log-density partials only)
  int32_t fd, nv;
  int64_t Kv;              // column stride of the partial arrays: K (analytic) or K * nv (fd)
};
