// hmc.h — HMC (src/samplers/hmc.jl:72-111) and MALA (src/samplers/mala.jl:67-86) as
// resumable machines, the same contract as nuts.h: advance() runs until it needs logf/grad
// at S.x (returns true; the caller fills S.lf and S.g and calls again) or the update is
// complete (returns false).  Line calls the model gradient inline; the logistic engine
// suspends the chain and evaluates the gradients of all chains as one batched MFMA GEMM.
//
// Vectors: element e in lane e % G, slot e / G (nuts.h layout).  SigmaL is chol(Sigma) lower,
// row-major d x d in global memory, or null for the reference's UniformScaling I.
// Arithmetic spec (restated by oracle/oracle.c orc_hmc / orc_mala):
//   L z      : out_e = sum_{k<=e} L[e,k] z_k, k ascending from 0.0
//   L' g     : out_k = sum_{i>=k} L[i,k] g_i, i ascending from 0.0
//   L^-1 w   : forward substitution, t_e = w_e - L[e,0]u_0 - ... - L[e,e-1]u_{e-1}, u_e = t_e / L[e,e]
//   sumabs2  : the NUTS dot (sequential per lane, then the group butterfly)
// MALA with Sigma: L = sqrt(eps) SigmaL entrywise, M2 g = 0.5 (L (L' g)) (reference: the
// explicit 0.5 L L' and inv(L); equal up to rounding).  With SigmaL = I the scalar forms
// of UniformScaling are used: L = sqrt(eps), Linv = 1/L, M2 = 0.5 (L L).
// Draws per update: d normals (momentum / proposal noise), then 1 uniform (accept).
#pragma once
#include "device.h"

enum : int32_t { HPC_BEGIN = 0, HPC_G0, HPC_STEP, HPC_MG1, HPC_DONE };

template <int G, int R>
struct HmcM {
  double v[R], x[R], p[R], g[R];
  double lf;            // logf at x (filled by the gradient provider)
  double logf0, k0;     // HMC: logf0, Kp0; MALA: logf0, q1
  int32_t pc, i;
};

template <int G, int R>
struct Hmc {
  using St = HmcM<G, R>;
  struct Env {
    int d, lane;
    int L;               // HMC leapfrog steps
    double eps;          // HMC/MALA epsilon
    const double* sigl;  // chol(Sigma) lower row-major, or null (I)
    mmb_rng rn, ru;
  };

  __device__ __forceinline__ static double dot(const Grp<G>& g, const double* a, int d) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r * G + g.lane < d) s = s + a[r] * a[r];
    return G == 1 ? s : g.sum(s);
  }
  // out = (sc L) in
  __device__ __forceinline__ static void lmul(const Grp<G>& g, const double* Lm, double sc, int d,
                                              const double* in, double* out) {
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0;
#pragma unroll
    for (int kr = 0; kr < R; ++kr)
      for (int kl = 0; kl < G; ++kl) {
        const int k = kr * G + kl;
        if (k >= d) break;
        const double zk = g.bcast(in[kr], kl);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int e = r * G + g.lane;
          if (e < d && k <= e) acc[r] = acc[r] + (sc * Lm[e * d + k]) * zk;
        }
      }
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = acc[r];
  }
  // out = (sc L)' in
  __device__ __forceinline__ static void ltmul(const Grp<G>& g, const double* Lm, double sc, int d,
                                               const double* in, double* out) {
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0;
#pragma unroll
    for (int ir = 0; ir < R; ++ir)
      for (int il = 0; il < G; ++il) {
        const int i = ir * G + il;
        if (i >= d) break;
        const double gi = g.bcast(in[ir], il);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int k = r * G + g.lane;
          if (k < d && i >= k) acc[r] = acc[r] + (sc * Lm[i * d + k]) * gi;
        }
      }
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = acc[r];
  }
  // w <- (sc L)^-1 w
  __device__ __forceinline__ static void lsolve(const Grp<G>& g, const double* Lm, double sc, int d, double* w) {
#pragma unroll
    for (int kr = 0; kr < R; ++kr)
      for (int kl = 0; kl < G; ++kl) {
        const int k = kr * G + kl;
        if (k >= d) break;
        if (g.lane == kl) w[kr] = w[kr] / (sc * Lm[k * d + k]);
        const double uk = g.bcast(w[kr], kl);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int e = r * G + g.lane;
          if (e < d && e > k) w[r] = w[r] - (sc * Lm[e * d + k]) * uk;
        }
      }
  }
  __device__ __forceinline__ static void normals(const Env& E, double* z) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = r * G + E.lane;
      z[r] = e < E.d ? mmb_normal(&E.rn, (uint32_t)e) : 0.0;
    }
  }
  // Kp = 0.5 * sumabs2(SigmaL^-1 p)  (hmc.jl:102-104)
  __device__ __forceinline__ static double kinetic(const Grp<G>& g, const Env& E, const double* p) {
    double w[R];
#pragma unroll
    for (int r = 0; r < R; ++r) w[r] = p[r];
    if (E.sigl) lsolve(g, E.sigl, 1.0, E.d, w);
    return 0.5 * dot(g, w, E.d);
  }

  // sample!(v::HMCVariate, logfgrad) (hmc.jl:72-111)
  __device__ static bool advance_hmc(St& S, const Env& E, const Grp<G>& g) {
    const double eps = E.eps;
    bool fin = false;
    switch (S.pc) {
      case HPC_BEGIN:  // x1 = v; logf0, grad0 = logfgrad(x1)
#pragma unroll
        for (int r = 0; r < R; ++r) S.x[r] = S.v[r];
        S.pc = HPC_G0;
        return true;
      case HPC_G0: {
        S.logf0 = S.lf;
        double z[R];
        normals(E, z);
        if (E.sigl) lmul(g, E.sigl, 1.0, E.d, z, S.p);  // p0 = SigmaL * randn(d)
        else
#pragma unroll
          for (int r = 0; r < R; ++r) S.p[r] = z[r];
        S.k0 = kinetic(g, E, S.p);
#pragma unroll
        for (int r = 0; r < R; ++r) S.p[r] = S.p[r] + (0.5 * eps) * S.g[r];
        S.i = 0;
        if (S.i < E.L) {
#pragma unroll
          for (int r = 0; r < R; ++r) S.x[r] = S.x[r] + eps * S.p[r];
          S.i = 1;
          S.pc = HPC_STEP;
          return true;
        }
        fin = true;  // L = 0: logf1, grad1 = logf0, grad0
        break;
      }
      case HPC_STEP:
#pragma unroll
        for (int r = 0; r < R; ++r) S.p[r] = S.p[r] + eps * S.g[r];
        if (S.i < E.L) {
#pragma unroll
          for (int r = 0; r < R; ++r) S.x[r] = S.x[r] + eps * S.p[r];
          S.i += 1;
          return true;
        }
        fin = true;
        break;
      default:
        return false;
    }
    if (fin) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        S.p[r] = S.p[r] - (0.5 * eps) * S.g[r];
        S.p[r] = S.p[r] * -1.0;
      }
      const double k1 = kinetic(g, E, S.p);
      const double u = mmb_uniform(&E.ru, 0u);
      if (u < mmb_exp((S.lf - k1) - (S.logf0 - S.k0))) {
#pragma unroll
        for (int r = 0; r < R; ++r) S.v[r] = S.x[r];
      }
      S.pc = HPC_DONE;
    }
    return false;
  }

  // M2 * grad -> out
  __device__ __forceinline__ static void m2mul(const Grp<G>& g, const Env& E, double s, const double* gr,
                                               double* out) {
    if (E.sigl) {
      double t[R];
      ltmul(g, E.sigl, s, E.d, gr, t);
      lmul(g, E.sigl, s, E.d, t, out);
#pragma unroll
      for (int r = 0; r < R; ++r) out[r] = 0.5 * out[r];
    } else {
      const double m2 = 0.5 * (s * s);
#pragma unroll
      for (int r = 0; r < R; ++r) out[r] = m2 * gr[r];
    }
  }
  // -0.5 * sumabs2(Linv * w)
  __device__ __forceinline__ static double qlog(const Grp<G>& g, const Env& E, double s, double* w) {
    if (E.sigl) lsolve(g, E.sigl, s, E.d, w);
    else {
      const double linv = 1.0 / s;
#pragma unroll
      for (int r = 0; r < R; ++r) w[r] = linv * w[r];
    }
    return -0.5 * dot(g, w, E.d);
  }

  // sample!(v::MALAVariate, logfgrad) (mala.jl:67-86)
  __device__ static bool advance_mala(St& S, const Env& E, const Grp<G>& g) {
    const double s = sqrt(E.eps);
    switch (S.pc) {
      case HPC_BEGIN:
#pragma unroll
        for (int r = 0; r < R; ++r) S.x[r] = S.v[r];
        S.pc = HPC_G0;
        return true;
      case HPC_G0: {  // y = v + M2 grad0 + L randn(d);  q1 (needs grad0) computed now
        S.logf0 = S.lf;
        double z[R], lz[R], w[R];
        normals(E, z);
        m2mul(g, E, s, S.g, S.p);
        if (E.sigl) lmul(g, E.sigl, s, E.d, z, lz);
        else
#pragma unroll
          for (int r = 0; r < R; ++r) lz[r] = s * z[r];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          S.x[r] = (S.v[r] + S.p[r]) + lz[r];
          w[r] = (S.x[r] - S.v[r]) - S.p[r];
        }
        S.k0 = qlog(g, E, s, w);  // q1
        S.pc = HPC_MG1;
        return true;
      }
      case HPC_MG1: {
        double m[R], w[R];
        m2mul(g, E, s, S.g, m);
#pragma unroll
        for (int r = 0; r < R; ++r) w[r] = (S.v[r] - S.x[r]) - m[r];
        const double q0 = qlog(g, E, s, w);
        const double u = mmb_uniform(&E.ru, 0u);
        if (u < mmb_exp((S.lf - S.k0) - (S.logf0 - q0))) {
#pragma unroll
          for (int r = 0; r < R; ++r) S.v[r] = S.x[r];
        }
        S.pc = HPC_DONE;
        return false;
      }
      default:
        return false;
    }
  }
};
