// samplers.h — block updates of src/samplers/{amwg,amm,slice}.jl for one chain
// advanced by a group of G lanes (element e of the block vector in lane e % G,
// register slot e / G).  RNG consumption follows mmb_math.h's documented layout and
// is mirrored draw for draw by oracle/oracle.c.
#pragma once
#include "models.h"

template <class M>
struct Smp {
  static constexpr int G = M::G, R = M::R, DMAX = M::DMAX, DP = M::DP, TP = M::TP;
  using St = typename M::St;
  using Lc = typename M::Lc;

  // ---------------------------------------------------------------- AMWG
  // amwg.jl:68-115 (sample!, setadapt!, amwg_sub!).
  __device__ __forceinline__ static void amwg(const SweepArgs& A, const DBlock& B, int c, const mmb_rng& rn,
                              const mmb_rng& ru, bool adapt, St& s, const Lc& l, const Grp<G>& g) {
    const int d = B.d;
    double x[R], sig[R], acc[R], z[R];
    M::unlist(B, s, g.lane, x);
    int m = B.t_m[c];
    int fl = B.t_flags[c];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      sig[r] = e < d ? B.t_sigma[(size_t)c * DP + e] : 0.0;
      acc[r] = e < d ? B.t_accept[(size_t)c * DP + e] : 0.0;
    }
    if (adapt && !(fl & 1)) {  // setadapt!: accept[:] = 0, m = 0
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.0;
      m = 0;
    }
    fl = adapt ? (fl | 1) : (fl & ~1);
    const double ad = adapt ? 1.0 : 0.0;
    if (adapt) m += 1;
    double logf0 = M::logf(A, B, s, l, g, x);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      z[r] = e < d ? sig[r] * mmb_normal(&rn, 2u * (uint32_t)e) : 0.0;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      for (int ln = 0; ln < G; ++ln) {
        int e = r * G + ln;
        if (e >= d) break;
        bool own = g.lane == ln;
        double xo = x[r];
        if (own) x[r] += z[r];
        double lpp = M::logf(A, B, s, l, g, x);
        if (mmb_uniform(&ru, (uint32_t)e) < mmb_exp(lpp - logf0)) {
          logf0 = lpp;
          if (own) acc[r] += ad;
        } else if (own) {
          x[r] = xo;
        }
      }
    }
    if (adapt && m % B.batchsize == 0) {  // amwg.jl:74-79 ((m/b)^-0.5 as 1/sqrt(m/b))
      double q = (double)m / (double)B.batchsize;
      double delta = 1.0 / sqrt(q);
      if (0.01 < delta) delta = 0.01;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        double eps = (acc[r] / (double)m < B.target) ? -delta : delta;
        sig[r] *= mmb_exp(eps);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      if (e < d) {
        B.t_sigma[(size_t)c * DP + e] = sig[r];
        B.t_accept[(size_t)c * DP + e] = acc[r];
      }
    }
    if (g.lane == 0) { B.t_m[c] = m; B.t_flags[c] = fl; }
    M::relist(B, s, g, x);
  }

  // ---------------------------------------------------------------- pivoted Cholesky
  // cholfact(Hermitian(S), Val{true}) restated as LAPACK dpstf2('U', tol = 0) op order
  // (see oracle.c orc_pchol).  S: packed symmetric in LDS (`mat`, slot(i,k));
  // factored in place: L[i][step k] ends in slot(i, piv[k]), L[i][pos_i] in slot(i,i).
  // pk[] receives the pivot order.  Returns the rank (group-uniform).
  __device__ __forceinline__ static int pchol(int d, double* mat, int* pk, const Grp<G>& g) {
    double diag0[R], work[R], Lrow[R][DMAX];
    int posv[R];
    bool done[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      done[r] = !(e < d);
      diag0[r] = e < d ? mat[mmb_tri(e) + e] : 0.0;
      work[r] = 0.0;
      posv[r] = e;
    }
    int rank = d;
    bool live = true;
#pragma unroll
    for (int j = 0; j < DMAX; ++j) {
      if (live && j < d) {
        double key = -__builtin_inf(), val = __builtin_nan("");
        int pos = 0x7fffffff, idx = -1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (!done[r]) {
            double dd = diag0[r] - work[r];
            double kk = isnan(dd) ? (posv[r] == j ? __builtin_inf() : -__builtin_inf()) : dd;
            if (kk > key || (kk == key && posv[r] < pos)) {
              key = kk; pos = posv[r]; val = dd; idx = r * G + g.lane;
            }
          }
        }
        g.argmax(key, pos, val, idx);
        if (!(val > 0.0)) {
          rank = j;
          live = false;
        } else {
          const int p = idx, ppos = pos;
#pragma unroll
          for (int r = 0; r < R; ++r) {  // swap positions j and ppos
            int e = r * G + g.lane;
            if (!done[r] && posv[r] == j) posv[r] = ppos;
            if (e == p) { posv[r] = j; done[r] = true; }
          }
          pk[j] = p;
          const double ajj = sqrt(val);
          const double rinv = 1.0 / ajj;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            int e = r * G + g.lane;
            if (e == p) {
              Lrow[r][j] = ajj;
              mat[mmb_tri(p) + p] = ajj;
            } else if (!done[r]) {
              double t = 0.0;
#pragma unroll
              for (int k = 0; k < j; ++k) t = fma(Lrow[r][k], mat[mmb_slot(p, pk[k])], t);
              double lij = (mat[mmb_slot(e, p)] - t) * rinv;
              Lrow[r][j] = lij;
              mat[mmb_slot(e, p)] = lij;
              work[r] = work[r] + lij * lij;
            }
          }
          grp_sync();
        }
      }
    }
    return rank;
  }

  __device__ __forceinline__ static void slot_ik(int s, int& i, int& k) {
    int ii = (int)((sqrt(8.0 * (double)s + 1.0) - 1.0) * 0.5);
    while (mmb_tri(ii + 1) <= s) ++ii;
    while (mmb_tri(ii) > s) --ii;
    i = ii;
    k = s - mmb_tri(ii);
  }

  // ---------------------------------------------------------------- AMM
  // amm.jl:181-223.  LDS per chain: mat[TP] | z2[DP] | vv[DP] | mv[DP] | ia[2*DP ints]
  __device__ __forceinline__ static void amm(const SweepArgs& A, const DBlock& B, int c, const mmb_rng& rn,
                             const mmb_rng& ru, bool adapt, St& s, const Lc& l, const Grp<G>& g,
                             double* lds) {
    const int d = B.d;
    const int T = mmb_tri(d);
    double* mat = lds;
    double* z2s = lds + TP;
    double* vvs = z2s + DP;
    double* mvs = vvs + DP;
    int* ia = (int*)(mvs + DP);  // piv / pos scratch (2*DP ints)
    double v[R], x[R], z1[R], z2[R], mv[R];
    M::unlist(B, s, g.lane, v);
    int m = B.t_m[c];
    int fl = B.t_flags[c];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      mv[r] = e < d ? B.t_Mv[(size_t)c * DP + e] : 0.0;
    }
    const bool fresh = adapt && !(fl & 1);
    if (fresh) {  // setadapt!: m = 0, Mv = v (aliased), Mvv = v v', SigmaLm = 0
      m = 0;
      fl = (fl | 2) & ~4;
#pragma unroll
      for (int r = 0; r < R; ++r) mv[r] = v[r];
    }
    fl = adapt ? (fl | 1) : (fl & ~1);
    // proposal: x = SigmaL * z1 [; x = beta*x + (1-beta)*SigmaLm*z2]; x += v
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      if (e < d) mmb_normal_pair(&rn, (uint32_t)e, &z1[r], &z2[r]);
      else { z1[r] = 0.0; z2[r] = 0.0; }
    }
    if (!B.sigl_diag) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int e = r * G + g.lane;
        if (e < d) vvs[e] = z1[r];
      }
      grp_sync();
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      double a = 0.0;
      if (e < d) {
        if (B.sigl_diag) {
          a = fma(B.sigl[e * d + e], z1[r], a);
        } else {
          for (int k = 0; k <= e; ++k) a = fma(B.sigl[e * d + k], vvs[k], a);
        }
      }
      x[r] = a;
    }
    if (m > 2 * d) {
      double y[R];
#pragma unroll
      for (int r = 0; r < R; ++r) y[r] = 0.0;
      if (fl & 4) {
        grp_sync();
        const double* Ls = B.t_Ls + (size_t)c * TP;
        for (int t = g.lane; t < T; t += G) mat[t] = Ls[t];
        const uint8_t* pv = B.t_piv + (size_t)c * DP;
        for (int k = g.lane; k < d; k += G) {
          int pk_ = pv[k];
          ia[k] = pk_;
          ia[DP + pk_] = k;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          int e = r * G + g.lane;
          if (e < d) z2s[e] = z2[r];
        }
        grp_sync();
#pragma unroll
        for (int r = 0; r < R; ++r) {
          int e = r * G + g.lane;
          if (e < d) {
            int pe = ia[DP + e];
            double a = 0.0;
            for (int k = 0; k < pe; ++k) a = fma(mat[mmb_slot(e, ia[k])], z2s[k], a);
            a = fma(mat[mmb_tri(e) + e], z2s[pe], a);
            y[r] = a;
          }
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) x[r] = B.beta * x[r] + (1.0 - B.beta) * y[r];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = x[r] + v[r];
    double lx = M::logf(A, B, s, l, g, x);
    double lv = M::logf(A, B, s, l, g, v);
    if (mmb_uniform(&ru, 0u) < mmb_exp(lx - lv)) {
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = x[r];
    }
    if (adapt) {  // amm.jl:196-206
      m += 1;
      const double p = (double)m / ((double)m + 1.0);
      const double q = 1.0 - p;
      if (fl & 2) {
#pragma unroll
        for (int r = 0; r < R; ++r) mv[r] = p * v[r] + q * v[r];
        fl &= ~2;
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) mv[r] = p * mv[r] + q * v[r];
      }
      grp_sync();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int e = r * G + g.lane;
        if (e < d) { vvs[e] = v[r]; mvs[e] = mv[r]; }
      }
      grp_sync();
      const double cc = (B.scale * B.scale / (double)d) / p;
      double* Mvv = B.t_Mvv + (size_t)c * TP;
      // fresh: Mvv = v_old v_old' was formed before the proposal; v_old is still unlist()
      // of the state `s`, so recompute it from s here (same products).
      double vold[R];
      if (fresh) M::unlist(B, s, g.lane, vold);
      if (fresh) {
        grp_sync();
#pragma unroll
        for (int r = 0; r < R; ++r) {
          int e = r * G + g.lane;
          if (e < d) z2s[e] = vold[r];
        }
        grp_sync();
      }
      for (int t = g.lane; t < T; t += G) {
        int i, k;
        slot_ik(t, i, k);
        double old = fresh ? z2s[i] * z2s[k] : Mvv[t];
        double nv = p * old + (q * vvs[k]) * vvs[i];
        Mvv[t] = nv;
        mat[t] = cc * (nv - mvs[k] * mvs[i]);
      }
      grp_sync();
      int pkv[DMAX];
      int rank = pchol(d, mat, pkv, g);
      if (rank == d) {
        double* Ls = B.t_Ls + (size_t)c * TP;
        for (int t = g.lane; t < T; t += G) Ls[t] = mat[t];
        uint8_t* pv = B.t_piv + (size_t)c * DP;
#pragma unroll
        for (int k = 0; k < DMAX; ++k)
          if (k < d && g.lane == (k % G)) pv[k] = (uint8_t)pkv[k];
        fl |= 4;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      if (e < d) B.t_Mv[(size_t)c * DP + e] = mv[r];
    }
    if (g.lane == 0) { B.t_m[c] = m; B.t_flags[c] = fl; }
    grp_sync();
    M::relist(B, s, g, v);
  }

  // ---------------------------------------------------------------- Slice
  __device__ __forceinline__ static double width(const DBlock& B, int e) {
    return B.width ? B.width[e] : B.width0;
  }
  // slice.jl:271-297 (Univariate)
  __device__ __forceinline__ static void slice_uni(const SweepArgs& A, const DBlock& B, const mmb_rng& ru, St& s,
                                   const Lc& l, const Grp<G>& g) {
    const int d = B.d;
    double x[R], lo[R], up[R];
    M::unlist(B, s, g.lane, x);
    double logf0 = M::logf(A, B, s, l, g, x);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      if (e < d) {
        double w = width(B, e);
        lo[r] = x[r] - w * mmb_uniform(&ru, (uint32_t)e);
        up[r] = lo[r] + w;
      } else { lo[r] = 0.0; up[r] = 0.0; }
    }
    uint32_t k = (uint32_t)d;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      for (int ln = 0; ln < G; ++ln) {
        int e = r * G + ln;
        if (e >= d) break;
        bool own = g.lane == ln;
        double p0 = logf0 + mmb_log(mmb_uniform(&ru, k++));
        double xo = x[r];
        double u = mmb_uniform(&ru, k++);
        if (own) x[r] = lo[r] + (up[r] - lo[r]) * u;
        for (int guard = 0; guard < 100000; ++guard) {
          logf0 = M::logf(A, B, s, l, g, x);
          if (!(logf0 < p0)) break;
          if (own) {
            double value = x[r];
            if (value < xo) lo[r] = value;
            else up[r] = value;
          }
          u = mmb_uniform(&ru, k++);
          if (own) x[r] = lo[r] + (up[r] - lo[r]) * u;
        }
      }
    }
    M::relist(B, s, g, x);
  }
  // slice.jl:300-322 (Multivariate)
  __device__ __forceinline__ static void slice_multi(const SweepArgs& A, const DBlock& B, const mmb_rng& ru, St& s,
                                     const Lc& l, const Grp<G>& g) {
    const int d = B.d;
    double v[R], x[R], lo[R], up[R];
    M::unlist(B, s, g.lane, v);
    uint32_t k = 0;
    double p0 = M::logf(A, B, s, l, g, v) + mmb_log(mmb_uniform(&ru, k++));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      if (e < d) {
        double w = width(B, e);
        lo[r] = v[r] - w * mmb_uniform(&ru, 1u + (uint32_t)e);
        up[r] = lo[r] + w;
        x[r] = w * mmb_uniform(&ru, 1u + (uint32_t)d + (uint32_t)e) + lo[r];
      } else { lo[r] = up[r] = x[r] = 0.0; }
    }
    k = 1u + 2u * (uint32_t)d;
    for (int guard = 0; guard < 100000; ++guard) {
      if (!(M::logf(A, B, s, l, g, x) < p0)) break;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int e = r * G + g.lane;
        if (e < d) {
          double value = x[r];
          if (value < v[r]) lo[r] = value;
          else up[r] = value;
          x[r] = lo[r] + (up[r] - lo[r]) * mmb_uniform(&ru, k + (uint32_t)e);
        }
      }
      k += (uint32_t)d;
    }
    M::relist(B, s, g, x);
  }
};
