// samplers.h — block updates of src/samplers/{amwg,amm,slice}.jl for one chain
// advanced by a group of G lanes (element e of the block vector in lane e % G,
// register slot e / G).  RNG consumption follows mmb_math.h's documented layout and
// is mirrored draw for draw by oracle/oracle.c.
#pragma once
#include "models.h"
#include "hmc.h"
#include "nuts.h"

template <class M>
struct Smp {
  static constexpr int G = M::G, R = M::R, DMAX = M::DMAX, DP = M::DP, TP = M::TP;
  static constexpr int NT = (TP + G - 1) / G;  // packed-triangle slots per lane
  using St = typename M::St;
  using Lc = typename M::Lc;

  // ---------------------------------------------------------------- per-iteration draws
  // Variates that do not depend on the chain state, drawn for every block of an iteration
  // at once with one block per lane (32-lane groups): lane b holds block b's Gibbs variate
  // (Mdl::gibbs_draw_kind: Gamma(a) by Marsaglia-Tsang or a standard normal) or its AMM
  // accept uniform.  Same substreams, counters and operations as the per-block draws
  // (mmb_gamma_mt is replayed in full whenever its first attempt does not accept), so the
  // values are bit-identical to drawing them inside the blocks.
  __device__ __forceinline__ static double predraw(const SweepArgs& A, uint32_t chain, int64_t it,
                                                   const Grp<G>& g) {
    int kind = 0;  // 0 none, 1 Gamma(a), 2 normal, 3 uniform
    double a = 0.0;
    for (int b = 0; b < A.nb; ++b) {
      const DBlock& B = mmb_block(A.blocks, b);
      double ab = 0.0;
      int k = 0;
      if (B.kind == MMB_SAMPLER_GIBBS) k = M::gibbs_draw_kind(B, &ab);
      else if (B.kind == MMB_SAMPLER_AMM) k = 3;
      kind = g.lane == b ? k : kind;
      a = g.lane == b ? ab : a;
    }
    const uint32_t b = (uint32_t)g.lane;
    const mmb_rng rn = mmb_rng_make(A.seed, chain, (uint32_t)it, b, kind == 1 ? MMB_SUB_GAMMA_N : MMB_SUB_NORMAL);
    const mmb_rng ru = mmb_rng_make(A.seed, chain, (uint32_t)it, b, kind == 1 ? MMB_SUB_GAMMA_U : MMB_SUB_UNIFORM);
    const double x = mmb_normal(&rn, 0u);
    const double u = mmb_uniform(&ru, 0u);
    if (kind != 1) return kind == 2 ? x : u;
    // mmb_gamma_mt's first attempt (normal #0, uniform #0)
    const double d = a - 1.0 / 3.0;
    const double c = 1.0 / sqrt(9.0 * d);
    double v = 1.0 + c * x;
    bool ok = false;
    double r = 0.0;
    if (v > 0.0) {
      v = v * v * v;
      const double x2 = x * x;
      if (u < 1.0 - 0.0331 * (x2 * x2)) ok = true;
      else if (mmb_log(u) < 0.5 * x2 + d * (1.0 - v + mmb_log(v))) ok = true;
      r = d * v;
    }
    if (!ok) {
      uint32_t kn = 0, ku = 0;
      r = mmb_gamma_mt(a, &rn, &ru, &kn, &ku);
    }
    return r;
  }
  // value of lane b (group-relative, wave-uniform b) of each 32-lane group
  __device__ __forceinline__ static double lane_value(double v, int b) {
    const uint64_t u = mmb_d2u(v);
    const int lo = (int)(uint32_t)u, hi = (int)(uint32_t)(u >> 32);
    const uint32_t lo0 = (uint32_t)__builtin_amdgcn_readlane(lo, b), hi0 = (uint32_t)__builtin_amdgcn_readlane(hi, b);
    const uint32_t lo1 = (uint32_t)__builtin_amdgcn_readlane(lo, b + 32), hi1 = (uint32_t)__builtin_amdgcn_readlane(hi, b + 32);
    const bool up = (threadIdx.x & 32) != 0;
    return mmb_u2d((uint64_t)(up ? lo1 : lo0) | ((uint64_t)(up ? hi1 : hi0) << 32));
  }

  // ---------------------------------------------------------------- AMWG
  // amwg_sub! decided for every coordinate at once (blocks whose logpdf is a butterfly over
  // per-lane terms that only the lane's own element changes: M::AMWG_SEP).  Coordinate j's
  // step compares its uniform with exp(delta_j), delta_j = logf(state with x_j') - logf0, two
  // rounded evaluations whose states differ only in lane j's terms; in exact arithmetic the
  // difference is d_j = (tp_j' - tp_j) - 0.5 invv (ts_j' - ts_j) whatever the other
  // coordinates' accept history.  Each rounded logf is within 9 u (sum_i |tp_i| + |yk| +
  // invv sum_i |ts_i|) of its exact value (a depth-5 tree sum, then three roundings), so
  // |delta_j - d_j| <= eps_j with the factor of 128 u taken below; a decision is CERTAIN
  // when the uniform is outside [exp(d_j - eps_j), exp(d_j + eps_j)] widened by the
  // (sub-ulp) error of mmb_exp.  All certain: x_j' where accepted -- the same values and
  // accept counts as the sequential loop, bit for bit, since certain decisions are its
  // decisions.  Any uncertain lane, a non-finite term or bound: false, and the caller runs
  // the sequential loop (RNG draws are the same precomputed z / uown either way).
  // The model gives, per lane j, d_j and the magnitude epsm_j its rounding band scales with
  // (M::amwg_dm: rats models.h, the node IR's separable blocks ir.h), and the band's relative
  // factor (M::amwg_epsf).
  __device__ __forceinline__ static bool amwg_lanes(const DBlock& B, const typename M::Prep& pc, const St& s,
                                                    const Lc& l, const Grp<G>& g, double* x, const double* z,
                                                    const double* uown, double* acc, double ad,
                                                    const SweepArgs& A) {
    const bool in = g.lane < B.d;
    const double x1 = x[0] + z[0];  // the sequential loop's x[r] += z[r]
    double del, epsm;
    bool bad;
    M::amwg_dm(A, B, pc, s, l, g, x[0], x1, del, epsm, bad);
    // (amwg_exact = 2, tests: a 2^30 times wider band, so that many updates fall back)
    const double eps = (A.amwg_exact == 2 ? 0x1p30 * M::amwg_epsf(B) : M::amwg_epsf(B)) * epsm;
    const double lo = del - eps, hi = del + eps;
    const double ue = uown[0];  // in [0, 1)
    const bool acc_c = lo >= 700.0 || (lo > -700.0 && ue < mmb_exp(lo) * (1.0 - 0x1p-48));
    const bool rej_c = (hi <= -700.0 && ue >= 1e-300) ||
                       (hi > -700.0 && hi < 700.0 && ue >= mmb_exp(hi) * (1.0 + 0x1p-48));
    bad = bad || !isfinite(eps);
    const bool unsure = in && (bad || !(acc_c || rej_c));
    const uint64_t bal = __ballot(unsure);
    const bool any = (threadIdx.x & 32) ? (bal >> 32) != 0 : (uint32_t)bal != 0;
    if (any) return false;
    if (in && acc_c) {
      x[0] = x1;
      acc[0] += ad;
    }
    return true;
  }

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
    const typename M::Prep pc = M::prep(B, s);
    // the proposal normals and (lane groups) the accept uniforms of every element at once,
    // element e on its own lane: the same Philox draws (index e) the sequential loop below
    // consumes, so the values are bit-identical; each step then takes its uniform from lane e
    // (readlane) instead of every lane recomputing it (-~60 VALU per coordinate)
    double uown[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      z[r] = e < d ? sig[r] * mmb_normal(&rn, 2u * (uint32_t)e) : 0.0;
      uown[r] = (G > 1 && e < d) ? mmb_uniform(&ru, (uint32_t)e) : 0.0;
    }
    bool seq = true;
    if constexpr (M::AMWG_SEP && G == 32 && R == 1) {
      if (M::AMWG_PROBE && A.amwg_probe != 0 && M::amwg_sep(B)) {
        // test-only (MMB_AMWG_PROBE=1, rats): uniforms a few ulps to 2^-12 off each coordinate's
        // accept threshold exp(d_j) (mmb_math.h mmb_amwg_probe_factor; the oracle draws the same),
        // so both the lane-parallel decision and its sequential fallback meet near-ties
        double del, em;
        bool bd;
        M::amwg_dm(A, B, pc, s, l, g, x[0], x[0] + z[0], del, em, bd);
        uown[0] = g.lane < d ? mmb_amwg_probe_uniform(del, &ru, (uint32_t)g.lane) : 0.0;
      }
      if (A.amwg_exact != 1 && M::amwg_sep(B)) {
        seq = !amwg_lanes(B, pc, s, l, g, x, z, uown, acc, ad, A);
        if (seq && g.lane == 0) atomicAdd(&A.nuts_stat[5], 1ull);
      }
    }
    if (seq) {  // amwg_sub!: one coordinate at a time, the block's logpdf at every proposal
      double logf0 = M::logf_p(A, B, pc, s, l, g, x);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        for (int ln = 0; ln < G; ++ln) {
          int e = r * G + ln;
          if (e >= d) break;
          bool own = g.lane == ln;
          double xo = x[r];
          if (own) x[r] += z[r];
          double lpp = M::logf_p(A, B, pc, s, l, g, x);
          const double ue = G == 32 ? lane_value(uown[r], ln) : mmb_uniform(&ru, (uint32_t)e);
          if (ue < mmb_exp(lpp - logf0)) {
            logf0 = lpp;
            if (own) acc[r] += ad;
          } else if (own) {
            x[r] = xo;
          }
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
  // cholfact(Hermitian(S), Val{true}) restated in LAPACK dpstf2('U', tol = 0) op order
  // (oracle.c orc_pchol): pivot = first maximum of the remaining diagonal in position
  // order, stop when it is <= 0 or NaN, row J as a dot product then scaled by ONE/AJJ.
  // The dot product runs on two accumulators (even / odd k) summed at the end (the
  // oracle does the same).  S: packed symmetric in LDS (`mat`, slot(i,k)); the pivot's
  // factor row is broadcast through `prow` (contiguous LDS) each step.  On full rank the
  // factor is written back in place: L[i][step k] -> slot(i, piv[k]), L[i][pos_i] ->
  // slot(i,i).  pk[] receives the pivot order.  Returns the rank (group-uniform).
  __device__ __forceinline__ static int pchol(int d, double* mat, double* prow, int* pks,
                                              const Grp<G>& g) {
    double diag0[R], work[R], Lrow[R][DMAX];
    bool done[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      done[r] = !(e < d);
      diag0[r] = e < d ? mat[mmb_tri(e) + e] : 0.0;
      work[r] = 0.0;
#pragma unroll
      for (int k = 0; k < DMAX; ++k) Lrow[r][k] = 0.0;
    }
    int rank = d;
    bool live = true;
#pragma unroll
    for (int j = 0; j < DMAX; ++j) {
      if (live && j < d) {
        // ---- pivot: first maximum of the remaining diagonal in position order ----
        double dl[R], cand[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          dl[r] = diag0[r] - work[r];
          cand[r] = done[r] ? -__builtin_inf() : dl[r];
        }
        int p;
        double val;
#ifdef MMB_EXP_NOPIVOT
        if (G == 32) {  // timing experiment only: no pivot search
          p = j;
          val = __shfl(dl[0], (int)(threadIdx.x & 32) + j, 64);
        } else
#endif
        if (G == 32) {
          // fast path: max-reduce, then the (usually unique) lane holding it
          double mx = cand[0];
          bool anynan = isnan(mx);
          mx = anynan ? -__builtin_inf() : mx;
          mx = fmax(mx, Grp<G>::template other_d<0>(mx));
          mx = fmax(mx, Grp<G>::template other_d<1>(mx));
          mx = fmax(mx, Grp<G>::template other_d<2>(mx));
          mx = fmax(mx, Grp<G>::template other_d<3>(mx));
          mx = fmax(mx, Grp<G>::template other_d<4>(mx));
          const unsigned long long bw = __ballot(!done[0] && cand[0] == mx);
          const unsigned long long bn = __ballot(!done[0] && anynan);
          const unsigned sh = threadIdx.x & 32;
          const unsigned win = (unsigned)(bw >> sh), nan_ = (unsigned)(bn >> sh);
          if (__builtin_popcount(win) == 1 && nan_ == 0) {
            p = __builtin_ctz(win);
            val = mx;
          } else {
            // rare: exact tie or NaN -> replay dpstf2's position swaps (pks history)
            int* perm = (int*)prow;  // group-private LDS scratch
            if (g.lane == 0) {
              for (int t = 0; t < d; ++t) perm[t] = t;
              for (int k = 0; k < j; ++k) {
                int q = pks[k], qpos = k;
                for (int t = k; t < d; ++t) if (perm[t] == q) qpos = t;
                int tmp = perm[k]; perm[k] = q; perm[qpos] = tmp;
              }
            }
            grp_sync();
            int mypos = 0x7fffffff;
            for (int t = j; t < d; ++t) if (perm[t] == g.lane) mypos = t;
            grp_sync();
            double key = done[0] ? -__builtin_inf()
                                 : (isnan(dl[0]) ? (mypos == j ? __builtin_inf() : -__builtin_inf()) : dl[0]);
            int pi = (done[0] ? 0x7fff : mypos) << 16 | g.lane;
            g.argmax(key, pi);
            p = pi & 0xffff;
            val = g.bcast(dl[0], p);
          }
        } else {
          // sequential lanes (G == 1): replay positions per chain
          int perm[DMAX];
#pragma unroll
          for (int t = 0; t < DMAX; ++t) perm[t] = t;
#pragma unroll
          for (int k = 0; k < DMAX; ++k) {
            if (k < j) {
              int q = pks[k];
              int qpos = k;
#pragma unroll
              for (int t = 0; t < DMAX; ++t) qpos = (t >= k && perm[t] == q) ? t : qpos;
              int tmp = perm[k];
#pragma unroll
              for (int t = 0; t < DMAX; ++t) perm[t] = (t == qpos) ? tmp : perm[t];
              perm[k] = q;
            }
          }
          // fold in position order: first strict maximum (oracle.c orc_pchol)
          int best = -1;
          double bv = 0.0;
#pragma unroll
          for (int t = 0; t < DMAX; ++t) {
            if (t >= j && t < d) {
              int e = perm[t];
              double de = dl[0];
#pragma unroll
              for (int r = 1; r < R; ++r) de = (e == r) ? dl[r] : de;
              if (best < 0) { best = e; bv = de; }
              else if (de > bv) { best = e; bv = de; }
            }
          }
          p = best;
          val = bv;
        }
        if (!(val > 0.0)) {
          rank = j;
          live = false;
        } else {
          if (g.lane == 0) pks[j] = p;
          const double ajj = sqrt(val);
          const double rinv = 1.0 / ajj;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if (r * G + g.lane == p) {
              done[r] = true;
              Lrow[r][j] = ajj;
#pragma unroll
              for (int k = 0; k + 1 < j; k += 2)
                *(double2*)(prow + k) = make_double2(Lrow[r][k], Lrow[r][k + 1]);
              if (j & 1) prow[j - 1] = Lrow[r][j - 1];
            }
          }
          grp_sync();
#pragma unroll
          for (int r = 0; r < R; ++r) {
            int e = r * G + g.lane;
            if (!done[r]) {
              double t0 = 0.0, t1 = 0.0;
#ifndef MMB_EXP_NODOT
#pragma unroll
              for (int k = 0; k + 1 < j; k += 2) {
                const double2 pp = *(const double2*)(prow + k);
                t0 = fma(Lrow[r][k], pp.x, t0);
                t1 = fma(Lrow[r][k + 1], pp.y, t1);
              }
              if (j & 1) t0 = fma(Lrow[r][j - 1], prow[j - 1], t0);
#endif
              double lij = (mat[mmb_slot(e, p)] - (t0 + t1)) * rinv;
              Lrow[r][j] = lij;
              work[r] = work[r] + lij * lij;
            }
          }
          grp_sync();
        }
      }
    }
    if (rank == d) {  // write the factor back in slot form
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int e = r * G + g.lane;
        if (e < d) {
          bool before = true;
#pragma unroll
          for (int k = 0; k < DMAX; ++k) {
            if (k < d) {
              const int q = pks[k];
              if (q == e) {
                mat[mmb_tri(e) + e] = Lrow[r][k];
                before = false;
              } else if (before) {
                mat[mmb_slot(e, q)] = Lrow[r][k];
              }
            }
          }
        }
      }
    }
    return rank;
  }

  // Exact pivot choice for the rare cases the fast search hands over (ties of the high
  // words, NaN candidates): replays dpstf2's position swaps from the pivot history and
  // takes the first maximum in position order.  Out of line: it is shared by every
  // unrolled step instead of being inlined 30 times.
  __device__ __forceinline__ static int pivot_exact(double dl, bool done, const int* pks, int j,
                                                              int d, int* perm, double* val) {
    const int lane = (int)(threadIdx.x & (G - 1));
    if (lane == 0) {
      for (int t = 0; t < d; ++t) perm[t] = t;
      for (int k = 0; k < j; ++k) {
        int q = pks[k], qpos = k;
        for (int t = k; t < d; ++t) if (perm[t] == q) qpos = t;
        int tmp = perm[k]; perm[k] = q; perm[qpos] = tmp;
      }
    }
    grp_sync();
    int mypos = 0x7fffffff;
    for (int t = j; t < d; ++t) if (perm[t] == lane) mypos = t;
    grp_sync();
    double key = done ? -__builtin_inf()
                      : (isnan(dl) ? (mypos == j ? __builtin_inf() : -__builtin_inf()) : dl);
    int pi = (done ? 0x7fff : mypos) << 16 | lane;
    Grp<G> g;
    g.argmax(key, pi);
    const int p = pi & 0xffff;
    *val = g.bcast(dl, p);
    return p;
  }

  // group max of an int over the 32 lanes: four row stages (DPP folded into v_max_i32)
  // and one permlane16 swap whose two outputs are the two rows of each half
  __device__ __forceinline__ static int gmax_i32(int x) {
    x = max(x, dpp_i<MMB_DPP_XOR1>(x));
    x = max(x, dpp_i<MMB_DPP_XOR2>(x));
    x = max(x, dpp_i<MMB_DPP_HMIRROR>(x));
    x = max(x, dpp_i<MMB_DPP_MIRROR>(x));
    auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    return max((int)r[0], (int)r[1]);
  }

  // The checked factorization as a compact loop (not unrolled; the row lives in a private
  // array): the rare redo after an optimistic pass of pchol32 that met a tie, a NaN or a
  // maximum outside the in-range square root's domain.  dpstf2's pivot (pivot_exact: first
  // maximum in position order, NaN semantics) and its ajj <= 0 stop, IEEE sqrt() and 1.0 / x,
  // and the same two-accumulator dot product (even / odd k) as the unrolled steps, so the
  // factor is bit-identical to what the checked unrolled pass computes.  Leaves the rows in
  // Lrow[], the positions in pe, done / work as the unrolled pass does.
#ifdef MMB_REDO_INLINE
  __device__ __forceinline__
#else
  __device__ __attribute__((noinline))
#endif
  static void redo_exact_impl(int d, double* mat, double* prow, int* pks,
                                                                    double diag0, int lc, bool inb, double* Lx,
                                                                    double* work_, bool* done_, int* pe_) {
    const int lane = (int)(threadIdx.x & (G - 1));
    double work = inb ? 0.0 : __builtin_inf();
    bool done = !inb, live = true;
    int pe = 0;
    for (int k = 0; k < DMAX; ++k) Lx[k] = 0.0;
#pragma nounroll
    for (int j = 0; j < d; ++j) {
      if (live) {
        const double dl = diag0 - work;
        double val;
        const int p = pivot_exact(dl, done, pks, j, d, (int*)prow, &val);
        if (!(val > 0.0)) {
          live = false;
        } else {
          if (lane == p) {
            pks[j] = p;
            for (int k = 0; k < j; ++k) prow[k] = Lx[k];
            const double ajj = sqrt(dl);
            prow[DMAX] = 1.0 / ajj;
            Lx[j] = ajj;
            pe = j;
            work = __builtin_inf();
            done = true;
          }
          grp_sync();
          if (j + 1 < d) {
            double t0 = 0.0, t1 = 0.0;
            for (int k = 0; k < j; ++k) {
              if (k & 1) t1 = fma(prow[k], Lx[k], t1);
              else t0 = fma(prow[k], Lx[k], t0);
            }
            const double lij = (mat[mmb_slot(lc, p)] - (t0 + t1)) * prow[DMAX];
            work = work + lij * lij;
            if (!done) Lx[j] = lij;
          }
          grp_sync();
        }
      }
    }
    *work_ = work;
    *done_ = done;
    *pe_ = pe;
  }
  __device__ __forceinline__ static void redo_exact(int d, double* mat, double* prow, int* pks, double diag0,
                                                    int lc, bool inb, double (&Lrow)[DMAX], double& work,
                                                    bool& done, int& pe) {
    double Lx[DMAX];
    redo_exact_impl(d, mat, prow, pks, diag0, lc, inb, Lx, &work, &done, &pe);
#pragma unroll
    for (int k = 0; k < DMAX; ++k) Lrow[k] = Lx[k];
  }

  // pchol for 32-lane groups with one row per lane (rats), same results as pchol():
  // * the pivot lane computes sqrt / reciprocal of its remaining diagonal by the in-range
  //   sequences of device.h (bit-identical to sqrt() and 1.0 / x there) and publishes the
  //   reciprocal through LDS together with its factor row;
  // * the search reduces the high words of the positive candidates as int32 (one DPP
  //   max per stage); a unique maximal high word is the unique maximum.  High-word ties
  //   and NaN candidates go to pivot_exact (dpstf2's first maximum in position order).
  // Measured (rats sweep, 16384 chains): 0.255 -> 0.248 ms; the factorization is bound by
  // its f64 work per step (sqrt, reciprocal, dot product), not by the pivot search.
  // rn1 != null: also returns in *ynext this lane's row of SigmaLm z2' for the next
  // iteration (z2' = the second normal of each element's pair from rn1), formed from the
  // factor rows still in registers: P L z2' (amm.jl:74), row e = sum_k L[pos e][k] z2'[k],
  // k ascending -- the order of the direct matvec in amm().
  //
  // On full rank the factor is left in `mat` in POSITION form (row at pivot position t, i.e.
  // row piv[t] of P'L... stored at tri(t) .. tri(t) + t, step order), and *pos receives this
  // lane's position; amm() stores it with the position bytes (the host converts to the
  // canonical slot form + pivot order, engine.cpp).
  __device__ __forceinline__ static int pchol32(int d, double* mat, double* prow, int* pks, const Grp<G>& g,
                                                int* pos_out, const DBlock* NB = nullptr,
                                                const SweepArgs& A = SweepArgs{}, int c = 0, uint32_t chain = 0,
                                                int64_t it = 0, int b = 0, int m = 0, int* redo = nullptr) {
#ifndef MMB_PCHOL_NOFULLD
    // a block as wide as the model's DMAX (rats: both 30-d blocks) runs a copy with d a
    // compile-time constant: no per-step scalar test and branch of j against d (9.58e7 ->
    // 9.90e7 rats chain-updates/s, A/B on one box, parity unchanged)
    if (d == DMAX)
      return pchol32_impl<true, true>(d, mat, prow, pks, pos_out, NB, A.seed, A.xepoch, c, chain, it, b, m, redo);
#endif
    return pchol32_impl<true>(d, mat, prow, pks, pos_out, NB, A.seed, A.xepoch, c, chain, it, b, m, redo);
  }
#if !defined(MMB_PCHOL_V1) && defined(MMB_PCHOL_EXACT_NOINLINE)
  // timing experiment: the checked pass (rare) out of line (measured 13 % slower: call ABI)
  __device__ __noinline__ static int pchol32_exact(int d, double* mat, double* prow, int* pks, int* pos_out,
                                                   const DBlock* NB, uint64_t seed, int64_t xepoch, int c,
                                                   uint32_t chain, int64_t it, int b, int m) {
    return pchol32_impl<false>(d, mat, prow, pks, pos_out, NB, seed, xepoch, c, chain, it, b, m, nullptr);
  }
#endif
  template <bool OPT, bool FULLD = false>
  __device__ __forceinline__ static int pchol32_impl(int d_arg, double* mat, double* prow, int* pks, int* pos_out,
                                                     const DBlock* NB, uint64_t seed, int64_t xepoch, int c,
                                                     uint32_t chain, int64_t it, int b, int m,
                                                     int* redo_out) {
    const int d = FULLD ? DMAX : d_arg;
    const Grp<G> g;
    constexpr int RI = DMAX;  // prow[RI]: the pivot's reciprocal
    const int lane = g.lane;
    const bool hi_half = (threadIdx.x & 32) != 0;
    const bool inb = lane < d;
    const int lc = inb ? lane : 0;
    const double diag0 = inb ? mat[mmb_tri(lane) + lane] : 0.0;
    double work = 0.0;
    double Lrow[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) Lrow[k] = 0.0;
    MMB_PROF_START
    bool done = !inb;
    int rank = d;
    int pe = 0;  // this lane's pivot position
    bool live = true;
    // the factorization's epilogue (carried proposal, write-back)
    auto tail = [&]() __attribute__((always_inline)) -> int {
      MMB_PROF_MARK(10, lane)
      // carried proposal of the next iteration (see amm): formed here, where the factor rows are
      // still in registers; skipped when the next proposal would need an older factor
      if (NB != nullptr && (rank == d || m <= 2 * d)) {
        const mmb_rng rn1 = mmb_rng_make(seed, chain, (uint32_t)(it + 1), (uint32_t)b, MMB_SUB_NORMAL);
        double z1n = 0.0, z2n = 0.0;
        if (inb) mmb_normal_pair(&rn1, (uint32_t)lane, &z1n, &z2n);
        double a = 0.0;
        if (inb) a = fma(NB->sigl[lane * d + lane], z1n, a);
        if (m > 2 * d) {
          // rows are zero past the lane's own step, so the full sweep adds exact zeros
          double y = 0.0;
#ifdef MMB_EXP_LDS_CARRY
          prow[lane] = z2n;
          grp_sync();
#pragma unroll
          for (int k = 0; k < DMAX; k += 2) {
            const double2 zz = *(const double2*)(prow + k);
            y = fma(Lrow[k], zz.x, y);
            if (k + 1 < DMAX) y = fma(Lrow[k + 1], zz.y, y);
          }
          grp_sync();
#else
          // z2'[k] lives in lane k: rows 0 / 1 of the group exchange theirs (permlane16 swap),
          // then each product takes z2'[k] from lane k % 16 of the row (DPP64 row_newbcast)
          const double zs = swap16_d(z2n);
          const bool row0 = (lane & 16) == 0;
          const double zA = row0 ? z2n : zs, zB = row0 ? zs : z2n;
#pragma unroll
          for (int k = 0; k < DMAX; ++k) fmac_rowbc_n(y, k < 16 ? zA : zB, Lrow[k], k & 15);
#endif
          a = NB->beta * a + (1.0 - NB->beta) * y;
        }
        if (inb) NB->t_xnext[(size_t)c * DP + lane] = a;
        if (lane == 0) NB->t_xtag[c] = (xepoch << 32) | (int64_t)(uint32_t)(it + 1);  // xtag()
      }
      MMB_PROF_MARK(11, lane)
      if (rank == d && inb) {  // the factor in position form: row at position pe at tri(pe) + k
        // one store per k from every lane, no exec-mask change: entries past the row's end
        // (k > pe, exact zeros) go to the lane's own dummy slot in the idle pivot-row buffer
        const int base = mmb_tri(pe);
#pragma unroll
        for (int k = 0; k < DMAX; ++k) {
          double* dst = k <= pe ? mat + base + k : prow + lane;
          *dst = Lrow[k];
        }
      }
      MMB_PROF_MARK(12, lane)
      *pos_out = pe;
      return rank;
    };
#ifndef MMB_PCHOL_V1
    // Two passes over the same Sigma (mat is only read until the write-back):
    // * the optimistic pass takes, per chain, the lane whose candidate dl = diag0 - work has
    //   the largest int32 high word (the lowest such lane on a tie) as the pivot and stops
    //   when every candidate is negative.  It never branches on the pivot search; it only
    //   accumulates, on the scalar unit, whether a step was outside what that rule decides
    //   exactly: a high-word tie, a NaN or >= 2^700 candidate, or a maximum below 2^-700
    //   (then the in-range square root / reciprocal of device.h would not be the IEEE ones);
    // * only if so (rare), the whole factorization is redone by the checked pass: the same
    //   steps, with dpstf2's exact choice (pivot_exact: first maximum in position order, its
    //   rank test) and sqrt() / division wherever a step needs them.
    // Both give dpstf2's pivots and bits.  A lane that is done (its row finished) or out of
    // range carries work = +inf, so its candidate is -inf and its key negative with no
    // per-step select.  The row update of lij is the !done select only; the dot product runs
    // on every lane (a DPP source lane must be active).
    if (!inb) work = __builtin_inf();
    // LDS byte address of mat (32-bit local address space)
    const uint32_t mat_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)mat;
    int hmask = hi_half ? -1 : 0;
    asm volatile("" : "+v"(hmask));  // keep it a VGPR (not a scalar lane mask + select)
    constexpr int KEY_LO = 0x14300000;     // high word of 2^-700
    constexpr double BIG = 0x1p700;
    // CHECKED: template constant (two inlined copies of the pass) or, with MMB_PCHOL_ONECOPY,
    // a wave-uniform run-time flag that one copy of the pass branches on per step
    auto pass = [&](auto checked_c) __attribute__((always_inline)) -> bool {
#ifdef MMB_PCHOL_ONECOPY
      const bool CHECKED = checked_c;
#else
      constexpr bool CHECKED = decltype(checked_c)::value;
#endif
      // POSTHOC (default): the optimistic pass keeps no per-step bookkeeping of whether its
      // choices were dpstf2's; everything that could make them differ is visible after the loop
      // (see the check below the step loop).  MMB_PCHOL_STEPCHECK: the round-3 per-step check.
#ifdef MMB_PCHOL_STEPCHECK
      constexpr bool POSTHOC = false;
#else
      constexpr bool POSTHOC = !CHECKED;
#endif
      // DW: the optimistic pass keeps no done flag: a lane is done iff its work is +inf (pivots set
      // it; an undone lane whose sum of squares overflowed counts as done too, which only a chain
      // that cannot reach full rank can meet -- its rank then disagrees with its steps and the
      // post-hoc check redoes it)
#ifdef MMB_PCHOL_DONEFLAG
      constexpr bool DW = false;
#else
      constexpr bool DW = POSTHOC;
#endif
      uint64_t needm = 0;  // wave-uniform: nonzero if a step of this pass was not decided exactly
      bool needl = false;  // per-lane form of needm (a lane mask: the OR stays on the scalar unit)
      double apiv = 1.0;   // POSTHOC: this lane's candidate when it was taken as the pivot
      double inf_s = __builtin_inf();
      asm volatile("" : "+s"(inf_s));  // +inf in an SGPR pair: one v_mov_b64 per pivot
#pragma unroll
      for (int j = 0; j < DMAX; ++j) {
        if (live && j < d) {
          const double dl = diag0 - work;
#ifdef MMB_EXP_HOIST
          // every lane's square root and reciprocal, independent of the search: the two
          // dependency chains interleave (the pivot lane then publishes at once)
          double ajj_h = 0.0, rinv_h = 0.0;
          if (!CHECKED) {
            mmb_sqrt_rcp_inrange(dl, &ajj_h, &rinv_h);
            asm volatile("" : "+v"(ajj_h), "+v"(rinv_h));
          }
#endif
          const int key = (int)(mmb_d2u(dl) >> 32);
          const int mx = gmax_i32(key);
          const uint64_t eq = __ballot(key == mx);
          uint32_t elo = (uint32_t)eq, ehi = (uint32_t)(eq >> 32);
          int p = 0;
          // one compare for the stop and the bookkeeping's ballot (pos = the complement mask)
          const uint64_t negm = __ballot(mx < 0);
          bool pos = mmb_inverse_ballot(~negm);  // dpstf2's ajj <= 0 stop
          bool fast = true;
#ifdef MMB_PCHOL_ONECOPY
          {
            const int plo = __builtin_ctz(elo | 0x80000000u), phi = __builtin_ctz(ehi | 0x80000000u);
            p = plo ^ ((plo ^ phi) & hmask);
          }
          if (CHECKED) {
#else
          if constexpr (!CHECKED) {
            // p = plo in the lower chain, phi in the upper one, as plo ^ ((plo ^ phi) & hmask)
            const int plo = __builtin_ctz(elo | 0x80000000u), phi = __builtin_ctz(ehi | 0x80000000u);
            p = plo ^ ((plo ^ phi) & hmask);
          } else {
#endif
            const uint64_t act = __builtin_amdgcn_read_exec();
            const uint64_t bad = __ballot(!(dl < BIG));      // NaN, +inf or >= 2^700
            const uint64_t big = __ballot(key >= KEY_LO);    // candidates >= 2^-700
            const uint64_t neg = __ballot(mx < 0);
            // per chain (32-bit half): inactive, or stopping, or a unique maximum >= 2^-700
            uint32_t alo = (uint32_t)act, ahi = (uint32_t)(act >> 32);
            uint32_t nlo = (uint32_t)neg, nhi = (uint32_t)(neg >> 32), blo = (uint32_t)big, bhi = (uint32_t)(big >> 32);
            asm("" : "+s"(elo), "+s"(ehi), "+s"(alo), "+s"(ahi));
            asm("" : "+s"(nlo), "+s"(nhi), "+s"(blo), "+s"(bhi));
            const bool ok_lo = alo == 0 || nlo != 0 || ((elo & (elo - 1)) == 0 && blo != 0);
            const bool ok_hi = ahi == 0 || nhi != 0 || ((ehi & (ehi - 1)) == 0 && bhi != 0);
            fast = bad == 0 && ok_lo && ok_hi;
            if (fast) {
              const int plo = __builtin_ctz(elo | 0x80000000u), phi = __builtin_ctz(ehi | 0x80000000u);
              p = plo ^ ((plo ^ phi) & hmask);
            } else {
              double val;
              p = pivot_exact(dl, done, pks, j, d, (int*)prow, &val);
              pos = val > 0.0;
            }
          }
#ifdef MMB_PCHOL_STOPBR
          constexpr bool NOBR = false;
#else
          // optimistic pass: no branch on the stop either -- a chain whose candidates are all
          // negative runs this step on a garbage pivot (one of its done / out-of-range lanes,
          // whose -inf keys are the largest negative ones) and stops after it; a stopped
          // chain's factor is never used (rank < d) and its done set is unchanged
          constexpr bool NOBR = !CHECKED;
#endif
          if (!NOBR && !pos) {
            live = false;  // rank = pivots taken, counted after the loop
          } else {
            // optimistic pass: the pivot is the lane holding the maximal high word (unique, or
            // the pass is redone; a stopping chain's garbage step may take several of its done /
            // out-of-range -inf lanes, which changes nothing that is used)
            // POSTHOC: no pivot on a stopping chain's step (its done lanes keep pe and row)
            const bool piv = CHECKED ? lane == p
                                     : POSTHOC ? mmb_inverse_ballot(eq & ~negm) : key == mx;
            if (piv) {
              if constexpr (POSTHOC) apiv = dl;  // (pks: only the checked pass replays it)
              else pks[j] = p;
              if (j + 1 < d) {  // the last step has no rows left to update: no readers
#pragma unroll
                for (int k = 0; k + 1 < j; k += 2) *(double2*)(prow + k) = make_double2(Lrow[k], Lrow[k + 1]);
                if (j & 1) prow[j - 1] = Lrow[j - 1];
              }
              double ajj, rinv;
              if (fast) {
#ifdef MMB_EXP_HOIST
                if (!CHECKED) {
                  ajj = ajj_h;
                  rinv = rinv_h;
                } else
#endif
                mmb_sqrt_rcp_inrange(dl, &ajj, &rinv);  // IEEE results in the fast range (device.h)
              } else {
                ajj = sqrt(dl);
                rinv = 1.0 / ajj;
              }
              prow[RI] = rinv;
              Lrow[j] = ajj;
              pe = j;
              work = inf_s;
              if constexpr (!DW) done = true;
            }
            grp_sync();
            if (j + 1 < d) {  // (j = d - 1: every lane is done)
              // pivot row: lane l of each 16-lane row reads elements l and 16 + l, then every
              // product takes element k from lane k % 16 of its row by a DPP64 row_newbcast operand
              double t0 = 0.0, t1 = 0.0;
              // Sigma(lc, p) at byte 8 slot = 4 a (a + 1) + 8 b, a = max, b = min
              const int sa = max(lc, p), sb = min(lc, p);
              int sq, ad;  // sa (sa + 1) in one instruction; byte address by two shift-adds
              asm("v_mad_u32_u24 %0, %1, %1, %1" : "=v"(sq) : "v"(sa));
              asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(ad) : "v"(sb), "v"(mat_lds));
              asm("v_lshl_add_u32 %0, %1, 2, %0" : "+v"(ad) : "v"(sq));
              double sig = *(const __attribute__((address_space(3))) double*)(uintptr_t)(uint32_t)ad;
              double rinv = prow[RI];
              double pA = prow[lane & 15];
              double pB = j > 16 ? prow[16 + (lane & 15)] : 0.0;
              asm volatile("" : "+v"(sig), "+v"(rinv), "+v"(pA));
              if (j > 16) asm volatile("" : "+v"(pB));
#ifdef MMB_EXP_MUL01
              // the first two products by plain multiplies of a broadcast read of the row's first
              // pair (fma(a, b, 0) and a * b are the same value): no accumulator zeroing per step
              if (j > 0) {
                const double2 p01 = *(const double2*)prow;
                t0 = p01.x * Lrow[0];
                if (j > 1) t1 = p01.y * Lrow[1];
#pragma unroll
                for (int k = 2; k < j; ++k) {
                  const double src = k < 16 ? pA : pB;
                  if (k & 1) fmac_rowbc_nf(t1, src, Lrow[k], k & 15, k == 2 || k == 16);
                  else fmac_rowbc_nf(t0, src, Lrow[k], k & 15, k == 2 || k == 16);
                }
#else
              if (j > 0) {
#pragma unroll
                for (int k = 0; k < j; ++k) {
                  const double src = k < 16 ? pA : pB;
                  if (k & 1) fmac_rowbc_ld(t1, src, Lrow[k], k & 15);
                  else fmac_rowbc_ld(t0, src, Lrow[k], k & 15);
                }
#endif
              }
              const double lij = (sig - (t0 + t1)) * rinv;
              const bool keep = DW ? work == inf_s : done;  // done lanes keep their rows
              // done lanes carry work = +inf, which absorbs lij^2: no select for work
              work = work + lij * lij;
              if (!keep) Lrow[j] = lij;
            }
            grp_sync();
            if (NOBR) live = live && pos;
          }
#ifndef MMB_PCHOL_ONECOPY
          if constexpr (!CHECKED && !POSTHOC)
#endif
          {
            // scalar bookkeeping off the step's dependency chain (after the row update, no
            // branch): ties of a chain that takes a pivot, NaN / huge candidates, tiny maxima
#ifdef MMB_EXP_SCHEDB
            __builtin_amdgcn_sched_barrier(0);
#endif
            const uint64_t bad = __ballot(!(dl < BIG));                     // NaN, +inf, >= 2^700
            const uint64_t tiny = __ballot((uint32_t)mx < (uint32_t)KEY_LO);  // 0 <= max < 2^-700
            const uint64_t neg = negm;
            uint32_t nlo = (uint32_t)neg, nhi = (uint32_t)(neg >> 32);
            asm("" : "+s"(elo), "+s"(ehi), "+s"(nlo), "+s"(nhi));
            // (a stopping chain's -inf keys tie: ignored.  A live lane cannot share the done lanes'
            // -inf key here: with every diagonal below 2^700 and every pivot above 2^-700, as this
            // pass checks, |lij| <= sqrt(Sigma_ll) < 2^350 for the PSD moment matrix, so work
            // stays finite; a -inf diagonal needs an overflowed Mv^2, whose Mvv is inf too: NaN.)
            const uint32_t tie = ((elo & (elo - 1)) & (nlo ? 0u : ~0u)) | ((ehi & (ehi - 1)) & (nhi ? 0u : ~0u));
            needl = needl | mmb_inverse_ballot(bad | tiny | (tie ? ~0ull : 0ull));
          }
        }
      }
      if constexpr (POSTHOC) {
        // What the optimistic choices could get wrong, checked once after the loop:
        // * a pivot outside the in-range square root's domain [2^-700, 2^700] -- a tiny or zero
        //   maximum, a huge or +inf one, a positive NaN key (it would have been the maximum);
        // * a NaN candidate that never became a pivot (dpstf2 may stop on it; its work stays NaN
        //   to the end because NaN + x = NaN and only pivots reset work);
        // * a high-word tie: every lane holding the maximal key became a pivot at that step, so
        //   the chain has more done lanes than steps that took pivots (pe values 0..max_pe, each
        //   taken once when exact: done == max_pe + 1).
        // On a tie the rows the pass computed after it are garbage; the redo replaces them.
        if constexpr (DW) done = work == inf_s;
        const bool inr = apiv >= 0x1p-700 && apiv <= 0x1p700;
        uint64_t need = __ballot(inb && (done ? !inr : isnan(diag0 - work)));
        const uint64_t dn = __ballot(done && inb);
        const int mpe = gmax_i32((done && inb) ? pe : -1);
        const uint64_t act = __builtin_amdgcn_read_exec();
        const int m0 = __builtin_amdgcn_readlane(mpe, 0), m1 = __builtin_amdgcn_readlane(mpe, 32);
        if ((uint32_t)act != 0u && __builtin_popcount((uint32_t)dn) != m0 + 1) need |= 1ull;
        if ((act >> 32) != 0u && __builtin_popcount((uint32_t)(dn >> 32)) != m1 + 1) need |= 1ull << 32;
        needm = need;
      } else {
        needm |= __ballot(needl);
      }
      return needm != 0;
    };
#if defined(MMB_PCHOL_ONECOPY)
    // one copy of the pass, run once optimistically and, rarely, again checked
#pragma nounroll
    for (int attempt = 0; attempt < 2; ++attempt) {
      int ck = attempt;
      asm volatile("" : "+s"(ck));  // opaque: no peeled second copy
      if (ck) {  // rare: redo with dpstf2's exact decisions
        work = inb ? 0.0 : __builtin_inf();
#pragma unroll
        for (int k = 0; k < DMAX; ++k) Lrow[k] = 0.0;
        done = !inb;
        pe = 0;
        live = true;
      }
      if (!pass(ck != 0) || ck) break;
    }
#else
    if constexpr (OPT) {
#if defined(MMB_EXP_FORCEFAST) || defined(MMB_EXP_NOREDO)
      (void)pass(mmb_bc<false>{});  // timing experiments only: the optimistic pass alone
#elif defined(MMB_PCHOL_EXACT_NOINLINE)
      if (pass(mmb_bc<false>{}))    // rare: redo with dpstf2's exact decisions, out of line
        return pchol32_exact(d, mat, prow, pks, pos_out, NB, seed, xepoch, c, chain, it, b, m);
#elif defined(MMB_PCHOL_COMPACT_REDO)
      if (pass(mmb_bc<false>{})) {  // rare: redo with dpstf2's exact decisions, compact loop
        redo_exact(d, mat, prow, pks, diag0, lc, inb, Lrow, work, done, pe);
      }
#else
      // rare (a few per thousand factorizations): redo with dpstf2's exact decisions; marked
      // unlikely so the block placement moves the checked pass out of the hot code
      if (__builtin_expect(pass(mmb_bc<false>{}), 0)) {
        if (redo_out) *redo_out = 1;
        work = inb ? 0.0 : __builtin_inf();
#pragma unroll
        for (int k = 0; k < DMAX; ++k) Lrow[k] = 0.0;
        done = !inb;
        pe = 0;
        live = true;
        (void)pass(mmb_bc<true>{});
      }
#endif
    } else {
      (void)pass(mmb_bc<true>{});
    }
#endif
    {
      const uint64_t dn = __ballot(done && inb);
      rank = __builtin_popcount(hi_half ? (uint32_t)(dn >> 32) : (uint32_t)dn);
#ifdef MMB_PCHOL_STEPCHECK
      // (an optimistic stop at step 0 of a 32-element block has no done / out-of-range lane to
      // take the garbage pivot: it marked one live lane)
      if (!live && d == G && rank == 1) rank = 0;
#endif
    }
#else
#pragma unroll
    for (int j = 0; j < DMAX; ++j) {
      if (live && j < d) {
        const double dl = diag0 - work;
        // sqrt / reciprocal of the candidate (the compiler keeps them on the pivot lane's
        // path); out of the fast range the pivot lane takes sqrt() and division instead
#ifdef MMB_EXP_RCP_SEQ
        double ajj_s = mmb_sqrt_inrange(dl);
        double rinv_s = mmb_rcp_inrange(ajj_s);
#else
        double ajj_s, rinv_s;
        mmb_sqrt_rcp_inrange(dl, &ajj_s, &rinv_s);
#endif
#ifdef MMB_EXP_PIN_SQRT
        // timing experiment: keep both sequences ahead of the search (the compiler otherwise
        // sinks them into the pivot lane's branch); measured 1 % slower
        asm volatile("" : "+v"(ajj_s), "+v"(rinv_s));
#endif
        // key: high word of a positive candidate, INT_MAX for a NaN candidate, else -1
        // (three independent selects: no branchy nest for the compiler to serialise)
        const int hiw = (int)(mmb_d2u(dl) >> 32);
        int key = dl > 0.0 ? hiw : -1;
        key = isnan(dl) ? 0x7fffffff : key;
        key = done ? -1 : key;
        const int mx = gmax_i32(key);
        const uint32_t win = (uint32_t)(__ballot(key == mx) >> (threadIdx.x & 32));
        int p = __builtin_ctz(win | 0x80000000u);
        bool pos = mx >= 0;
        if (!(mx < 0 || (mx != 0x7fffffff && __builtin_popcount(win) == 1))) {
          double val;
          p = pivot_exact(dl, done, pks, j, d, (int*)prow, &val);
          pos = val > 0.0;
        }
        if (!pos) {
          rank = j;
          live = false;
        } else {
          pks[j] = p;  // same value from every lane of the group: no exec-mask change
          const bool piv = lane == p;
          double ajj = 0.0;
          if (piv) {
            if (j + 1 < d) {  // the last step has no rows left to update: no readers
#pragma unroll
              for (int k = 0; k + 1 < j; k += 2) *(double2*)(prow + k) = make_double2(Lrow[k], Lrow[k + 1]);
              if (j & 1) prow[j - 1] = Lrow[j - 1];
            }
            ajj = ajj_s;  // IEEE results in the fast range (device.h)
            double rinv = rinv_s;
            if (!mmb_fast_range(dl)) {
              ajj = sqrt(dl);
              rinv = 1.0 / ajj;
            }
            prow[RI] = rinv;
          }
          grp_sync();
          if (piv) { Lrow[j] = ajj; pe = j; }
          done = done || piv;
#ifndef MMB_EXP_LDS_DOT
          // pivot row: lane l of each 16-lane row reads elements l and 16 + l (two 8-byte reads
          // instead of j/2 16-byte broadcast reads per lane), then every product takes element k
          // from lane k % 16 of its row by a DPP64 row_newbcast operand.  Every lane of the group
          // runs the dot product (a DPP source lane must be active); done lanes discard it.
          double t0 = 0.0, t1 = 0.0;
          // Sigma(lane, p) and the pivot's reciprocal are read with the row pieces (one LDS wait)
          // Sigma(lc, p) at byte 8 slot = 4 a (a + 1) + 8 b, a = max, b = min: max, min, one
          // 24-bit multiply-add and two shift-adds
          const int sa = max(lc, p), sb = min(lc, p);
          int sq;  // sa (sa + 1) in one instruction (the compiler splits it into three)
          asm("v_mad_u32_u24 %0, %1, %1, %1" : "=v"(sq) : "v"(sa));
          double sig = *(const double*)((const char*)mat + ((sq + 2 * sb) << 2));
          double rinv = prow[RI];
          double pA = prow[lane & 15];
          double pB = j > 16 ? prow[16 + (lane & 15)] : 0.0;
          asm volatile("" : "+v"(sig), "+v"(rinv), "+v"(pA), "+v"(pB));
          if (j > 0 && j + 1 < d) {  // (j = d - 1: every lane is done)
#pragma unroll
            for (int k = 0; k < j; ++k) {
              const double src = k < 16 ? pA : pB;
              if (k & 1) fmac_rowbc_ld(t1, src, Lrow[k], k & 15);
              else fmac_rowbc_ld(t0, src, Lrow[k], k & 15);
            }
          }
#endif
          if (!done) {
#ifdef MMB_EXP_LDS_DOT
            double t0 = 0.0, t1 = 0.0;
#pragma unroll
            for (int k = 0; k + 1 < j; k += 2) {
              const double2 pp = *(const double2*)(prow + k);
              t0 = fma(Lrow[k], pp.x, t0);
              t1 = fma(Lrow[k + 1], pp.y, t1);
            }
            if (j & 1) t0 = fma(Lrow[j - 1], prow[j - 1], t0);
            const double sig = mat[mmb_slot(lane, p)], rinv = prow[RI];
#endif
            const double lij = (sig - (t0 + t1)) * rinv;
            Lrow[j] = lij;
            work = work + lij * lij;
          }
          grp_sync();
        }
      }
    }
#endif  // MMB_PCHOL_V1
    return tail();
  }

  // (i, k) of every packed slot, i << 8 | k, one table per workgroup in LDS (filled once per
  // launch by ik_fill): the moment update reads it instead of inverting tri() per slot
  static constexpr bool IKTAB = (G == 32);
  __device__ __forceinline__ static uint16_t* ik_table() {
    __shared__ uint16_t tab[IKTAB ? TP : 1];
    return tab;
  }
  __device__ __forceinline__ static void ik_fill() {
    if constexpr (IKTAB) {
      for (int t = (int)threadIdx.x; t < TP; t += (int)blockDim.x) {
        int i, k;
        slot_ik(t, i, k);
        ik_table()[t] = (uint16_t)(i << 8 | k);
      }
    }
  }
  // (i, k) of packed slot s = tri(i) + k: float square root estimate, integer correction
  __device__ __forceinline__ static void slot_ik(int s, int& i, int& k) {
    int ii = (int)((sqrtf((float)(8 * s + 1)) - 1.0f) * 0.5f);
    ii += (mmb_tri(ii + 1) <= s) ? 1 : 0;
    ii -= (mmb_tri(ii) > s) ? 1 : 0;
    i = ii;
    k = s - mmb_tri(ii);
  }

  // AMM factorization counters of one update (mmb_amm_stats): rank(F) == n (amm.jl:88), the
  // rank, the factorization steps the group executed (min(rank + 1, n) per chain; on the 32-lane
  // kernels the two chains of a wave step together, so the wave's count is the larger one) and
  // whether the optimistic pass was redone.  Diagnostics: lane 0 of the group, 20 bytes.
  __device__ __forceinline__ static void amm_count(const DBlock& B, int c, int d, int rank, int redo,
                                                   const Grp<G>& g) {
    const int st = rank < d ? rank + 1 : d;
    int ws = st;
    if constexpr (G == 32) {
      const uint64_t act = __builtin_amdgcn_read_exec();  // the upper group may have exited (c >= K)
      const int s0 = __builtin_amdgcn_readlane(st, 0), s1 = __builtin_amdgcn_readlane(st, 32);
      ws = max((uint32_t)act != 0u ? s0 : 0, (act >> 32) != 0u ? s1 : 0);
    }
    if (g.lane == 0) {
      // no-return atomics: fire-and-forget, no HBM round trip on the update's path (a plain
      // load-add-store would wait for the load)
      uint64_t* a = B.t_astat + (size_t)c * MMB_AMM_STAT_STRIDE;
      (void)__hip_atomic_fetch_add(a + 0, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (rank == d) (void)__hip_atomic_fetch_add(a + 1, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      (void)__hip_atomic_fetch_add(a + 2, (uint64_t)rank, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      (void)__hip_atomic_fetch_add(a + 3, (uint64_t)ws, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (redo) (void)__hip_atomic_fetch_add(a + 4, (uint64_t)redo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  // ---------------------------------------------------------------- AMM
  // amm.jl:66-108.  LDS per chain: mat[TP] | z2[DP] | vv[DP] | mv[DP] | ia[2*DP ints]
  // Carried proposal (32-lane groups, diagonal SigmaL): the proposal of the NEXT iteration,
  // x' - v = SigmaL z1' [beta * . + (1 - beta) SigmaLm z2'] (amm.jl:72-76), depends only on
  // that iteration's draws (Philox keyed by the iteration), the tune m after this update and
  // the factor this update computes -- and v is unchanged in between (only this block samples
  // its nodes).  So it is formed right after the factorization, with the factor rows still in
  // registers (no pivot decode), and carried through HBM (t_xnext, 30 doubles) instead of
  // re-reading the factor (465 doubles) next time.  Same operations in the same order, so the
  // draws are bit-identical; the tag (host epoch, iteration) makes any host write of the chain
  // state or a skipped update fall back to the direct path.
  static constexpr bool CARRY = (G == 32 && R == 1);
  // factor storage on device: position form + position bytes (pchol32) or slot form + pivot
  // order (pchol); the host converts to the canonical slot form (engine.cpp mmb_get_tune)
  static constexpr bool POSFORM = (G == 32 && R == 1);
  __device__ __forceinline__ static int64_t xtag(const SweepArgs& A, int64_t it) {
    return (A.xepoch << 32) | (int64_t)(uint32_t)it;
  }
  __device__ __forceinline__ static void amm(const SweepArgs& A, const DBlock& B, int c, uint32_t chain,
                             int64_t it, int b, const mmb_rng& rn,
                             const mmb_rng& ru, bool adapt, St& s, const Lc& l, const Grp<G>& g,
                             double* lds, double upre) {
    const int d = B.d;
    const int T = mmb_tri(d);
    double* mat = lds;
    double* z2s = lds + TP;
    double* vvs = z2s + DP;
    double* mvs = vvs + DP;
    int* ia = (int*)(mvs + DP);  // piv / pos scratch (2*DP ints)
    double v[R], x[R], z1[R], z2[R], mv[R];
    MMB_PROF_START
    M::unlist(B, s, g.lane, v);
    int m = B.t_m[c];
    int fl = B.t_flags[c];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int e = r * G + g.lane;
      mv[r] = e < d ? B.t_Mv[(size_t)c * DP + e] : 0.0;
    }
    const bool fresh = adapt && !(fl & 1);
    bool carried = false;
    if constexpr (CARRY) carried = B.t_xtag != nullptr && !fresh && B.t_xtag[c] == xtag(A, it);
    if (fresh) {  // setadapt!: m = 0, Mv = v (aliased), Mvv = v v', SigmaLm = 0
      m = 0;
      fl = (fl | 2) & ~4;
#pragma unroll
      for (int r = 0; r < R; ++r) mv[r] = v[r];
    }
    fl = adapt ? (fl | 1) : (fl & ~1);
    MMB_PROF_MARK(1, g.lane)
    // proposal: x = SigmaL * z1 [; x = beta*x + (1-beta)*SigmaLm*z2]; x += v
    if (carried) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int e = r * G + g.lane;
        x[r] = e < d ? B.t_xnext[(size_t)c * DP + e] : 0.0;
      }
    } else {
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
        double lt[NT];  // all loads issued before the first use (one HBM latency, not NT)
#pragma unroll
        for (int u = 0; u < NT; ++u) lt[u] = (u * G + g.lane < T) ? Ls[u * G + g.lane] : 0.0;
#pragma unroll
        for (int u = 0; u < NT; ++u)
          if (u * G + g.lane < T) mat[u * G + g.lane] = lt[u];
        if constexpr (POSFORM) {
          // position form: this lane's row starts at tri(pos e); y = sum_{k <= pos e} L z2s[k]
          // in k order (the diagonal last), as the slot-form matvec below
          const int e = g.lane;
          const int pe = e < d ? (int)B.t_piv[(size_t)c * DP + e] : 0;
          if (e < d) z2s[e] = z2[0];
          grp_sync();
          const double* row = mat + mmb_tri(pe);
          double a = 0.0;
#pragma unroll
          for (int k = 0; k < DMAX; ++k)
            if (k < d) a = k <= pe ? fma(row[k], z2s[k], a) : a;
          if (e < d) y[0] = a;
        } else {
        // pivot order: the chain's DP bytes as DP/4 words in registers (uniform per group),
        // so the matvec's LDS reads are independent of each other (no ia[k] -> mat chain)
        uint32_t pw[DP / 4];
        const uint32_t* pvw = (const uint32_t*)(B.t_piv + (size_t)c * DP);
#pragma unroll
        for (int w = 0; w < DP / 4; ++w) pw[w] = pvw[w];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          int e = r * G + g.lane;
          if (e < d) z2s[e] = z2[r];
        }
        grp_sync();
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int e = r * G + g.lane;
          int pe = 0;  // position of e in the pivot order
#pragma unroll
          for (int k = 0; k < DMAX; ++k)
            if (k < d && (int)((pw[k >> 2] >> (8 * (k & 3))) & 0xffu) == e) pe = k;
          double a = 0.0;
#pragma unroll
          for (int k = 0; k < DMAX; ++k) {
            if (k < d) {
              const int q = (int)((pw[k >> 2] >> (8 * (k & 3))) & 0xffu);
              const double m_ = mat[mmb_slot(e, q)];
              const double z_ = z2s[k];
              a = (k < pe) ? fma(m_, z_, a) : a;
            }
          }
          if (e < d) y[r] = fma(mat[mmb_tri(e) + e], z2s[pe], a);
        }
        }  // !POSFORM
      }
#pragma unroll
      for (int r = 0; r < R; ++r) x[r] = B.beta * x[r] + (1.0 - B.beta) * y[r];
    }
    }  // !carried
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = x[r] + v[r];
    MMB_PROF_MARK(2, g.lane)
    const typename M::Prep pc = M::prep(B, s);
    double lx, lv;
    M::logf_p2(A, B, pc, s, l, g, x, v, lx, lv);
    const double ua = G == 32 ? upre : mmb_uniform(&ru, 0u);  // predraw() for 32-lane groups
    if (ua < mmb_exp(lx - lv)) {
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = x[r];
    }
    MMB_PROF_MARK(3, g.lane)
    if (adapt) {  // amm.jl:81-91
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
      // (v[e], Mv[e]) pairs interleaved over the vvs|mvs scratch: one 16-byte read per index
      double2* vm = (double2*)vvs;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int e = r * G + g.lane;
        if (e < d) vm[e] = make_double2(v[r], mv[r]);
      }
      const double cc = (B.scale * B.scale / (double)d) / p;
      double* Mvv = B.t_Mvv + (size_t)c * TP;
      // fresh: Mvv = v_old v_old' was formed before the proposal; v_old is still unlist()
      // of the state `s`, so recompute it from s here (same products).
      double vold[R];
      if (fresh) {
        M::unlist(B, s, g.lane, vold);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          int e = r * G + g.lane;
          if (e < d) z2s[e] = vold[r];
        }
      }
      grp_sync();
      // the lane's own Mvv slots straight into registers, all loads in flight at once.  Slots
      // T <= t < TP are the row's padding (never read as Mvv / Sigma): they are updated like the
      // others from stale scratch, so no slot needs a branch (rats: NT * G == TP exactly), and
      // the new values are stored after the slot loop -- an HBM store between two uses of the
      // loaded values would make every use wait for the stores before it (vmcnt(0)).
      double lt[NT];
#pragma unroll
      for (int u = 0; u < NT; ++u) lt[u] = (!fresh && u * G + g.lane < TP) ? Mvv[u * G + g.lane] : 0.0;
      // slot t = u G + lane: HBM and LDS addresses are the lane's base + a constant per u
      // (immediate offsets), the fresh / steady choice is made once outside the slot loop
      double* const Mvv_l = Mvv + g.lane;
      double* const mat_l = mat + g.lane;
      auto slots = [&](auto fresh_c) {
        constexpr bool FRESH = decltype(fresh_c)::value;
#ifndef MMB_EXP_IK_PERSLOT
        // opaque once per update: the table reads can be issued together (one LDS wait), but
        // not hoisted out of the iteration loop (2 * NT ints live across it: spills)
        int li0 = g.lane;
        asm volatile("" : "+v"(li0));
#endif
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int t = u * G + g.lane;
          if ((u + 1) * G <= TP || t < TP) {
            int i, k;
            if constexpr (IKTAB) {
#ifdef MMB_EXP_IK_PERSLOT
              int li = g.lane;
              asm volatile("" : "+v"(li));
#else
              const int li = li0;
#endif
              const int w = ik_table()[li + u * G];
              i = w >> 8;
              k = w & 255;
            } else {
              int ti = t;
              asm volatile("" : "+v"(ti));
              slot_ik(ti, i, k);
            }
            const double2 a = vm[k], bi = vm[i];
            const double old = FRESH ? z2s[i] * z2s[k] : lt[u];
            const double nv = p * old + (q * a.x) * bi.x;
            lt[u] = nv;
            mat_l[u * G] = cc * (nv - a.y * bi.y);
          }
        }
      };
      if (fresh) slots(mmb_bc<true>{});
      else slots(mmb_bc<false>{});
#pragma unroll
      for (int u = 0; u < NT; ++u)
        if ((u + 1) * G <= TP || u * G + g.lane < TP) Mvv_l[u * G] = lt[u];
      grp_sync();
      // everything but the factorization is finished first; the chain state is parked
      // in LDS so the Cholesky's register footprint does not stack on top of it
#pragma unroll
      for (int r = 0; r < R; ++r) {
        int e = r * G + g.lane;
        if (e < d) B.t_Mv[(size_t)c * DP + e] = mv[r];
      }
      if (g.lane == 0) { B.t_m[c] = m; B.t_flags[c] = fl; }
      M::relist(B, s, g, v);
      M::stash(lds, s, g.lane);
      int* pks = (int*)z2s;  // pivot order (group-uniform values), LDS
      grp_sync();
      MMB_PROF_MARK(4, g.lane)
#ifdef MMB_EXP_NOPCHOL
      int rank = d;  // timing experiment only
#else
      int rank;
      int redo = 0;
      const bool carry = CARRY && B.t_xtag != nullptr && B.sigl_diag;
#ifndef MMB_PCHOL_GENERIC
      int pe = 0;
      if constexpr (G == 32 && R == 1)
        rank = pchol32(d, mat, (double*)ia, pks, g, &pe, carry ? &B : nullptr, A, c, chain, it, b, m, &redo);
      else
#endif
        rank = pchol(d, mat, (double*)ia, pks, g);
#endif
      grp_sync();
      MMB_PROF_MARK(5, g.lane)
      if (B.t_astat != nullptr) amm_count(B, c, d, rank, redo, g);
      if (rank == d) {
        double* Ls = B.t_Ls + (size_t)c * TP;
#pragma unroll
        for (int u = 0; u < NT; ++u)
          if (u * G + g.lane < T) Ls[u * G + g.lane] = mat[u * G + g.lane];
        uint8_t* pv = B.t_piv + (size_t)c * DP;
        if constexpr (POSFORM) {
          if (g.lane < d) pv[g.lane] = (uint8_t)pe;  // position of element lane
        } else {
          for (int k = g.lane; k < d; k += G) pv[k] = (uint8_t)pks[k];
        }
        if (g.lane == 0) B.t_flags[c] = fl | 4;
      }
      M::unstash(lds, s, g.lane);
      grp_sync();
      MMB_PROF_MARK(6, g.lane)
      return;
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
  // The reference shrinks until it accepts (slice.jl:78-88,103-113); a kernel must end, so
  // after MMB_SLICE_MAX_SHRINK rejections the update stops, the chain-update is counted in
  // stat[3] and mmb_run fails with MMB_E_STATE (never a silent out-of-slice draw).  Only a
  // degenerate target gets there (e.g. an infinite width: every candidate is NaN, -Inf).
  __device__ __forceinline__ static void slice_overflow(const SweepArgs& A, const Grp<G>& g) {
    if (g.lane == 0) atomicAdd(&A.nuts_stat[3], 1ull);
  }
  __device__ __forceinline__ static double width(const DBlock& B, int e) {
    return B.width ? B.width[e] : B.width0;
  }
  // The sequential uniforms of a lane group's update (Slice, univariate) 32 at a time: lane j of
  // the group draws index base + j (the same Philox draws, bit-identical), a step takes its index
  // from its lane (ds_bpermute: the two groups of a wave may be at different indices); a group
  // that runs past the window refills it.  Replaces one all-lane Philox per draw.
  struct UWin {
    double u;
    uint32_t base;
  };
  __device__ __forceinline__ static double uwin_next(const mmb_rng& ru, UWin& w, uint32_t k, const Grp<G>& g) {
    if (k - w.base >= (uint32_t)G) {  // group-uniform
      w.base = k;
      w.u = mmb_uniform(&ru, k + (uint32_t)g.lane);
    }
    const int src = (int)(threadIdx.x & 63 & ~(G - 1)) + (int)(k - w.base);
    return __shfl(w.u, src, 64);
  }
  // slice.jl:66-92 (Univariate) with the shrink loop's candidates evaluated four at a time
  // (models with M::SLICE_CAND: lanes 8q .. 8q+7 of the chain evaluate candidate q).  Given that
  // every earlier candidate was rejected, the candidates of a coordinate are fixed in advance:
  // candidate j = lo + (up - lo) * u_j, then lo or up moves to it by its side of the current
  // value -- the loop's arithmetic on its uniforms, independent of the logpdf values.  A round
  // forms the next four on every lane, evaluates them at once (exact logf values: the model's
  // evaluator sums the same tree), and takes the first that the loop would accept; the uniform
  // index, the logf0 carried to the next coordinate and the overflow case follow the loop.  The
  // draws are the sequential loop's, bit for bit.
  __device__ __forceinline__ static void slice_uni_cand(const SweepArgs& A, const DBlock& B, const mmb_rng& ru,
                                                        St& s, const Lc& l, const Grp<G>& g, double* lds) {
    constexpr int SD = M::SLICE_CAND_D;
    constexpr int NC = M::SLICE_NC, LPC = 32 / NC;  // candidates per round, lanes per candidate
    constexpr uint32_t LEAD = NC == 2 ? 0x00010001u : NC == 4 ? 0x01010101u : 0x11111111u;  // group leaders' ballot bits
    static_assert(MMB_SLICE_MAX_SHRINK % NC == 0, "rounds of candidates end at the cap");
    const int d = B.d;
    double x[R];
    M::unlist(B, s, g.lane, x);
    typename M::SCtx cx;
    M::slice_cand_prep(A, B, s, l, g, lds, cx);
#ifndef MMB_EXP_SLICE_LOGF  // (experiment: logf recomputing every sum)
    double logf0 = M::slice_logf0(A, B, s, l, g, x, cx);  // logf, reusing the prep's sums
#else
    double logf0 = M::logf(A, B, s, l, g, x);
#endif
    double lo = 0.0, up = 0.0;
    if (g.lane < d) {
      const double w = width(B, g.lane);
      lo = x[0] - w * mmb_uniform(&ru, (uint32_t)g.lane);
      up = lo + w;
    }
    typename M::SMemo memo;
    double xu[SD], lou[SD], upu[SD];  // element values and intervals, group-uniform
#pragma unroll
    for (int a = 0; a < SD; ++a) {
      xu[a] = a < d ? g.bcast(x[0], a) : 0.0;
      lou[a] = a < d ? g.bcast(lo, a) : 0.0;
      upu[a] = a < d ? g.bcast(up, a) : 0.0;
    }
    uint32_t k = (uint32_t)d;
    UWin uw{0.0, 0xffffffffu - (uint32_t)G};
    const int q = g.lane / LPC;
    const int gbase = (int)(threadIdx.x & 63) & ~(G - 1);
    for (int e = 0; e < d; ++e) {
      const double p0 = logf0 + mmb_log(uwin_next(ru, uw, k++, g));
      double xo = xu[0], lo_ = lou[0], up_ = upu[0];
#pragma unroll
      for (int a = 1; a < SD; ++a)
        if (a == e) { xo = xu[a]; lo_ = lou[a]; up_ = upu[a]; }
      double xn = 0.0, lfn = 0.0;
      // candidate j (from 1) takes uniform k + j - 1
      for (uint32_t j0 = 0;; j0 += NC) {
        double cand[NC];
#pragma unroll
        for (int t = 0; t < NC; ++t) {
          const double cv = lo_ + (up_ - lo_) * uwin_next(ru, uw, k + j0 + (uint32_t)t, g);
          cand[t] = cv;
          if (cv < xo) lo_ = cv;
          else up_ = cv;
        }
        double mine = cand[0];
#pragma unroll
        for (int t = 1; t < NC; ++t) mine = q == t ? cand[t] : mine;
        double xv[SD];
#pragma unroll
        for (int a = 0; a < SD; ++a) xv[a] = a == e ? mine : xu[a];
        const double lp = M::slice_cand_logf(A, B, s, cx, xv, g.lane, memo);
        const bool hit = !(lp < p0) && j0 + (uint32_t)q + 1u <= (uint32_t)MMB_SLICE_MAX_SHRINK;
        const uint64_t bal = __ballot(hit && (g.lane & (LPC - 1)) == 0);
        const uint32_t hb = (uint32_t)(bal >> gbase) & LEAD;  // candidate q -> bit LPC q
        if (hb != 0u) {
          const int qs = __builtin_ctz(hb) / LPC;
          xn = cand[0];
#pragma unroll
          for (int t = 1; t < NC; ++t) xn = qs == t ? cand[t] : xn;
          lfn = __shfl(lp, gbase + LPC * qs, 64);
          k += j0 + (uint32_t)qs + 1u;
          break;
        }
        if (j0 + (uint32_t)NC >= (uint32_t)MMB_SLICE_MAX_SHRINK) {  // every candidate up to the cap rejected:
          xn = lo_ + (up_ - lo_) * uwin_next(ru, uw, k + j0 + (uint32_t)NC, g);  // the loop's last draw
          lfn = __shfl(lp, gbase + LPC * (NC - 1), 64);                           // logf of the cap-th
          k += j0 + (uint32_t)NC + 1u;
          slice_overflow(A, g);
          break;
        }
      }
#pragma unroll
      for (int a = 0; a < SD; ++a) xu[a] = a == e ? xn : xu[a];
      logf0 = lfn;
      if (g.lane == e) x[0] = xn;
    }
    M::relist(B, s, g, x);
  }
  // slice.jl:66-92 (Univariate)
  __device__ __forceinline__ static void slice_uni(const SweepArgs& A, const DBlock& B, const mmb_rng& ru, St& s,
                                   const Lc& l, const Grp<G>& g, double* lds) {
    if constexpr (M::SLICE_CAND && G == 32 && R == 1) {
      if (A.slice_exact == 0 && M::slice_cand_ok(B)) {
        slice_uni_cand(A, B, ru, s, l, g, lds);
        return;
      }
    }
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
    UWin uw{0.0, 0xffffffffu - (uint32_t)G};  // empty window: the first draw fills it
    auto next_u = [&](uint32_t kk) __attribute__((always_inline)) -> double {
      if constexpr (G == 32) return uwin_next(ru, uw, kk, g);
      else return mmb_uniform(&ru, kk);
    };
#pragma unroll
    for (int r = 0; r < R; ++r) {
      for (int ln = 0; ln < G; ++ln) {
        int e = r * G + ln;
        if (e >= d) break;
        bool own = g.lane == ln;
        double p0 = logf0 + mmb_log(next_u(k++));
        double xo = x[r];
        double u = next_u(k++);
        if (own) x[r] = lo[r] + (up[r] - lo[r]) * u;
        bool hit = false;
        for (int guard = 0; guard < MMB_SLICE_MAX_SHRINK; ++guard) {
          logf0 = M::logf(A, B, s, l, g, x);
          if (!(logf0 < p0)) { hit = true; break; }
          if (own) {
            double value = x[r];
            if (value < xo) lo[r] = value;
            else up[r] = value;
          }
          u = next_u(k++);
          if (own) x[r] = lo[r] + (up[r] - lo[r]) * u;
        }
        if (!hit) slice_overflow(A, g);
      }
    }
    M::relist(B, s, g, x);
  }
  // slice.jl:95-117 (Multivariate), candidates four at a time as slice_uni_cand: candidate 1 is
  // w u + lo per element, candidate j > 1 moves each lo / up to candidate j - 1's element by its
  // side of the current value and draws lo + (up - lo) u, uniforms 1 + 2d + (j - 2) d + e
  __device__ __forceinline__ static void slice_multi_cand(const SweepArgs& A, const DBlock& B, const mmb_rng& ru,
                                                          St& s, const Lc& l, const Grp<G>& g, double* lds) {
    constexpr int SD = M::SLICE_CAND_D;
    const int d = B.d;
    double v[R];
    M::unlist(B, s, g.lane, v);
    UWin uw{0.0, 0xffffffffu - (uint32_t)G};
    typename M::SCtx cx;
    M::slice_cand_prep(A, B, s, l, g, lds, cx);
#ifndef MMB_EXP_SLICE_LOGF
    const double p0 = M::slice_logf0(A, B, s, l, g, v, cx) + mmb_log(uwin_next(ru, uw, 0u, g));
#else
    const double p0 = M::logf(A, B, s, l, g, v) + mmb_log(uwin_next(ru, uw, 0u, g));
#endif
    typename M::SMemo memo;
    double vu[SD], lo[SD], up[SD], x1[SD];
#pragma unroll
    for (int a = 0; a < SD; ++a) {
      vu[a] = a < d ? g.bcast(v[0], a) : 0.0;
      lo[a] = up[a] = x1[a] = 0.0;
      if (a < d) {
        const double w = width(B, a);
        lo[a] = vu[a] - w * uwin_next(ru, uw, 1u + (uint32_t)a, g);
        up[a] = lo[a] + w;
        x1[a] = w * uwin_next(ru, uw, 1u + (uint32_t)d + (uint32_t)a, g) + lo[a];
      }
    }
    constexpr int NC = M::SLICE_NC, LPC = 32 / NC;
    constexpr uint32_t LEAD = NC == 2 ? 0x00010001u : NC == 4 ? 0x01010101u : 0x11111111u;
    const int q = g.lane / LPC;
    const int gbase = (int)(threadIdx.x & 63) & ~(G - 1);
    double prev[SD], xn[SD];
    // candidate j > 1 from candidate j - 1 (the loop's shrink and redraw)
    auto next = [&](const double* pv, uint32_t j, double* out) __attribute__((always_inline)) {
      const uint32_t kk = 1u + 2u * (uint32_t)d + (j - 2u) * (uint32_t)d;
#pragma unroll
      for (int a = 0; a < SD; ++a) {
        if (a < d) {
          if (pv[a] < vu[a]) lo[a] = pv[a];
          else up[a] = pv[a];
          out[a] = lo[a] + (up[a] - lo[a]) * uwin_next(ru, uw, kk + (uint32_t)a, g);
        } else {
          out[a] = 0.0;
        }
      }
    };
    for (uint32_t j0 = 0;; j0 += NC) {
      double cand[NC][SD];
#pragma unroll
      for (int t = 0; t < NC; ++t) {
        if (j0 + (uint32_t)t == 0u) {
#pragma unroll
          for (int a = 0; a < SD; ++a) cand[t][a] = x1[a];
        } else {
          next(t == 0 ? prev : cand[t - 1], j0 + (uint32_t)t + 1u, cand[t]);
        }
      }
#pragma unroll
      for (int a = 0; a < SD; ++a) prev[a] = cand[NC - 1][a];
      double xv[SD];
#pragma unroll
      for (int a = 0; a < SD; ++a) {
        xv[a] = cand[0][a];
#pragma unroll
        for (int t = 1; t < NC; ++t) xv[a] = q == t ? cand[t][a] : xv[a];
      }
      const double lp = M::slice_cand_logf(A, B, s, cx, xv, g.lane, memo);
      const bool hit = !(lp < p0) && j0 + (uint32_t)q + 1u <= (uint32_t)MMB_SLICE_MAX_SHRINK;
      const uint64_t bal = __ballot(hit && (g.lane & (LPC - 1)) == 0);
      const uint32_t hb = (uint32_t)(bal >> gbase) & LEAD;
      if (hb != 0u) {
        const int qs = __builtin_ctz(hb) / LPC;
#pragma unroll
        for (int a = 0; a < SD; ++a) {
          xn[a] = cand[0][a];
#pragma unroll
          for (int t = 1; t < NC; ++t) xn[a] = qs == t ? cand[t][a] : xn[a];
        }
        break;
      }
      if (j0 + (uint32_t)NC >= (uint32_t)MMB_SLICE_MAX_SHRINK) {  // the cap: the loop's last shrink and draw
        next(prev, j0 + (uint32_t)NC + 1u, xn);
        slice_overflow(A, g);
        break;
      }
    }
    double x[R];
    x[0] = 0.0;
#pragma unroll
    for (int a = 0; a < SD; ++a)
      if (g.lane == a && a < d) x[0] = xn[a];
    M::relist(B, s, g, x);
  }
  // slice.jl:95-117 (Multivariate)
  __device__ __forceinline__ static void slice_multi(const SweepArgs& A, const DBlock& B, const mmb_rng& ru, St& s,
                                     const Lc& l, const Grp<G>& g, double* lds) {
    if constexpr (M::SLICE_CAND && G == 32 && R == 1) {
      if (A.slice_exact == 0 && M::slice_cand_ok(B)) {
        slice_multi_cand(A, B, ru, s, l, g, lds);
        return;
      }
    }
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
    bool hit = false;
    for (int guard = 0; guard < MMB_SLICE_MAX_SHRINK; ++guard) {
      if (!(M::logf(A, B, s, l, g, x) < p0)) { hit = true; break; }
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
    if (!hit) slice_overflow(A, g);
    M::relist(B, s, g, x);
  }

  // ---------------------------------------------------------------- NUTS
  // sample!(v::NUTSVariate) with the model gradient computed inline (nuts.h machine).
  // Model path: adapts iff iter <= burnin (nuts.jl:52).
  __device__ __forceinline__ static void nuts(const SweepArgs& A, const DBlock& B, int c, int64_t it, int b,
                                              St& s, const Grp<G>& g) {
    using NU = Nuts<G, R>;
    typename NU::St S;
    const double* tn = B.t_nuts + (size_t)c * 8;
    S.t_eps = tn[0]; S.t_epsbar = tn[1]; S.t_Hbar = tn[2]; S.t_mu = tn[3];
    S.t_alpha = tn[4]; S.t_nalpha = tn[5];
    S.t_m = B.t_m[c];
    S.t_flags = B.t_flags[c];
    M::unlist(B, s, g.lane, S.v);
    S.pc = NPC_BEGIN;
    const uint32_t chain = A.chain_offset + (uint32_t)c;
    typename NU::Env E;
    E.d = B.d;
    E.lane = g.lane;
    E.adapt = it <= A.model_burnin;
    E.target = B.target;
    E.rn = mmb_rng_make(A.seed, chain, (uint32_t)it, (uint32_t)b, MMB_SUB_NORMAL);
    E.ru = mmb_rng_make(A.seed, chain, (uint32_t)it, (uint32_t)b, MMB_SUB_UNIFORM);
    E.ri = mmb_rng_make(A.seed, chain, (uint32_t)it, (uint32_t)b, MMB_SUB_INIT);
    E.F = B.t_nfr + (size_t)c * NutsFrames<NU::DV>::DBL;
    E.stat = A.nuts_stat;
    while (NU::advance(S, E, g)) S.lf = M::logf_grad(A, B, s, S.x, S.g);
    double* tw = B.t_nuts + (size_t)c * 8;
    if (g.lane == 0) {
      tw[0] = S.t_eps; tw[1] = S.t_epsbar; tw[2] = S.t_Hbar; tw[3] = S.t_mu;
      tw[4] = S.t_alpha; tw[5] = S.t_nalpha;
      B.t_m[c] = S.t_m;
      B.t_flags[c] = S.t_flags;
    }
    M::relist(B, s, g, S.v);
  }

  // ---------------------------------------------------------------- HMC / MALA
  // sample!(v::HMCVariate) (hmc.jl:72-111) / sample!(v::MALAVariate) (mala.jl:67-86), hmc.h
  // machines with the model gradient computed inline; tune (epsilon, L) is per chain.
  template <bool MALA>
  __device__ __forceinline__ static void hmc(const SweepArgs& A, const DBlock& B, int c, const mmb_rng& rn,
                                             const mmb_rng& ru, St& s, const Grp<G>& g) {
    using HM = Hmc<G, R>;
    typename HM::St S;
    typename HM::Env E;
    const double* th = B.t_hmc + (size_t)c * 2;
    E.d = B.d;
    E.lane = g.lane;
    E.eps = th[0];
    E.L = (int)th[1];
    E.sigl = B.sigl;
    E.rn = rn;
    E.ru = ru;
    M::unlist(B, s, g.lane, S.v);
    S.pc = HPC_BEGIN;
    if (MALA) {
      while (HM::advance_mala(S, E, g)) S.lf = M::logf_grad(A, B, s, S.x, S.g);
    } else {
      while (HM::advance_hmc(S, E, g)) S.lf = M::logf_grad(A, B, s, S.x, S.g);
    }
    M::relist(B, s, g, S.v);
  }
};
