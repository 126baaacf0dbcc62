/*
 * mmb_math.h — counter-based RNG and elementary functions used bit for bit by
 * the HIP kernels AND the CPU oracle (oracle/oracle.c includes this header; with
 * ir_math.h, the node IR's element densities, it is the only product code the oracle shares).
 *
 * Why shared: Mamba.jl's MersenneTwister/ziggurat streams and openlibm cannot
 * be reproduced, so parity is oracle <-> GPU on identical Philox streams
 * (SURVEY §8c).  Bit-exact accept decisions and bit-exact AMM pivoted-Cholesky
 * rank decisions (src/samplers/amm.jl:86-90) need identical exp/log/sincos on
 * host and device: ocml and glibc differ in the last ulp.  Everything here uses
 * only correctly rounded IEEE operations (+ - * / sqrt, explicit fma) and
 * integer arithmetic; build with -ffp-contract=off on both sides.
 * This layer is pinned independently: Philox against the Random123 known-answer
 * vectors (cross-checked with rocRAND's header), exp/log/sincos against libm in
 * tests/test_math.py.
 *
 * RNG layout.  One 128-bit Philox4x32-10 block per (key=seed, counter):
 *   ctr.x = block index within the substream, ctr.y = tag = block*16 + substream,
 *   ctr.z = iteration (Model.iter), ctr.w = global chain id.
 * uniform #k of a substream  = 53-bit [0,1) from 64-bit half (k&1) of block k>>1
 * normal pair #q            = Box-Muller on the two uniforms of block q: (r cos t, r sin t)
 * normal #k                 = component (k&1) of pair k>>1.
 */
#ifndef MMB_MATH_H
#define MMB_MATH_H

#if !defined(__HIPCC_RTC__)
#include <stdint.h>
#include <math.h>
#endif

#if defined(__HIPCC__) || defined(__HIP__)
#define MMB_HD __host__ __device__ static inline
#else
#define MMB_HD static inline
#endif

/* substreams */
#define MMB_SUB_NORMAL 0u   /* proposal normals (AMWG z, AMM z1/z2, NUTS momentum, Gibbs normals) */
#define MMB_SUB_UNIFORM 1u  /* accept / slice / tree uniforms (running index) */
#define MMB_SUB_GAMMA_N 2u  /* Marsaglia-Tsang normals */
#define MMB_SUB_GAMMA_U 3u  /* Marsaglia-Tsang uniforms */
#define MMB_SUB_INIT 4u     /* nutsepsilon momentum (nuts.jl:194) */

#define MMB_LOG2PI 1.8378770664093454835606594728112352797
#define MMB_TWOPI_HI 6.28318530717958623200e+00
#define MMB_TWOPI_LO 2.44929359829470635445e-16

MMB_HD uint64_t mmb_d2u(double x) {
  union { double d; uint64_t u; } c;
  c.d = x;
  return c.u;
}
MMB_HD double mmb_u2d(uint64_t u) {
  union { double d; uint64_t u; } c;
  c.u = u;
  return c.d;
}

/* ------------------------------------------------------------------ Philox4x32-10 */
MMB_HD void mmb_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                              uint32_t k0, uint32_t k1, uint32_t out[4]) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

typedef struct {
  uint32_t k0, k1;  /* seed */
  uint32_t tag;     /* block*16 + substream */
  uint32_t iter;    /* Model.iter */
  uint32_t chain;   /* global chain id */
} mmb_rng;

MMB_HD mmb_rng mmb_rng_make(uint64_t seed, uint32_t chain, uint32_t iter, uint32_t block,
                            uint32_t sub) {
  mmb_rng s;
  s.k0 = (uint32_t)seed;
  s.k1 = (uint32_t)(seed >> 32);
  s.tag = block * 16u + sub;
  s.iter = iter;
  s.chain = chain;
  return s;
}

MMB_HD void mmb_rng_block(const mmb_rng* s, uint32_t idx, uint64_t* a, uint64_t* b) {
  uint32_t o[4];
  mmb_philox4x32_10(idx, s->tag, s->iter, s->chain, s->k0, s->k1, o);
  *a = (uint64_t)o[0] | ((uint64_t)o[1] << 32);
  *b = (uint64_t)o[2] | ((uint64_t)o[3] << 32);
}

/* 53-bit uniform on [0,1) (Julia rand() is [0,1) too) */
MMB_HD double mmb_u01(uint64_t bits) { return (double)(bits >> 11) * 0x1.0p-53; }

MMB_HD double mmb_uniform(const mmb_rng* s, uint32_t k) {
  uint64_t a, b;
  mmb_rng_block(s, k >> 1, &a, &b);
  return mmb_u01((k & 1u) ? b : a);
}

/* Test-only AMWG probe (MMB_AMWG_PROBE=1, kernels and oracle alike): coordinate j's accept
 * uniform becomes exp(d_j) * (1 + k 2^-52), d_j the coordinate's log-density difference formed
 * from its own terms (samplers.h amwg_lanes), so the uniforms sit a few ulps to ~2^-12 off the
 * accept threshold.  Per block update (the uniform stream's chain, iteration and tag) a hash
 * picks mode 0 -- every |k| >= 2^20, outside the lane-parallel decision's band, so the update
 * is decided lane-parallel -- or mode 1 -- |k| in {0, 2^3 .. 2^18}, the band edge and inside, so
 * the update falls back to the sequential loop; the sign is per coordinate.  This returns
 * 1 + k 2^-52 (exact). */
MMB_HD double mmb_amwg_probe_factor(const mmb_rng* s, uint32_t j) {
  uint32_t h = (s->chain * 0x9E3779B1u) ^ (s->iter * 0x85EBCA77u) ^ (s->tag * 0xC2B2AE3Du);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  uint32_t q = h ^ (j * 0x27D4EB2Fu);
  q ^= q >> 13;
  q *= 0x165667B1u;
  q ^= q >> 16;
  int e;
  if ((h & 1u) == 0u) {
    const uint32_t r = q & 3u;
    e = r == 0u ? 20 : r == 1u ? 24 : r == 2u ? 30 : 40;
  } else {
    e = 3 + (int)(q & 15u);  /* 3 .. 18 */
    if (((q >> 4) & 7u) == 0u) return 1.0;  /* k = 0 */
  }
  const double f = mmb_u2d((uint64_t)(1023 + e - 52) << 52); /* 2^(e - 52) */
  return ((q >> 8) & 1u) ? 1.0 - f : 1.0 + f;
}

/* ------------------------------------------------------------------ log (fdlibm e_log.c) */
MMB_HD double mmb_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
               Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
               Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  uint64_t u = mmb_d2u(x);
  int32_t hx = (int32_t)(u >> 32);
  uint32_t lx = (uint32_t)u;
  int32_t k = 0;
  if (hx < 0x00100000) { /* x < 2**-1022 */
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -__builtin_inf();
    if (hx < 0) return __builtin_nan("");
    k -= 54;
    x *= two54;
    u = mmb_d2u(x);
    hx = (int32_t)(u >> 32);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  x = mmb_u2d(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (u & 0xffffffffull));
  k += (i >> 20);
  double f = x - 1.0;
  double dk, R;
  if ((0x000fffff & (2 + hx)) < 3) { /* -2**-20 <= f < 2**-20 */
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  double s = f / (2.0 + f);
  dk = (double)k;
  double z = s * s;
  i = hx - 0x6147a;
  double w = z * z;
  int32_t j = 0x6b851 - hx;
  double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  if (i > 0) {
    double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* ------------------------------------------------------------------ exp (fdlibm e_exp.c) */
MMB_HD double mmb_exp(double x) {
  const double o_threshold = 7.09782712893383973096e+02,
               u_threshold = -7.45133219101941108420e+02, ln2HI = 6.93147180369123816490e-01,
               ln2LO = 1.90821492927058770002e-10, invln2 = 1.44269504088896338700e+00,
               P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08, twom1000 = 9.33263618503218878990e-302;
  uint64_t u = mmb_d2u(x);
  uint32_t hx = (uint32_t)(u >> 32);
  int xsb = (int)((hx >> 31) & 1u);
  hx &= 0x7fffffffu;
  double hi = 0.0, lo = 0.0, c, t, y;
  int k = 0;
  if (hx >= 0x40862E42u) { /* |x| >= 709.78 */
    if (hx >= 0x7ff00000u) {
      if (((hx & 0xfffffu) | (uint32_t)u) != 0) return x + x; /* NaN */
      return xsb == 0 ? x : 0.0;
    }
    if (x > o_threshold) return __builtin_inf();
    if (x < u_threshold) return 0.0;
  }
  if (hx > 0x3fd62e42u) { /* |x| > 0.5 ln2 */
    if (hx < 0x3FF0A2B2u) { /* and |x| < 1.5 ln2 */
      if (xsb == 0) { hi = x - ln2HI; lo = ln2LO; k = 1; }
      else { hi = x + ln2HI; lo = -ln2LO; k = -1; }
    } else {
      k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
      t = (double)k;
      hi = x - t * ln2HI; /* exact */
      lo = t * ln2LO;
    }
    x = hi - lo;
  } else if (hx < 0x3e300000u) { /* |x| < 2**-28 */
    return 1.0 + x;
  } else {
    k = 0;
  }
  t = x * x;
  c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
  y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
  if (k >= -1021) return mmb_u2d(mmb_d2u(y) + ((uint64_t)(int64_t)k << 52));
  return mmb_u2d(mmb_d2u(y) + ((uint64_t)(int64_t)(k + 1000) << 52)) * twom1000;
}

/* log1p via the Goldberg trick (exact-argument correction) */
/* The probe's uniform (see mmb_amwg_probe_factor): exp(d_j) (1 + k 2^-52), kept inside a uniform's
 * range [0, 1) -- the lane-parallel decision's certainty tests assume it (a threshold >= 1 is a
 * certain accept for every real uniform); a NaN d_j gives the largest uniform. */
MMB_HD double mmb_amwg_probe_uniform(double del, const mmb_rng* s, uint32_t j) {
  const double u = mmb_exp(del) * mmb_amwg_probe_factor(s, j);
  const double umax = 0x1.fffffffffffffp-1;
  return u < umax ? u : umax;
}

MMB_HD double mmb_log1p(double t) {
  double u = 1.0 + t;
  if (u == 1.0) return t;
  return mmb_log(u) * (t / (u - 1.0));
}

/* ------------------------------------------------------------------ sin/cos of 2*pi*u, u in [0,1) */
MMB_HD double mmb_ksin(double x) { /* fdlibm __kernel_sin(x, 0, 0), |x| <= pi/4 */
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x;
  double v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x + v * (S1 + z * r);
}
MMB_HD double mmb_kcos(double x) { /* fdlibm __kernel_cos(x, 0), |x| <= pi/4 */
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  uint32_t ix = (uint32_t)(mmb_d2u(x) >> 32) & 0x7fffffffu;
  if (ix < 0x3e400000u) return 1.0; /* |x| < 2**-27 */
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333u) return 1.0 - (0.5 * z - (z * r));
  double qx;
  if (ix > 0x3fe90000u) qx = 0.28125;
  else qx = mmb_u2d((uint64_t)(ix - 0x00200000u) << 32);
  double hz = 0.5 * z - qx;
  double a = 1.0 - qx;
  return a - (hz - (z * r));
}
MMB_HD void mmb_sincos2pi(double u, double* s, double* c) {
  double q = rint(4.0 * u); /* nearest quarter turn, exact */
  int iq = (int)q;
  double y = u - 0.25 * q; /* exact, |y| <= 1/8 */
  double th = fma(y, MMB_TWOPI_HI, y * MMB_TWOPI_LO);
  double sk = mmb_ksin(th), ck = mmb_kcos(th);
  switch (iq & 3) {
    case 0: *s = sk; *c = ck; break;
    case 1: *s = ck; *c = -sk; break;
    case 2: *s = -sk; *c = -ck; break;
    default: *s = -ck; *c = sk; break;
  }
}

/* ------------------------------------------------------------------ normals */
/* Box-Muller of one Philox block (a, b): the pair mmb_normal_pair returns */
MMB_HD void mmb_normal_pair_bits(uint64_t a, uint64_t b, double* z0, double* z1) {
  double u0 = mmb_u01(a), u1 = mmb_u01(b);
  double r = sqrt(-2.0 * mmb_log(1.0 - u0));
  double sn, cs;
  mmb_sincos2pi(u1, &sn, &cs);
  *z0 = r * cs;
  *z1 = r * sn;
}
MMB_HD void mmb_normal_pair(const mmb_rng* s, uint32_t q, double* z0, double* z1) {
  uint64_t a, b;
  mmb_rng_block(s, q, &a, &b);
  mmb_normal_pair_bits(a, b, z0, z1);
}
MMB_HD double mmb_normal(const mmb_rng* s, uint32_t k) {
  double z0, z1;
  mmb_normal_pair(s, k >> 1, &z0, &z1);
  return (k & 1u) ? z1 : z0;
}

/* ------------------------------------------------------------------ Gamma(a, 1), a >= 1
 * Marsaglia & Tsang (2000).  Normals from substream GAMMA_N (running index *kn),
 * uniforms from GAMMA_U (running index *ku).  Used by rand(InverseGamma(a, b)) = b / G. */
MMB_HD double mmb_gamma_mt(double a, const mmb_rng* sn, const mmb_rng* su, uint32_t* kn,
                           uint32_t* ku) {
  double d = a - 1.0 / 3.0;
  double c = 1.0 / sqrt(9.0 * d);
  for (;;) {
    double x, v;
    do {
      x = mmb_normal(sn, (*kn)++);
      v = 1.0 + c * x;
    } while (!(v > 0.0));
    v = v * v * v;
    double u = mmb_uniform(su, (*ku)++);
    double x2 = x * x;
    if (u < 1.0 - 0.0331 * (x2 * x2)) return d * v;
    if (mmb_log(u) < 0.5 * x2 + d * (1.0 - v + mmb_log(v))) return d * v;
  }
}

/* ---- logistic likelihood (BASELINE config 4): y ~ Bernoulli(invlogit(eta)).
 * Per observation: log-density y*eta - softplus(eta) and score residual y - invlogit(eta),
 * both from t = exp(-|eta|) (stable for any eta).  Summation spec of the batched gradient
 * (restated by the oracle): rows are split into MMB_LG_NG groups of MMB_LG_NS sub-ranges of
 * mmb_lg_rps(N) rows (a multiple of the 16-row MFMA tile).  Within a sub-range each
 * gradient component is one fma chain over its rows in order; a group's partial is
 * ((P0 + P1) + P2) + ... over its MMB_LG_NS sub-ranges; the gradient is -beta/sd^2 + G0 + G1 + ... in group order. */
#ifndef MMB_LG_NG
#define MMB_LG_NG 32
#endif
#ifndef MMB_LG_NS
#define MMB_LG_NS 2
#endif
#define MMB_LG_DV 64 /* coefficients per chain, padded (p <= 64) */
MMB_HD int mmb_lg_rps(int N) {
  int per = (N + MMB_LG_NG * MMB_LG_NS - 1) / (MMB_LG_NG * MMB_LG_NS);
  return ((per + 15) / 16) * 16;
}
/* exp(x) for x <= 0, branch- and division-free (the logistic per-row terms run it for every
 * row x chain of every gradient): k = round(x / ln2) by the 1.5*2^52 shift, two-step
 * reduction by fma (|r| <= ln2/2), degree-13 Taylor polynomial in Horner form (truncation
 * < 2^-57), 2^k through the exponent field (two steps below 2^-1021).  Only IEEE +, *, fma:
 * bit-identical on host and device.  x < -745.2 -> 0; NaN -> NaN. */
MMB_HD double mmb_exp_neg(double x) {
  const double shift = 0x1.8p52, invln2 = 1.44269504088896338700e+00,
               ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10;
  const double xc = x > -745.2 ? x : -745.2;             /* NaN stays NaN through fma below */
  const double kd = fma(xc, invln2, shift) - shift;
  double r = fma(-kd, ln2HI, xc);
  r = fma(-kd, ln2LO, r);
  double p = 1.6059043836821613e-10;                  /* 1/13! */
  p = fma(p, r, 2.08767569878681e-09);              /* 1/12! */
  p = fma(p, r, 2.505210838544172e-08);
  p = fma(p, r, 2.755731922398589e-07);
  p = fma(p, r, 2.7557319223985893e-06);
  p = fma(p, r, 2.48015873015873e-05);
  p = fma(p, r, 1.984126984126984e-04);
  p = fma(p, r, 1.388888888888889e-03);
  p = fma(p, r, 8.333333333333333e-03);
  p = fma(p, r, 4.1666666666666664e-02);
  p = fma(p, r, 1.6666666666666666e-01);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  const int32_t k = (int32_t)kd;                          /* -1075 .. 0 */
  const double big = mmb_u2d(mmb_d2u(p) + ((uint64_t)(int64_t)k << 52));
  const double small = mmb_u2d(mmb_d2u(p) + ((uint64_t)(int64_t)(k + 1000) << 52)) * 9.33263618503218878990e-302;
  const double e = k >= -1021 ? big : small;
  const double z = x > -745.2 ? e : 0.0 * e; /* e used on both sides: the compiler keeps it branch-free */
  return x != x ? x : z;
}

/* Per-row terms of the logistic likelihood: t = exp(-|eta|), a = 1 + t, R = 1/a (one IEEE
 * division);  lin = y*eta - max(eta, 0),  lp = lin - log(a)  (so lp = y*eta - softplus(eta)),
 * res = y - invlogit(eta) = y - (eta >= 0 ? R : t R).
 * The log(a) terms are not taken per row: a lane multiplies its rows' factors a (each in
 * [1, 2]) into P * 2^E and takes one log at the end (mmb_lg_lane_lp).  Renormalising P is a
 * scaling by a power of two, exact in the normal range, so the product's value does not
 * depend on when it is renormalised -- only on the multiplication order (the spec). */
MMB_HD void mmb_logistic_row(double eta, double y, double* lin, double* a, double* res) {
  const double t = mmb_exp_neg(-fabs(eta));
  const double aa = 1.0 + t;
  const double R = 1.0 / aa;
  *lin = y * eta - (eta > 0.0 ? eta : 0.0);
  *a = aa;
  *res = y - (eta >= 0.0 ? R : t * R);
}
/* P = m 2^e (finite, >= 1) -> P = m in [1, 2), E += e; NaN / inf stay as they are */
MMB_HD void mmb_lg_renorm(double* P, int* E) {
  const uint64_t u = mmb_d2u(*P);
  const int ex = (int)((u >> 52) & 0x7ff);
  const int fin = ex != 0x7ff;
  *E += fin ? ex - 1023 : 0;
  *P = fin ? mmb_u2d((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull) : *P;
}
/* a lane's lp partial: (sum of its lin) - log(product of its a) */
MMB_HD double mmb_lg_lane_lp(double A, double P, int E) {
  mmb_lg_renorm(&P, &E);
  return A - (mmb_log(P) + (double)E * 6.93147180559945286227e-01);
}

#endif /* MMB_MATH_H */
