/*
 * ir_math.h — elementwise layer of the node IR, shared bit for bit by
 * the HIP kernels (ir.h) and the CPU oracle (oracle.c), like mmb_math.h: element log
 * densities of the Distributions 0.10 families (not vendored; formulas restated, DESIGN.md
 * §2), the transform rules of src/distributions/transformdistribution.jl:6-93, the unary
 * operators of the expression code (Mamba's invlogit/logit, src/utils.jl:64-68) and lgamma.
 * Pinned independently: element densities against scipy.stats and lgamma against libm
 * (tests/test_ir.py).
 */
#ifndef MMB_IR_MATH_H
#define MMB_IR_MATH_H
#include "../../include/mamba_hip.h"
#include "mmb_math.h"

/* lgamma(x) for x > 0: shift to z >= 10 by the product x(x+1)...(x+k-1), then Stirling's
 * series through z^-13 (truncation < 4e-17 at z = 10); ~1e-15 relative error. */
MMB_HD double mmb_lgamma(double x) {
  if (!(x > 0.0)) return x == 0.0 ? __builtin_inf() : __builtin_nan("");
  if (x > 1e300) return __builtin_inf();
  double z = x, p = 1.0;
  while (z < 10.0) {
    p = p * z;
    z = z + 1.0;
  }
  const double iz = 1.0 / z, iz2 = iz * iz;
  double s = 1.0 / 156.0;
  s = s * iz2 + (-691.0 / 360360.0);
  s = s * iz2 + (1.0 / 1188.0);
  s = s * iz2 + (-1.0 / 1680.0);
  s = s * iz2 + (1.0 / 1260.0);
  s = s * iz2 + (-1.0 / 360.0);
  s = s * iz2 + (1.0 / 12.0);
  const double half_log2pi = 0.91893853320467274178032973640561764;
  double r = (z - 0.5) * mmb_log(z) - z + half_log2pi + s * iz;
  if (p != 1.0) r = r - mmb_log(p);
  return r;
}

/* Mamba invlogit / logit (src/utils.jl:64-68) */
MMB_HD double mmb_invlogit(double x) { return 1.0 / (mmb_exp(-x) + 1.0); }
MMB_HD double mmb_logit(double x) { return mmb_log(x / (1.0 - x)); }

MMB_HD double mmb_ir_unary(int op, double a) {
  switch (op) {
    case MMB_IR_OP_NEG: return -a;
    case MMB_IR_OP_EXP: return mmb_exp(a);
    case MMB_IR_OP_LOG: return mmb_log(a);
    case MMB_IR_OP_SQRT: return sqrt(a);
    case MMB_IR_OP_INVLOGIT: return mmb_invlogit(a);
    case MMB_IR_OP_LOGIT: return mmb_logit(a);
    default: return a < 0.0 ? -a : a; /* MMB_IR_OP_ABS */
  }
}

/* link kind of a family (transformdistribution.jl): 0 identity (RealDistribution, 53-61),
 * 1 log (PositiveDistribution, 66-78), 2 logit (UnitDistribution, 83-93), 3 affine logit
 * (bounded TransformDistribution, 6-48) */
MMB_HD int mmb_ir_link_kind(int fam) {
  switch (fam) {
    case MMB_IR_INVGAMMA: case MMB_IR_GAMMA: case MMB_IR_EXPONENTIAL: return 1;
    case MMB_IR_BETA: return 2;
    case MMB_IR_UNIFORM: return 3;
    default: return 0;
  }
}
MMB_HD double mmb_ir_link(int kind, double x, double a, double b) {
  if (kind == 1) return mmb_log(x);
  if (kind == 2) return mmb_logit(x);
  if (kind == 3) return mmb_logit((x - a) / (b - a));
  return x;
}
MMB_HD double mmb_ir_invlink(int kind, double x, double a, double b) {
  if (kind == 1) return mmb_exp(x);
  if (kind == 2) return mmb_invlogit(x);
  if (kind == 3) return (b - a) * mmb_invlogit(x) + a;
  return x;
}

/* logpdf_sub(d, x, transform) of one element (distributionstruct.jl:138-140):
 * insupport(d, x) ? logpdf(d, x[, transform]) : -Inf.  (a, b) = the family's parameters in
 * Distributions order; ct = host-computed constant of a discrete observation (log binomial
 * coefficient, -lgamma(k+1)); [lo, hi] = Uniform bounds (constants). */
/* mmb_ir_lp's Normal with log(sigma) supplied (lb = mmb_log(b)): the generated kernels form it
   once for all the elements a lane evaluates when sigma does not depend on the element */
MMB_HD double mmb_ir_normal_lb(double x, double a, double b, double lb) {
  if (x != x) return -__builtin_inf();
  const double z = (x - a) / b;
  return -(z * z + MMB_LOG2PI) / 2.0 - lb;
}

MMB_HD double mmb_ir_lp(int fam, double x, double a, double b, double ct, int tr, double lo, double hi) {
  const double NINF = -__builtin_inf(), INF = __builtin_inf();
  switch (fam) {
    case MMB_IR_NORMAL: { /* normlogpdf(mu, sig, x) */
      if (x != x) return NINF;
      const double z = (x - a) / b;
      return -(z * z + MMB_LOG2PI) / 2.0 - mmb_log(b);
    }
    case MMB_IR_INVGAMMA: { /* a log b - lgamma(a) - (a + 1) log x - b / x */
      if (!(0.0 <= x && x <= INF)) return NINF;
      const double lx = mmb_log(x);
      const double lp = a * mmb_log(b) - mmb_lgamma(a) - (a + 1.0) * lx - b / x;
      return tr ? lp + lx : lp;
    }
    case MMB_IR_GAMMA: { /* -lgamma(k) - k log theta + (k - 1) log x - x / theta */
      if (!(0.0 <= x && x <= INF)) return NINF;
      const double lx = mmb_log(x);
      const double lp = -mmb_lgamma(a) - a * mmb_log(b) + (a - 1.0) * lx - x / b;
      return tr ? lp + lx : lp;
    }
    case MMB_IR_EXPONENTIAL: { /* -log theta - x / theta */
      if (!(0.0 <= x && x <= INF)) return NINF;
      const double lp = -mmb_log(a) - x / a;
      return tr ? lp + mmb_log(x) : lp;
    }
    case MMB_IR_UNIFORM: { /* -log(b - a); Jacobian log((x - a)(b - x)/(b - a)) */
      if (!(lo <= x && x <= hi)) return NINF;
      const double lp = -mmb_log(hi - lo);
      return tr ? lp + mmb_log((x - lo) * (hi - x) / (hi - lo)) : lp;
    }
    case MMB_IR_BETA: { /* (a-1) log x + (b-1) log(1-x) - lbeta(a, b); Jacobian log(x(1-x)) */
      if (!(0.0 <= x && x <= 1.0)) return NINF;
      const double lb = mmb_lgamma(a) + mmb_lgamma(b) - mmb_lgamma(a + b);
      const double lp = (a - 1.0) * mmb_log(x) + (b - 1.0) * mmb_log(1.0 - x) - lb;
      return tr ? lp + mmb_log(x * (1.0 - x)) : lp;
    }
    case MMB_IR_BINOMIAL: { /* lchoose(n, k) + xlogy(k, p) + xlog1py(n - k, -p) */
      const double t1 = x == 0.0 ? 0.0 : x * mmb_log(b);
      const double t2 = (a - x) == 0.0 ? 0.0 : (a - x) * mmb_log1p(-b);
      return ct + t1 + t2;
    }
    case MMB_IR_POISSON: { /* xlogy(k, lambda) - lambda - lgamma(k + 1) */
      const double t1 = x == 0.0 ? 0.0 : x * mmb_log(a);
      return ct + t1 - a;
    }
    case MMB_IR_BERNOULLI: /* x ? log p : log(1 - p) */
      return x == 1.0 ? mmb_log(a) : mmb_log(1.0 - a);
    default:
      return 0.0; /* Logical nodes contribute 0 */
  }
}

#endif /* MMB_IR_MATH_H */
