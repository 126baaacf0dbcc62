"""Independent numpy restatement of the config-3 rats Gibbs + AMM scheme (adapt=:all) at the
rats.rst run length, and the fixture it writes: tests/golden/rats_amm_restatement.json.

Why: with the always-adapting AMM of src/samplers/amm.jl:66-108 the s2_c chain mean over
10000 iterations (burnin 2500, thin 2, doc/examples/rats.rst:37-40) sits well below the
published posterior mean 37.25 -- the proposal covariance is estimated from the chain's own
early, strongly autocorrelated history and grows slowly.  This script fixes
what the reference ALGORITHM gives, so tests/test_gpu_rats_long.py can hold the GPU engine to
it within 5 combined standard errors instead of a wide window.

Shares nothing with oracle/oracle.c or the HIP kernels: numpy RNG, numpy arithmetic, and a
batched non-pivoted Cholesky (the pivot order changes the factor, not the proposal
distribution x = beta SigmaL z1 + (1 - beta) SigmaLm z2 of amm.jl:72-76).  Written from:
  amm.jl:66-94 sample!: x = SigmaL z1; if m > 2n: x = beta x + (1 - beta) SigmaLm z2;
      x += v; accept iff rand() < exp(logf(x) - logf(v)); if adapt: m += 1, p = m/(m+1),
      Mv = p Mv + (1-p) v, Mvv = p Mvv + (1-p) v v', Sigma = scale^2/n/p (Mvv - Mv Mv'),
      SigmaLm = chol(Sigma) when it succeeds (else kept, amm.jl:88-90);
  amm.jl:97-108 setadapt!: m = 0, Mv = v (the variate itself: after the first update Mv is
      the accepted value), Mvv = v v', SigmaLm = 0;
  doc/examples/rats.jl:48-97: y[i,j] ~ Normal(alpha[i] + beta[i] (x[j] - xbar), sqrt(s2_c)),
      alpha[i] ~ Normal(mu_alpha, sqrt(s2_alpha)), beta[i] ~ Normal(mu_beta, sqrt(s2_beta)),
      mu ~ Normal(0, 1000), s2 ~ InverseGamma(0.001, 0.001); alpha0 = mu_alpha - xbar mu_beta;
  scheme (build-defined config 3, mamba.jl_amd/model.py rats_scheme_gibbs_amm): Gibbs s2_c,
      AMM(alpha, I), Gibbs mu_alpha, Gibbs s2_alpha, AMM(beta, 0.01 I), Gibbs mu_beta,
      Gibbs s2_beta, the conjugate full conditionals of INTEGRATION.md §3.
Inits: the first K rows of model.rats_init_ls(16384, seed=1), the inits of the GPU run.

  python tests/golden/make_rats_amm_restatement.py [K] [seed]     (default 4096 chains, seed 7)

writes the per-monitor mean over chains of the kept-draw chain means and its between-chain
standard error (8 worker processes over chain ranges; about 10 minutes at K = 4096 here).
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "rats_amm_restatement.json")
ITERS, BURNIN, THIN = 10000, 2500, 2


def chol_batch(S):
    """Non-pivoted Cholesky of every K x n x n matrix; ok[k] False where a pivot is <= 0."""
    K, n, _ = S.shape
    L = np.zeros_like(S)
    ok = np.ones(K, bool)
    for j in range(n):
        d = S[:, j, j] - np.einsum("ki,ki->k", L[:, j, :j], L[:, j, :j])
        good = d > 0
        ok &= good
        ljj = np.sqrt(np.where(good, d, 1.0))
        L[:, j, j] = ljj
        if j + 1 < n:
            L[:, j + 1:, j] = (S[:, j + 1:, j] - np.einsum("kij,kj->ki", L[:, j + 1:, :j], L[:, j, :j])) / ljj[:, None]
    return L, ok


class AMM:
    """AMMTune + sample! for K chains of one n-dimensional block, adapt=:all."""

    def __init__(self, K, n, sigma_scale, rng):
        self.L = np.sqrt(sigma_scale) * np.eye(n)
        self.rng = rng
        self.m = 0
        self.Mv = self.Mvv = None
        self.Lm = np.zeros((K, n, n))

    def step(self, v, logf):
        rng, n = self.rng, v.shape[1]
        if self.Mv is None:                                   # setadapt! at the first update
            self.m, self.Mvv = 0, v[:, :, None] * v[:, None, :]
        x = rng.standard_normal(v.shape) @ self.L.T
        if self.m > 2 * n:
            x = 0.05 * x + 0.95 * np.einsum("kij,kj->ki", self.Lm, rng.standard_normal(v.shape))
        x = x + v
        acc = rng.random(v.shape[0]) < np.exp(logf(x) - logf(v))
        v = np.where(acc[:, None], x, v)
        self.m += 1
        p = self.m / (self.m + 1.0)
        self.Mv = v.copy() if self.Mv is None else p * self.Mv + (1 - p) * v   # Mv = v alias (amm.jl:102)
        self.Mvv = p * self.Mvv + (1 - p) * v[:, :, None] * v[:, None, :]
        # (Mvv and Mv Mv' are exactly symmetric here; chol_batch reads the lower triangle)
        S = (2.38 ** 2 / n / p) * (self.Mvv - self.Mv[:, :, None] * self.Mv[:, None, :])
        Lm, ok = chol_batch(S)
        self.Lm[ok] = Lm[ok]                                  # rank(F) < n: SigmaLm kept
        return v


def run(args):
    """Chains [lo, hi) of the inits, numpy stream (seed, lo): returns their kept-draw sums."""
    lo, hi, seed = args
    sys.path.insert(0, ROOT)
    import _mamba_path
    mb = _mamba_path.load()
    Y = np.asarray(mb.model.RATS_Y, float).reshape(30, 5)
    Xm = np.asarray([8.0, 15.0, 22.0, 29.0, 36.0]) - 22.0
    init = mb.model.rats_init_ls(16384, seed=1)[lo:hi]
    K = hi - lo
    al, be = init[:, 1:31].copy(), init[:, 33:63].copy()
    mua, s2a, mub, s2b = init[:, 31].copy(), init[:, 32].copy(), init[:, 63].copy(), init[:, 64].copy()
    rng = np.random.default_rng([seed, lo])

    def inv_gamma(shape, scale):                              # InverseGamma(shape, scale) draws
        return scale / rng.gamma(shape, 1.0, size=scale.shape)

    def resid(a, b):
        return Y[None] - a[:, :, None] - b[:, :, None] * Xm[None, None]

    A1, A2 = AMM(K, 30, 1.0, rng), AMM(K, 30, 0.01, rng)
    sums = np.zeros((K, 3))
    nk, t0 = 0, time.time()
    for it in range(1, ITERS + 1):
        r = resid(al, be)
        s2c = inv_gamma(0.001 + 75, 0.001 + (r * r).sum((1, 2)) / 2)
        al = A1.step(al, lambda x: -0.5 * ((x - mua[:, None]) ** 2).sum(1) / s2a
                     - 0.5 * (resid(x, be) ** 2).sum((1, 2)) / s2c)
        prec = 30 / s2a + 1e-6
        mua = rng.normal(al.sum(1) / s2a / prec, 1 / np.sqrt(prec))
        s2a = inv_gamma(0.001 + 15, 0.001 + ((al - mua[:, None]) ** 2).sum(1) / 2)
        be = A2.step(be, lambda x: -0.5 * ((x - mub[:, None]) ** 2).sum(1) / s2b
                     - 0.5 * (resid(al, x) ** 2).sum((1, 2)) / s2c)
        prec = 30 / s2b + 1e-6
        mub = rng.normal(be.sum(1) / s2b / prec, 1 / np.sqrt(prec))
        s2b = inv_gamma(0.001 + 15, 0.001 + ((be - mub[:, None]) ** 2).sum(1) / 2)
        if it > BURNIN and (it - BURNIN) % THIN == 0:         # mcmc.jl:76 keep rule
            sums += np.stack([s2c, mub, mua - 22.0 * mub], axis=1)
            nk += 1
        if it % 1000 == 0 and lo == 0:
            print(f"iter {it} {time.time() - t0:.0f}s", flush=True)
    return sums / nk, nk


def main():
    from multiprocessing import Pool
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    W = min(8, os.cpu_count() or 1)
    cut = [K * w // W for w in range(W + 1)]
    with Pool(W) as pool:
        parts = pool.map(run, [(cut[w], cut[w + 1], seed) for w in range(W)])
    cm = np.concatenate([c for c, _ in parts])
    nk = parts[0][1]
    out = {"what": "config-3 rats Gibbs+AMM (adapt=:all), numpy restatement of amm.jl:66-108",
           "generator": "tests/golden/make_rats_amm_restatement.py", "chains": K, "seed": seed,
           "inits": "model.rats_init_ls(16384, seed=1)[:chains]", "iters": ITERS, "burnin": BURNIN,
           "thin": THIN, "kept": nk, "names": ["s2_c", "mu_beta", "alpha0"],
           "mean": [float(x) for x in cm.mean(0)], "se": [float(x) for x in cm.std(0) / np.sqrt(K)]}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
