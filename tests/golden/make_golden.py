"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root in the build container (needs hipcc for the rocRAND probe and
read access to /root/reference for the CODA data files):

    python tests/golden/make_golden.py

Fixtures (all small JSON, committed):
  philox_kat.json   Philox4x32-10 outputs from rocRAND's header (philox_probe.cpp), plus the
                    three Random123 known-answer vectors (kat_vectors, philox4x32 10).
  logpdf.json       block log densities at fixed states, computed independently with
                    scipy.stats (Normal, InverseGamma, iid Normal == IsoNormal, Bernoulli),
                    following the node/target structure of logpdf! (simulation.jl:77-90).
  coda_line.json    the reference's own CODA fixture doc/mcmc/line{1,2}.{out,ind} (OpenBUGS
                    output, 200 iters x {alpha, beta, sigma} x 2 chains) and its
                    Gelman-Rubin PSRF computed by a numpy restatement of gelmandiag.jl.
  line_posterior.json  exact posterior moments/quantiles of the line model by quadrature
                    (beta grid x analytic s2 marginal); statistical target for the samplers.
  rats_published.json  summaries printed in doc/examples/rats.rst:37-52 (10k iters,
                    burnin 2500, thin 2, 2 chains, the reference Slice+AMWG scheme).
  ir_published.json  "Empirical Posterior Estimates" (Mean, SD, MCSE) printed in
                    doc/examples/{seeds,pumps,surgical,dyes,salm,blocker}.rst for the node-IR examples.
"""
import json
import os
import subprocess
import sys

import numpy as np
from scipy import stats
from scipy.special import gammaln

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

LINE_X = np.array([1.0, 2, 3, 4, 5])
LINE_Y = np.array([1.0, 3, 3, 3, 5])
RATS_Y = np.array([
    151, 199, 246, 283, 320, 145, 199, 249, 293, 354, 147, 214, 263, 312, 328,
    155, 200, 237, 272, 297, 135, 188, 230, 280, 323, 159, 210, 252, 298, 331,
    141, 189, 231, 275, 305, 159, 201, 248, 297, 338, 177, 236, 285, 350, 376,
    134, 182, 220, 260, 296, 160, 208, 261, 313, 352, 143, 188, 220, 273, 314,
    154, 200, 244, 289, 325, 171, 221, 270, 326, 358, 163, 216, 242, 281, 312,
    160, 207, 248, 288, 324, 142, 187, 234, 280, 316, 156, 203, 243, 283, 317,
    157, 212, 259, 307, 336, 152, 203, 246, 286, 321, 154, 205, 253, 298, 334,
    139, 190, 225, 267, 302, 146, 191, 229, 272, 302, 157, 211, 250, 285, 323,
    132, 185, 237, 286, 331, 160, 207, 257, 303, 345, 169, 216, 261, 295, 333,
    157, 205, 248, 289, 316, 137, 180, 219, 258, 291, 153, 200, 244, 286, 324], dtype=float)
RATS_X = np.array([8.0, 15.0, 22.0, 29.0, 36.0])


def ir_published():
    """Mean / SD / MCSE columns of the first summary table of each example's .rst."""
    out = {}
    for ex in ("seeds", "pumps", "surgical", "dyes", "salm", "blocker"):
        lines = open(os.path.join(REF, "doc", "examples", ex + ".rst")).read().splitlines()
        i = next(k for k, ln in enumerate(lines) if "Empirical Posterior Estimates" in ln) + 2
        rows = {}
        while i < len(lines) and lines[i].strip():
            f = lines[i].split()
            rows[f[0]] = {"mean": float(f[1]), "sd": float(f[2]), "mcse": float(f[4])}
            i += 1
        it = next(ln for ln in lines if "Iterations =" in ln).split("=")[1].strip()
        out[ex] = {"iterations": it, "rows": rows}
    return out


def philox():
    exe = "/tmp/mmb_philox_probe"
    subprocess.check_call(["hipcc", "-O1", "--offload-arch=gfx950", "-o", exe,
                           os.path.join(HERE, "philox_probe.cpp")])
    rocrand = json.loads(subprocess.check_output([exe]).decode())
    random123 = [  # Random123 kat_vectors "philox4x32 10 ..."
        {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]},
        {"ctr": [0xffffffff] * 4, "key": [0xffffffff] * 2,
         "out": [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]},
        {"ctr": [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], "key": [0xa4093822, 0x299f31d0],
         "out": [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]},
    ]
    return {"rocrand": rocrand, "random123": random123}


def ig_lp(x, a=0.001, b=0.001):
    return stats.invgamma.logpdf(x, a, scale=b)


def line_block(vals, block, x):
    """line model, doc/tutorial/line.jl.  vals=[b1,b2,s2]; x = unlisted block vector."""
    v = np.array(vals, float)
    if block == "beta_s2":          # AMWG/AMM([:beta, :s2]) transform=true
        v[:2] = x[:2]; v[2] = np.exp(x[2])
        jac = x[2]                  # log |d s2 / d log s2|
        lp = stats.multivariate_normal.logpdf(v[:2], np.zeros(2), 1000.0 * np.eye(2)) + ig_lp(v[2]) + jac
    elif block == "beta":           # NUTS(:beta)
        v[:2] = x
        lp = stats.multivariate_normal.logpdf(v[:2], np.zeros(2), 1000.0 * np.eye(2))
    elif block == "s2":             # Slice(:s2, 3.0) transform=false
        v[2] = x[0]
        if v[2] <= 0:
            return -np.inf
        lp = ig_lp(v[2])
    mu = v[0] + LINE_X * v[1]
    return float(lp + stats.norm.logpdf(LINE_Y, mu, np.sqrt(v[2])).sum())


def rats_block(vals, block, x):
    """rats model, doc/examples/rats.jl:48-97.  canonical vals (65)."""
    v = np.array(vals, float)
    xm = RATS_X - RATS_X.mean()
    s2c, al, mua, s2a, be, mub, s2b = v[0], v[1:31], v[31], v[32], v[33:63], v[63], v[64]

    def ylp(al, be, s2c):
        mu = np.repeat(al, 5) + np.repeat(be, 5) * np.tile(xm, 30)
        return stats.norm.logpdf(RATS_Y, mu, np.sqrt(s2c)).sum()

    if block == "s2_c":
        s2c = x[0]
        if s2c <= 0:
            return -np.inf
        return float(ig_lp(s2c) + ylp(al, be, s2c))
    if block == "alpha":
        al = np.array(x)
        return float(stats.norm.logpdf(al, mua, np.sqrt(s2a)).sum() + ylp(al, be, s2c))
    if block == "beta":
        be = np.array(x)
        return float(stats.norm.logpdf(be, mub, np.sqrt(s2b)).sum() + ylp(al, be, s2c))
    if block == "mu_s2_alpha":
        mua, s2a = x
        if s2a <= 0:
            return -np.inf
        return float(stats.norm.logpdf(mua, 0, 1000) + ig_lp(s2a) + stats.norm.logpdf(al, mua, np.sqrt(s2a)).sum())
    if block == "mu_s2_beta":
        mub, s2b = x
        if s2b <= 0:
            return -np.inf
        return float(stats.norm.logpdf(mub, 0, 1000) + ig_lp(s2b) + stats.norm.logpdf(be, mub, np.sqrt(s2b)).sum())
    raise ValueError(block)


def logistic_lp(X, y, beta, sd):
    eta = X @ beta
    return float(stats.bernoulli.logpmf(y, 1 / (1 + np.exp(-eta))).sum()
                 + stats.norm.logpdf(beta, 0, sd).sum())


def logistic_grad(X, y, beta, sd):
    eta = X @ beta
    return (X.T @ (y - 1 / (1 + np.exp(-eta))) - beta / sd**2).tolist()


def logpdf_cases():
    rng = np.random.default_rng(20261015)
    out = {"line": [], "rats": [], "logistic": []}
    for _ in range(6):
        vals = [rng.normal(0.5, 1), rng.normal(0.8, 0.3), rng.gamma(2, 0.7)]
        x = [vals[0], vals[1], np.log(vals[2])]
        out["line"].append({"vals": vals, "block": "beta_s2", "x": x, "lp": line_block(vals, "beta_s2", x)})
        out["line"].append({"vals": vals, "block": "beta", "x": vals[:2], "lp": line_block(vals, "beta", vals[:2])})
        s = [vals[2] if _ % 3 else -0.5]
        out["line"].append({"vals": vals, "block": "s2", "x": s, "lp": line_block(vals, "s2", s)})
    for _ in range(5):
        al = rng.normal(240, 10, 30)
        be = rng.normal(6, 0.3, 30)
        vals = np.concatenate([[rng.gamma(30, 1.2)], al, [rng.normal(240, 5), rng.gamma(20, 6)], be,
                               [rng.normal(6.2, 0.2), rng.gamma(5, 0.06)]]).tolist()
        for block, x in [("s2_c", [vals[0]]), ("alpha", vals[1:31]), ("beta", vals[33:63]),
                         ("mu_s2_alpha", [vals[31], vals[32]]), ("mu_s2_beta", [vals[63], vals[64]]),
                         ("mu_s2_alpha", [vals[31], -3.0])]:
            out["rats"].append({"vals": vals, "block": block, "x": list(map(float, x)),
                                "lp": rats_block(vals, block, x)})
    N, p, sd = 64, 5, 10.0
    X = rng.normal(0, 1, (N, p))
    bt = rng.normal(0, 0.5, p)
    y = (rng.random(N) < 1 / (1 + np.exp(-X @ bt))).astype(float)
    for _ in range(4):
        b = rng.normal(0, 0.7, p)
        out["logistic"].append({"beta": b.tolist(), "lp": logistic_lp(X, y, b, sd),
                                "grad": logistic_grad(X, y, b, sd)})
    out["logistic_data"] = {"N": N, "p": p, "sd": sd, "X": X.ravel().tolist(), "y": y.tolist()}
    # line NUTS gradients (analytic, block [beta] and [beta, s2] with log s2)
    grads = []
    for _ in range(4):
        b = rng.normal(0.5, 1, 2); s2 = rng.gamma(2, 0.7)
        r = LINE_Y - (b[0] + LINE_X * b[1])
        g_beta = [r.sum() / s2 - b[0] / 1000, (LINE_X * r).sum() / s2 - b[1] / 1000]
        g_ls2 = -(0.001 + 2.5) + (0.5 * (r @ r) + 0.001) / s2
        grads.append({"vals": [b[0], b[1], s2], "grad_beta": g_beta, "grad_ls2": g_ls2})
    out["line_grad"] = grads
    return out


# ---- Gelman-Rubin: numpy restatement of src/output/gelmandiag.jl:3-60 -------------
def gelmandiag_np(psi, alpha=0.05, mpsrf=False):
    n, p, m = psi.shape
    S2 = np.stack([np.cov(psi[:, :, k], rowvar=False).reshape(p, p) for k in range(m)], 2)
    W = S2.mean(2)
    psibar = psi.mean(0).T                      # m x p
    B = n * np.atleast_2d(np.cov(psibar, rowvar=False))
    w = np.diag(W); b = np.diag(B)
    s2 = np.stack([np.diag(S2[:, :, k]) for k in range(m)])  # m x p
    psibar2 = psibar.mean(0)
    var_w = s2.var(0, ddof=1) / m
    var_b = (2.0 / (m - 1)) * b**2

    def cov2(a, c):
        return ((a - a.mean(0)) * (c - c.mean(0))).sum(0) / (m - 1)
    var_wb = (n / m) * (cov2(s2, psibar**2) - 2.0 * psibar2 * cov2(s2, psibar))
    V = ((n - 1) / n) * w + ((m + 1) / (m * n)) * b
    var_V = ((n - 1)**2 * var_w + ((m + 1) / m)**2 * var_b + (2.0 * (n - 1) * (m + 1) / m) * var_wb) / n**2
    df = 2.0 * V**2 / var_V
    B_df = m - 1
    W_df = 2.0 * w**2 / var_w
    psrf = np.empty((p, 2))
    R_fixed = (n - 1) / n
    R_random_scale = (m + 1) / (m * n)
    q = 1.0 - alpha / 2.0
    for i in range(p):
        corr = (df[i] + 3.0) / (df[i] + 1.0)
        R_random = R_random_scale * b[i] / w[i]
        psrf[i, 0] = np.sqrt(corr * (R_fixed + R_random))
        if not np.isnan(R_random):
            R_random *= stats.f.ppf(q, B_df, W_df[i])
        psrf[i, 1] = np.sqrt(corr * (R_fixed + R_random))
    mp = None
    if mpsrf:
        try:
            np.linalg.cholesky(W)
            mp = R_fixed + R_random_scale * np.max(np.real(np.linalg.eigvals(np.linalg.solve(W, B))))
        except np.linalg.LinAlgError:
            mp = float("nan")
    return psrf, mp


def coda():
    def read(chain):
        ind = [l.split() for l in open(f"{REF}/doc/mcmc/line{chain}.ind") if l.strip()]
        out = np.loadtxt(f"{REF}/doc/mcmc/line{chain}.out")
        cols = []
        for name, a, b in ind:
            cols.append(out[int(a) - 1:int(b), 1])
        return [x[0] for x in ind], np.stack(cols, 1)
    names, c1 = read(1)
    _, c2 = read(2)
    psi = np.stack([c1, c2], 2)
    psrf, mp = gelmandiag_np(psi, mpsrf=True)
    # link() transform (chains.jl:237-246): log for positive columns
    psil = psi.copy()
    for j in range(psi.shape[1]):
        x = psi[:, j, :]
        if x.min() > 0:
            psil[:, j, :] = np.log(x / (1 - x)) if x.max() < 1 else np.log(x)
    psrf_t, mp_t = gelmandiag_np(psil, mpsrf=True)
    return {"names": names, "chains": [c1.tolist(), c2.tolist()],
            "psrf": psrf.tolist(), "mpsrf": mp, "psrf_transform": psrf_t.tolist(), "mpsrf_transform": mp_t}


def line_posterior():
    """p(b, s2 | y) ∝ N2(b; 0, 1000 I) IG(s2; 0.001, 0.001) N(y; Xb, s2 I).
    Integrate s2 analytically: p(b|y) ∝ N2(b) * (0.001 + SSR(b)/2)^-(0.001 + 2.5)."""
    b1 = np.linspace(-25, 25, 2001)
    b2 = np.linspace(-8, 9, 1201)
    B1, B2 = np.meshgrid(b1, b2, indexing="ij")
    ssr = sum((LINE_Y[i] - B1 - B2 * LINE_X[i])**2 for i in range(5))
    a = 0.001 + 2.5
    bb = 0.001 + ssr / 2
    lw = -(B1**2 + B2**2) / 2000 - a * np.log(bb)
    w = np.exp(lw - lw.max()); w /= w.sum()
    Eb1 = (w * B1).sum(); Eb2 = (w * B2).sum()
    sd1 = np.sqrt((w * (B1 - Eb1)**2).sum()); sd2 = np.sqrt((w * (B2 - Eb2)**2).sum())
    Es2 = (w * bb / (a - 1)).sum()                       # E[s2 | b] = b/(a-1)
    # s2 quantiles by mixture CDF on a grid
    s2g = np.exp(np.linspace(np.log(0.02), np.log(500), 3000))
    wf, bf = w.ravel(), bb.ravel()
    keep = wf > 1e-12
    cdf = np.array([(wf[keep] * stats.invgamma.cdf(s, a, scale=bf[keep])).sum() for s in s2g])
    qs = {str(q): float(np.interp(q, cdf, s2g)) for q in (0.025, 0.25, 0.5, 0.75, 0.975)}
    return {"E_beta1": Eb1, "E_beta2": Eb2, "sd_beta1": sd1, "sd_beta2": sd2, "E_s2": Es2,
            "s2_quantiles": qs}


def rats_published():
    return {"source": "doc/examples/rats.rst:37-52",
            "iters": 10000, "burnin": 2500, "thin": 2, "chains": 2,
            "mean": {"s2_c": 37.2543133, "mu_beta": 6.1830663, "alpha0": 106.6259925},
            "sd": {"s2_c": 6.026634572, "mu_beta": 0.108042927, "alpha0": 3.459210115},
            "mcse": {"s2_c": 0.2337982327, "mu_beta": 0.0017921615, "alpha0": 0.0526804390},
            "q": {"s2_c": [27.778388, 33.0906026, 36.4630047, 40.5538472, 51.5713716],
                  "mu_beta": [5.969850, 6.1110307, 6.1836454, 6.2538831, 6.3964953],
                  "alpha0": [99.815707, 104.3369878, 106.6105679, 108.9124224, 113.5045347]}}


def main():
    def dump(name, obj):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1, default=float)
        print("wrote", name)
    dump("philox_kat.json", philox())
    dump("logpdf.json", logpdf_cases())
    dump("coda_line.json", coda())
    dump("line_posterior.json", line_posterior())
    dump("rats_published.json", rats_published())
    dump("ir_published.json", ir_published())


if __name__ == "__main__":
    sys.exit(main())
