"""Config 3 at the rats.rst run length on the GPU (doc/examples/rats.rst:37-52: 10000
iterations, burnin 2500, thin 2), 16384 chains per scheme, against the published summaries
(tests/golden/rats_published.json).  Chain means come from the on-device per-chain sums
(mmb_chain_summary), so the 2 GB of kept draws never leave HBM; our standard error is the
between-chain SD of those means / sqrt(K).

* reference scheme Slice + AMWG (rats.jl:112-116) and the Gibbs + AMM scheme with the AMM
  blocks frozen (adapt=:none): s2_c, mu_beta, alpha0 within 5 combined MCSE of the
  published means;
* Gibbs + AMM with adapt=:all (the headline workload): mu_beta and alpha0 within 5 MCSE of
  the published means; s2_c is biased LOW.  That is a property of the reference algorithm,
  not of this engine: setadapt! aliases tune.Mv to the variate (amm.jl:102, `tune.Mv = v`), so
  in every chain whose first adaptive proposal was accepted Mvv - Mv Mv' starts as
  (v0 v0' - v1 v1') / 2, indefinite at the scale |v| |v1 - v0|, and the running averages shrink
  it only like 2 / (m + 1); dpstf2 then stops after a few pivots every update and SigmaLm stays
  at setadapt!'s zeros (amm.jl:88-90, 104), so about half the alpha chains (a third of the beta
  chains) propose 0.05 SigmaL z1 only -- steps far below the posterior sd -- and hug their
  per-rat fits, which biases s2_c low (the mechanism is pinned on the oracle by
  tests/test_oracle.py::test_rats_amm_alias_leaves_first_accepted_chains_without_factor).
  tests/golden/make_rats_amm_restatement.py, an independent numpy restatement (numpy RNG,
  batched plain Cholesky of the same Sigma, the same alias), run on the same inits and
  schedule (rats_init_ls(16384, seed=1)[:4096], 10000 / 2500 / 2) gives
  tests/golden/rats_amm_restatement.json; all three GPU means must lie within 5 combined
  standard errors of it."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PUB = json.load(open(os.path.join(HERE, "golden", "rats_published.json")))
RESTATED = json.load(open(os.path.join(HERE, "golden", "rats_amm_restatement.json")))
NAMES = ["s2_c", "mu_beta", "alpha0"]


def run(mamba, scheme, K=16384, iters=10000, burnin=2500, thin=2, seed=20261016):
    m = mamba.rats()
    m.setinputs(mamba.model.RATS_DATA)
    m.setsamplers(scheme)
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.rats_init_ls(K, seed=1), seed=seed)
    eng.run(iters, burnin=burnin, thin=thin, keep_device=True)
    n = eng.num_kept()
    assert n == (iters - burnin) // thin
    shift = np.array([PUB["mean"][k] for k in NAMES])
    s1 = eng.chain_summary(shift, 100, 0)[:, :, 0]          # F_S1: per-chain shifted sums
    cm = shift + s1 / n                                       # K x 3 chain means
    eng.close()
    assert np.isfinite(cm).all()
    return cm.mean(0), cm.std(0) / np.sqrt(K)


def _within(mean, se, names, nsig=5.0):
    for j, k in enumerate(NAMES):
        if k not in names:
            continue
        tol = nsig * np.hypot(PUB["mcse"][k], se[j])
        assert abs(mean[j] - PUB["mean"][k]) < tol, (k, mean[j], PUB["mean"][k], tol)


@pytest.mark.parametrize("scheme", ["reference", "gibbs_amm_frozen"])
def test_rats_published_summaries(mamba, scheme):
    if scheme == "reference":
        sch = mamba.model.rats_scheme_reference()
    else:
        G = mamba.Gibbs
        sch = [G("s2_c"), mamba.AMM("alpha", np.eye(30), adapt="none"), G("mu_alpha"), G("s2_alpha"),
               mamba.AMM("beta", 0.01 * np.eye(30), adapt="none"), G("mu_beta"), G("s2_beta")]
    mean, se = run(mamba, sch)
    _within(mean, se, NAMES)


def test_rats_gibbs_amm_adaptive(mamba):
    mean, se = run(mamba, mamba.model.rats_scheme_gibbs_amm())
    _within(mean, se, ["mu_beta", "alpha0"])
    # the adaptive-AMM s2_c deficit (published 37.25, MCSE 0.23) against the numpy restatement
    # of the reference algorithm on the same inits and schedule (34.53, SE 0.04)
    assert RESTATED["names"] == NAMES and RESTATED["iters"] == 10000 and RESTATED["burnin"] == 2500
    for j, k in enumerate(NAMES):
        tol = 5.0 * np.hypot(RESTATED["se"][j], se[j])
        assert abs(mean[j] - RESTATED["mean"][j]) < tol, (k, mean[j], RESTATED["mean"][j], tol)
