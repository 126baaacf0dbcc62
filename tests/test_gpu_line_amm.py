"""BASELINE configs[1] (line regression, one AMM block, 4096 chains) on the four-lanes-per-chain
kernel (csrc/line_amm.hip) against the generic one-lane sweep kernel (MMB_LINE_GENERIC=1)
and the CPU oracle.  The quad kernel replicates the generic kernel's arithmetic (only the
Philox blocks and the two logpdf evaluations are split over lanes; the tune state lives in
registers for a launch), so draws, chain values and tune state must be BIT-EXACT
against both, at the configuration's full 4096 chains and across launch / window splits
(amm.jl:66-108, mcmc.jl:62-83)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCHEMES = {
    "amm": lambda M: [M.AMM(["beta", "s2"], np.eye(3))],
    "amm_dense": lambda M: [M.AMM(["beta", "s2"], np.array([[1.0, 0.3, 0.0], [0.3, 0.5, 0.1], [0.0, 0.1, 2.0]]))],
    "amm_s2_beta": lambda M: [M.AMM(["s2", "beta"], 0.5 * np.eye(3), beta=0.2, scale=1.5)],
    "amm_burnin": lambda M: [M.AMM(["beta", "s2"], np.eye(3), adapt="burnin")],
    "amm_beta_only": lambda M: [M.AMM("beta", np.array([[2.0, 0.1], [0.1, 0.4]]))],
    "amm_s2_only": lambda M: [M.AMM("s2", np.eye(1))],
}


def _model(mamba, name):
    m = mamba.line()
    m.setinputs(mamba.model.LINE_DATA)
    return m.setsamplers(SCHEMES[name](mamba))


def _run(mamba, m, init, windows, seed=5, generic=False, model_burnin=None):
    """windows: list of (iters, burnin, thin) run back to back on one engine."""
    if generic:
        os.environ["MMB_LINE_GENERIC"] = "1"
    try:
        eng = mamba.Engine(m)
        eng.init_chains(init, seed=seed)
        out = [eng.run(n, burnin=b, thin=t, model_burnin=model_burnin) for n, b, t in windows]
        return out, eng.values(), eng.tune()
    finally:
        os.environ.pop("MMB_LINE_GENERIC", None)


@pytest.mark.parametrize("name", sorted(SCHEMES))
def test_line_amm_quad_vs_generic_4096(mamba, name, monkeypatch):
    """Full configs[1] size; 300 iterations at 64 per launch = 4 launches + a ragged one (the
    default is 256 per launch); adaptive switch at m > 2d."""
    monkeypatch.setenv("MMB_ITERS_PER_LAUNCH", "64")
    m = _model(mamba, name)
    init = mamba.model.line_init_matrix(4096, seed=11)
    fq, vq, tq = _run(mamba, m, init, [(300, 100, 2)], model_burnin=150)
    fg, vg, tg = _run(mamba, m, init, [(300, 100, 2)], generic=True, model_burnin=150)
    np.testing.assert_array_equal(fq[0], fg[0])
    np.testing.assert_array_equal(vq, vg)
    np.testing.assert_array_equal(tq, tg)
    assert np.isfinite(fq[0]).all() and fq[0].shape == (100, 3, 4096)


@pytest.mark.parametrize("name", ["amm", "amm_burnin", "amm_s2_only"])
def test_line_amm_quad_vs_oracle_4096(mamba, oracle, name):
    m = _model(mamba, name)
    init = mamba.model.line_init_matrix(4096, seed=12)
    eng = mamba.Engine(m)
    eng.init_chains(init, seed=19)
    dg = eng.run(200, burnin=50, thin=3, model_burnin=120)
    st = oracle.new_state(m, init)
    do = oracle.run(m, st, 200, burnin=50, thin=3, seed=19, model_burnin=120, nthreads=8)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])


def test_line_amm_quad_window_splits(mamba, monkeypatch):
    """Register-resident tune state is written back at every launch end: windows of 1, 63, 65
    and 71 iterations at 16 iterations per launch (launch boundaries inside and across windows)
    equal one 200-iteration run at the default 256 per launch (a single ragged launch), and a
    host round trip of values + tune (set_values / set_tune) in between changes nothing."""
    m = _model(mamba, "amm")
    init = mamba.model.line_init_matrix(4096, seed=13)
    full, vf, tf = _run(mamba, m, init, [(200, 0, 1)])
    monkeypatch.setenv("MMB_ITERS_PER_LAUNCH", "16")
    eng = mamba.Engine(m)
    eng.init_chains(init, seed=5)
    parts = [eng.run(1), eng.run(63), eng.run(65)]
    eng.set_values(eng.values())
    eng.set_tune(eng.tune())
    parts.append(eng.run(71))
    np.testing.assert_array_equal(np.concatenate(parts, axis=0), full[0])
    np.testing.assert_array_equal(eng.values(), vf)
    np.testing.assert_array_equal(eng.tune(), tf)
