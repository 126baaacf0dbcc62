"""Node IR on the GPU: the IR sweep kernel through the C ABI
(mmb_create_ir) against the oracle's restatement of the IR on identical Philox streams, and
the reference's published posterior summaries (doc/examples/{seeds,pumps,surgical,dyes,salm,blocker}.rst)
reproduced by many chains.  The kernel sums element terms in lane partials + the 32-lane DPP
butterfly and the oracle mirrors that order, so draws, values and tune are asserted
identical (zero differing bits)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def example(mamba, name, K, seed=5, scheme=None):
    ir = mamba.ir
    rng = np.random.default_rng(seed)
    if name == "seeds":
        m = ir.seeds_model().setinputs(ir.SEEDS)
        m.setsamplers(scheme or [mamba.AMM(["alpha0", "alpha1", "alpha2", "alpha12"], 0.01 * np.eye(4)),
                                 mamba.AMWG("b", 0.01), mamba.AMWG("s2", 0.1)])        # seeds.jl:69-71
        inits = [ir.seeds_inits()[k % 2] for k in range(K)]
    elif name == "pumps":
        m = ir.pumps_model().setinputs(ir.PUMPS)
        m.setsamplers(scheme or [mamba.Slice(["alpha", "beta"], 1.0, mamba.Univariate),
                                 mamba.Slice("theta", 1.0, mamba.Univariate)])      # pumps.jl:52-53
        inits = [{"y": ir.PUMPS["y"], "alpha": 1.0, "beta": 1.0, "theta": rng.gamma(1.0, 1.0, 10)}
                 for _ in range(K)]
    elif name == "surgical":
        m = ir.surgical_model().setinputs(ir.SURGICAL)
        m.setsamplers(scheme or [mamba.NUTS("b"), mamba.Slice(["mu", "s2"], 1.0)])  # surgical.jl:51-52
        inits = [{"r": ir.SURGICAL["r"], "b": [0.1] * 12, "s2": 1.0, "mu": 0.0} if k % 2 == 0 else
                 {"r": ir.SURGICAL["r"], "b": [0.5] * 12, "s2": 10.0, "mu": 1.0} for k in range(K)]
    elif name == "dyes":
        m = ir.dyes_model().setinputs(ir.dyes_inputs())
        m.setsamplers(scheme or [mamba.NUTS(["mu", "theta"]), mamba.Slice(["s2_within", "s2_between"], 1000.0)])
        inits = [{"y": ir.DYES_Y, "theta": 1500, "s2_within": 1, "s2_between": 1, "mu": [1500] * 6} if k % 2 == 0
                 else {"y": ir.DYES_Y, "theta": 3000, "s2_within": 10, "s2_between": 10, "mu": [3000] * 6}
                 for k in range(K)]
    elif name == "salm":
        m = ir.salm_model().setinputs(ir.SALM)
        m.setsamplers(scheme or [mamba.Slice(["alpha", "beta", "gamma"], [1.0, 1.0, 0.1]),
                                 mamba.AMWG(["lam", "s2"], 0.1)])                     # salm.jl:60-61
        inits = [ir.salm_inits()[k % 2] for k in range(K)]
    elif name == "blocker":
        m = ir.blocker_model().setinputs(ir.BLOCKER)
        m.setsamplers(scheme or [mamba.AMWG("mu", 0.1), mamba.AMWG(["delta", "delta_new"], 0.1),
                                 mamba.Slice(["d", "s2"], 1.0)])                      # blocker.jl:77-79
        inits = [ir.blocker_inits()[k % 2] for k in range(K)]
    elif name == "line":
        m = ir.line_model().setinputs(mamba.model.LINE_DATA)
        m.setsamplers(scheme)
        v = mamba.model.line_init_matrix(K, seed=seed)
        inits = [{"y": [1.0, 3, 3, 3, 5], "beta": v[k, :2], "s2": v[k, 2]} for k in range(K)]
    else:
        raise ValueError(name)
    return m, m.init_matrix(inits, K)


def run_both(mamba, oracle, m, V, iters, burnin, thin, seed=11, jit=True):
    eng = mamba.Engine(m)
    # the specialised kernel (ir_jit.cpp, hipRTC; cached by tools/jit_prebuild.py) unless the
    # interpreter was asked for with MMB_IR_JIT=0
    assert eng.ir_jit()[0] == jit, eng.ir_jit()
    eng.init_chains(V, seed=seed)
    dg = eng.run(iters, burnin=burnin, thin=thin)
    st = oracle.new_state(m, V)
    do = oracle.run(m, st, iters, burnin=burnin, thin=thin, seed=seed, nthreads=8)
    return eng, dg, st, do


CASES = {
    "seeds_amm_amwg": ("seeds", None),
    "pumps_slice_uni": ("pumps", None),
    "surgical_nuts_slice": ("surgical", None),
    "dyes_nuts_slice": ("dyes", None),
    "salm_slice_amwg": ("salm", None),
    "blocker_amwg_slice": ("blocker", None),
    "dyes_mala_slice": ("dyes", lambda M: [M.MALA("theta", 50.0), M.MALA("mu", 50.0, np.eye(6)),
                                           M.Slice(["s2_within", "s2_between"], 1000.0)]),   # dyes.jl:61-63
    "dyes_hmc_slice": ("dyes", lambda M: [M.HMC("theta", 10.0, 5), M.HMC("mu", 10.0, 5, np.eye(6)),
                                          M.Slice(["s2_within", "s2_between"], 1000.0)]),    # dyes.jl:65-67
    "line_amwg": ("line", lambda M: [M.AMWG(["beta", "s2"], 1.0)]),
    "line_amm_multislice": ("line", lambda M: [M.AMM("beta", np.eye(2)), M.Slice("s2", 2.0, M.Multivariate)]),
}


@pytest.mark.parametrize("kernel", ["specialised", "interpreter"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_ir_gpu_vs_oracle(mamba, oracle, case, kernel, monkeypatch):
    """Both device forms of the node IR -- the model compiled to straight-line code at
    mmb_create_ir (hipRTC) and the generic interpreter (MMB_IR_JIT=0) -- equal the oracle's
    restatement bit for bit."""
    if kernel == "interpreter":
        monkeypatch.setenv("MMB_IR_JIT", "0")
    name, sch = CASES[case]
    m, V = example(mamba, name, 96, scheme=sch(mamba) if sch else None)
    eng, dg, st, do = run_both(mamba, oracle, m, V, 60, 20, 2, jit=kernel == "specialised")
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])


@pytest.mark.parametrize("name", ["rats", "seeds", "blocker"])
def test_ir_lane_parallel_amwg(mamba, oracle, name, monkeypatch):
    """AMWG blocks whose logpdf! separates by coordinate (engine.cpp ir_sep_table: every element
    term reads at most one coordinate -- rats alpha / beta through the y gather, seeds b, blocker
    delta) decide all coordinates at once in the specialised kernel (ir.h amwg_dm); the draws,
    values and tune equal the one-coordinate-at-a-time loop (MMB_IR_SEP=0), the band-widened mode
    (MMB_AMWG_EXACT=2, many fallbacks) and the oracle bit for bit, and the fallback is rare."""
    if name == "rats":
        m = mamba.ir.rats_model().setinputs(mamba.ir.rats_inputs()).setsamplers(mamba.model.rats_scheme_reference())
        V = m.init_matrix([{**mamba.model.RATS_INITS[k % 2], "y": mamba.model.RATS_Y} for k in range(256)], 256)
        nsep = 2
    else:
        m, V = example(mamba, name, 256)
        nsep = 1 if name == "seeds" else 2  # seeds: b (s2 is one coordinate); blocker: mu, [delta, delta_new]
    out, seq = {}, {}
    for mode in ("sep", "sequential", "wide"):
        monkeypatch.setenv("MMB_IR_SEP", "0" if mode == "sequential" else "1")
        monkeypatch.setenv("MMB_AMWG_EXACT", "2" if mode == "wide" else "0")
        eng = mamba.Engine(m)
        jit, info = eng.ir_jit()
        assert jit, info
        if mode != "sequential":
            assert f"lane-parallel AMWG blocks: {nsep} of" in info, info
        eng.init_chains(V, seed=23)
        d = eng.run(80, burnin=20, thin=2)
        out[mode] = (d, eng.values(), eng.tune())
        seq[mode] = eng.amwg_stats()["sequential_updates"]
    st = oracle.new_state(m, V)
    do = oracle.run(m, st, 80, burnin=20, thin=2, seed=23, nthreads=8)
    for mode in out:
        np.testing.assert_array_equal(out[mode][0], do)
        np.testing.assert_array_equal(out[mode][1], st["values"])
        np.testing.assert_array_equal(out[mode][2], st["tune"][:, :st["tl"]])
    updates = nsep * V.shape[0] * 80
    assert seq["sep"] <= 0.01 * updates, (seq, updates)
    assert seq["wide"] > seq["sep"], seq


def test_ir_rats_reference_scheme_gpu_vs_oracle(mamba, oracle, monkeypatch):
    """rats through the node IR with the reference Slice + AMWG scheme (rats.jl:112-116): the
    specialised kernel, the interpreter and the oracle agree bit for bit."""
    scheme = mamba.model.rats_scheme_reference()
    base = mamba.model.RATS_INITS
    inits = [{**base[k % 2], "y": mamba.model.RATS_Y} for k in range(64)]
    m = mamba.ir.rats_model().setinputs(mamba.ir.rats_inputs()).setsamplers(scheme)
    V = m.init_matrix(inits, 64)
    eng, dg, st, do = run_both(mamba, oracle, m, V, 40, 10, 2)
    np.testing.assert_array_equal(dg, do)
    monkeypatch.setenv("MMB_IR_JIT", "0")
    m2 = mamba.ir.rats_model().setinputs(mamba.ir.rats_inputs()).setsamplers(scheme)
    V2 = m2.init_matrix(inits, 64)
    eng2, dg2, _, _ = run_both(mamba, oracle, m2, V2, 40, 10, 2, jit=False)
    np.testing.assert_array_equal(dg2, dg)


@pytest.mark.parametrize("variant", ["slice_nc4", "logf_call", "slice_exact"])
def test_ir_generator_variants(mamba, oracle, variant, monkeypatch):
    """The specialised kernel's code-generation switches change instruction streams, not draws:
    four Slice candidates per round instead of two (MMB_IR_SLICE_NC=4: four virtual lanes, three
    cross-lane butterfly levels), logf called instead of inlined (MMB_IR_LOGF_INLINE=0), and the
    sequential shrink loop (MMB_SLICE_EXACT=1) -- rats via the IR with the reference scheme equals
    the oracle bit for bit in each (each variant compiles its own kernel on first use)."""
    env = {"slice_nc4": ("MMB_IR_SLICE_NC", "4"), "logf_call": ("MMB_IR_LOGF_INLINE", "0"),
           "slice_exact": ("MMB_SLICE_EXACT", "1")}[variant]
    monkeypatch.setenv(*env)
    inits = [{**mamba.model.RATS_INITS[k % 2], "y": mamba.model.RATS_Y} for k in range(64)]
    m = mamba.ir.rats_model().setinputs(mamba.ir.rats_inputs()).setsamplers(mamba.model.rats_scheme_reference())
    V = m.init_matrix(inits, 64)
    eng, dg, st, do = run_both(mamba, oracle, m, V, 40, 10, 2)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])


@pytest.mark.parametrize("name", ["seeds", "pumps", "surgical", "dyes", "salm", "blocker"])
def test_ir_published_summaries(mamba, name):
    """Posterior means of the reference's example runs reproduced by 2048 chains of the same run
    (iterations, burnin, thin 2 as printed in the .rst; 2 chains there): |ours - published|
    within 5 published MCSE (+ 4 of our own SE)."""
    g = json.load(open(os.path.join(GOLD, "ir_published.json")))[name]
    pub = g["rows"]
    first, last = (int(t) for t in g["iterations"].split(":"))
    m, V = example(mamba, name, 2048, seed=21)
    eng = mamba.Engine(m)
    eng.init_chains(V, seed=2026)
    d = eng.run(last, burnin=first - 2, thin=2)
    for j, nm in enumerate(m.monitor_names):
        if nm not in pub:
            continue
        x = d[:, j, :]
        cm = x.mean(axis=0)
        est, se = float(cm.mean()), float(cm.std(ddof=1) / np.sqrt(cm.size))
        tol = 5.0 * pub[nm]["mcse"] + 4.0 * se
        assert abs(est - pub[nm]["mean"]) < tol, (nm, est, pub[nm]["mean"], tol)
