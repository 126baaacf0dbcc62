"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle on identical
Philox streams.  line (one chain per lane) and rats (32 lanes per chain: the oracle restates
the kernel's lane partials and 32-lane butterfly, oracle.c rats_ssr / bfly) are required to be
BIT-EXACT: draws, values and every tune field."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def line(mamba, scheme):
    m = mamba.line()
    m.setinputs(mamba.model.LINE_DATA)
    return m.setsamplers(scheme)


def rats(mamba, scheme):
    m = mamba.rats()
    m.setinputs(mamba.model.RATS_DATA)
    return m.setsamplers(scheme)


def both(mamba, oracle, m, init, iters, burnin, thin, seed=17, offset=0, model_burnin=None):
    eng = mamba.Engine(m)
    eng.init_chains(init, chain_offset=offset, seed=seed)
    dg = eng.run(iters, burnin=burnin, thin=thin, model_burnin=model_burnin)
    st = oracle.new_state(m, init)
    do = oracle.run(m, st, iters, burnin=burnin, thin=thin, seed=seed, chain_offset=offset,
                    model_burnin=model_burnin, nthreads=8)
    return eng, dg, st, do


LINE_SCHEMES = {
    "amwg": lambda M: [M.AMWG(["beta", "s2"], 1.0)],
    "amwg_burnin": lambda M: [M.AMWG(["beta", "s2"], [0.5, 0.2, 1.0], adapt="burnin", batchsize=20)],
    "amm": lambda M: [M.AMM(["beta", "s2"], np.eye(3))],
    "amm_dense": lambda M: [M.AMM(["beta", "s2"], np.array([[1.0, 0.3, 0.0], [0.3, 0.5, 0.1], [0.0, 0.1, 2.0]]))],
    "slice_uni": lambda M: [M.Slice(["beta", "s2"], [3.0, 1.0, 2.0], M.Univariate)],
    "slice_multi": lambda M: [M.Slice(["beta", "s2"], 2.0)],
    "gibbs": lambda M: [M.Gibbs("beta"), M.Gibbs("s2")],
    "amwg_slice": lambda M: [M.AMWG("beta", 1.0), M.Slice("s2", 3.0, transform=True)],
    "nuts": lambda M: [M.NUTS(["beta", "s2"])],
    "nuts_slice": lambda M: [M.NUTS("beta"), M.Slice("s2", 3.0)],        # doc/tutorial/line.jl:49-50
    "hmc": lambda M: [M.HMC(["beta", "s2"], 0.05, 8)],
    "hmc_sigma_slice": lambda M: [M.HMC("beta", 0.1, 5, np.array([[1.6, -0.45], [-0.45, 0.15]])),
                                  M.Slice("s2", 3.0)],
    "hmc_l0": lambda M: [M.HMC(["beta", "s2"], 0.05, 0)],
    "mala": lambda M: [M.MALA(["beta", "s2"], 0.01)],
    "mala_sigma_gibbs": lambda M: [M.MALA("beta", 0.3, np.array([[1.6, -0.45], [-0.45, 0.15]])),
                                   M.Gibbs("s2")],
    # the reference's default gradient is Calculus :forward differences (the schemes above);
    # dtype="analytic" selects the hand-derived one
    "nuts_analytic": lambda M: [M.NUTS(["beta", "s2"], dtype="analytic")],
    "hmc_analytic": lambda M: [M.HMC(["beta", "s2"], 0.05, 8, dtype="analytic")],
    "mala_analytic_gibbs": lambda M: [M.MALA("beta", 0.3, dtype="analytic"), M.Gibbs("s2")],
    # analytic gradients on blocks in non-canonical order / holding s2 alone (through emap)
    "nuts_analytic_s2_beta": lambda M: [M.NUTS(["s2", "beta"], dtype="analytic")],
    "nuts_analytic_s2_only": lambda M: [M.Gibbs("beta"), M.NUTS("s2", dtype="analytic")],
    "hmc_analytic_s2_beta": lambda M: [M.HMC(["s2", "beta"], 0.05, 6, dtype="analytic")],
}


@pytest.mark.parametrize("name", sorted(LINE_SCHEMES))
def test_line_bit_exact(mamba, oracle, name):
    m = line(mamba, LINE_SCHEMES[name](mamba))
    init = mamba.model.line_init_matrix(512, seed=4)
    eng, dg, st, do = both(mamba, oracle, m, init, 400, 100, 2, model_burnin=150)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])


RATS_SCHEMES = {
    "reference": lambda M: M.model.rats_scheme_reference(),
    "gibbs_amm": lambda M: M.model.rats_scheme_gibbs_amm(),
}


@pytest.mark.parametrize("name", sorted(RATS_SCHEMES))
def test_rats_parity(mamba, oracle, name):
    m = rats(mamba, RATS_SCHEMES[name](mamba))
    init = mamba.model.rats_init_ls(256, seed=2) if name == "gibbs_amm" else mamba.model.rats_init_matrix(256)
    eng, dg, st, do = both(mamba, oracle, m, init, 160, 40, 2)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    # every tune field (AMWG adapt, m, sigma, accept; AMM adapt, m, valid, alias, Mv, Mvv, the
    # factor in slot form and its pivot order) bit for bit
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])


@pytest.mark.parametrize("name", sorted(RATS_SCHEMES))
def test_rats_parity_config3_scale(mamba, oracle, name):
    """BASELINE configs[2]'s model at 4096 chains x 300 iterations (well past AMM's m > 2n
    switch at 61), the bench's own inits: zero differing bits in draws, values and tune."""
    m = rats(mamba, RATS_SCHEMES[name](mamba))
    init = (mamba.model.rats_init_ls(16384, seed=1000)[:4096] if name == "gibbs_amm"
            else mamba.model.rats_init_matrix(4096))
    eng, dg, st, do = both(mamba, oracle, m, init, 300, 100, 2, seed=20261015)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])


@pytest.mark.parametrize("case", ["rats_gibbs_amm", "line_amm_quad", "line_amm_generic"])
def test_amm_stats_match_oracle(mamba, oracle, case, monkeypatch):
    """mmb_amm_stats (the bench's full-rank fraction and mean factorization steps) counts what
    the oracle's dpstf2 restatement decides: cholfact calls, rank(F) == n (amm.jl:87-90) and
    the rank sum, exactly, per AMM block; the steps the device executed lie between the chain's
    own min(rank + 1, n) and the wavefront's (two chains step together on the 32-lane kernel)."""
    if case == "line_amm_generic":
        monkeypatch.setenv("MMB_LINE_GENERIC", "1")
    if case.startswith("rats"):
        m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
        init = mamba.model.rats_init_ls(16384, seed=1000)[:256]
        iters = 160
    else:
        m = line(mamba, [mamba.AMM(["beta", "s2"], np.eye(3))])
        init = mamba.model.line_init_matrix(1024, seed=4)
        iters = 300
    oracle.amm_stats(reset=True)
    eng, dg, st, do = both(mamba, oracle, m, init, iters, 0, 1)
    so, sg = oracle.amm_stats(reset=True), eng.amm_stats()
    assert sorted(sg) == sorted(so) and sg
    for b in sg:
        g, o = sg[b], so[b]
        assert (g["updates"], g["full_rank"], g["rank_sum"]) == (o["updates"], o["full_rank"], o["rank_sum"]), (b, g, o)
        assert g["updates"] == init.shape[0] * iters
        d = m.block_dim(m.samplers[b])
        chain_steps = g["rank_sum"] + (g["updates"] - g["full_rank"])  # min(rank + 1, d) summed
        assert chain_steps <= g["steps_sum"] <= 2 * chain_steps
        assert g["steps_sum"] <= d * g["updates"]
        assert 0 <= g["redo"] <= g["updates"]
    if case.startswith("rats"):  # the alias split of the bench workload is visible here already
        assert 0.15 < sg[1]["full_rank"] / sg[1]["updates"] < 0.8


def test_chain_order_refresh_interval(mamba, monkeypatch):
    """The table is recomputed after a window only once MMB_ORDER_EVERY (default 64) iterations
    have passed since the last one (the classes persist); a host write of the tune state forces a
    fresh one before the next window."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    init = mamba.model.rats_init_ls(16384, seed=1000)[:256]
    monkeypatch.delenv("MMB_ORDER_EVERY", raising=False)
    eng = mamba.Engine(m)
    eng.init_chains(init, seed=7)
    eng.run(100, burnin=0, thin=2, draws=False)   # >= 64: recomputed after the window
    t100 = eng.chain_order().copy()
    eng.run(30, burnin=0, thin=2, draws=False)    # 30 < 64: kept
    np.testing.assert_array_equal(eng.chain_order(), t100)
    eng.run(40, burnin=0, thin=2, draws=False)    # 70 since: recomputed (a sort of the current classes)
    t170 = eng.chain_order()
    assert sorted(t170.tolist()) == list(range(256))
    eng.close()


def test_chain_order_does_not_change_results(mamba, oracle, monkeypatch):
    """engine.cpp order_chains pairs chains of one factor-validity class in a wavefront before
    every window (the second window below runs permuted: the first set the flags).  The table is
    computed on the device after each window (sweep.hip order_chains_kernel) and must be the
    sort of the chains by (alpha valid, beta valid) of every MMB_ORDER_MODE.  Every chain keeps its own state,
    draws column and Philox id, so the draws, values and tune equal the identity-order run
    (MMB_ORDER_CHAINS=0) and the oracle bit for bit."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    init = mamba.model.rats_init_ls(16384, seed=1000)[:600]
    out = {}
    monkeypatch.setenv("MMB_ORDER_EVERY", "1")  # a fresh table after every window (checked below)
    for mode in ("ordered", "descending", "balanced", "identity"):
        monkeypatch.setenv("MMB_ORDER_MODE", {"descending": "1", "balanced": "2"}.get(mode, "0"))
        if mode == "identity":
            monkeypatch.setenv("MMB_ORDER_CHAINS", "0")
        eng = mamba.Engine(m)
        eng.init_chains(init, seed=33)
        a = eng.run(90, burnin=0, thin=3)
        b = eng.run(60, burnin=0, thin=3)
        ta = eng.tune()
        out[mode] = (a, b, eng.values(), ta)
        order = eng.chain_order()  # the next window's table, from the flags after b
        K = init.shape[0]
        if mode == "identity":
            np.testing.assert_array_equal(order, np.arange(K))
            continue
        (oa, da), (ob, db) = [(o, d) for o, d in _amm_offsets(mamba, m)]
        key = (ta[:, oa + 2] != 0).astype(int) * 2 + (ta[:, ob + 2] != 0).astype(int)
        srt = np.argsort(key, kind="stable")
        if mode == "descending":
            srt = srt[::-1]
        if mode == "balanced":  # pair q -> wave q // NF of workgroup q % NF (8 chains, 4 waves)
            NF, exp = K // 8, srt.copy()
            for pos in range(NF * 8):
                q = pos >> 1
                exp[(q % NF) * 8 + 2 * (q // NF) + (pos & 1)] = srt[pos]
            srt = exp
        np.testing.assert_array_equal(order, srt)
    for mode in ("ordered", "descending", "balanced"):
        for x, y in zip(out[mode], out["identity"]):
            np.testing.assert_array_equal(x, y)
    st = oracle.new_state(m, init)
    do = oracle.run(m, st, 150, burnin=0, thin=3, seed=33, nthreads=8)
    np.testing.assert_array_equal(np.concatenate(out["ordered"][:2]), do)
    tv = out["ordered"][3]
    assert 0.2 < (tv[:, 2] != 0).mean() < 0.9  # alpha factor validity split: the order is not the identity


def _amm_offsets(mamba, m):
    """(offset in the canonical tune row, d) of each AMM block."""
    out, off = [], 0
    for s, n in zip(m.samplers, mamba_tune_lens(mamba, m)):
        if s.kind == mamba.abi.MMB_SAMPLER_AMM:
            out.append((off, m.block_dim(s)))
        off += n
    return out


def test_amwg_lane_parallel_path_matches_sequential(mamba, oracle, monkeypatch):
    """samplers.h amwg_lanes decides every coordinate of the rats alpha / beta AMWG blocks at
    once when each accept test is certain under the logpdf's rounding bound, and falls back to
    amwg_sub!'s sequential loop otherwise; the scalar-block Slice updates evaluate their shrink
    candidates four at a time (slice_uni_cand / slice_multi_cand).  Default, sequential-only
    for both (MMB_AMWG_EXACT=1 with MMB_SLICE_EXACT=1) and a
    2^30 times wider band (=2: many chains of a wavefront fall back while their partner does
    not) give the same draws, values and tune as the oracle, bit for bit; by default the
    fallback is rare."""
    m = rats(mamba, mamba.model.rats_scheme_reference())
    init = mamba.model.rats_init_matrix(1024)
    iters = 120
    out, seqn = {}, {}
    for mode in ("0", "1", "2"):
        monkeypatch.setenv("MMB_AMWG_EXACT", mode)
        monkeypatch.setenv("MMB_SLICE_EXACT", "1" if mode == "1" else "0")
        eng = mamba.Engine(m)
        eng.init_chains(init, seed=71)
        d = eng.run(iters, burnin=30, thin=2)
        out[mode] = (d, eng.values(), eng.tune())
        seqn[mode] = eng.amwg_stats()["sequential_updates"]
    st = oracle.new_state(m, init)
    do = oracle.run(m, st, iters, burnin=30, thin=2, seed=71, nthreads=8)
    for mode in out:
        np.testing.assert_array_equal(out[mode][0], do)
        np.testing.assert_array_equal(out[mode][1], st["values"])
        np.testing.assert_array_equal(out[mode][2], st["tune"][:, :st["tl"]])
    updates = 2 * init.shape[0] * iters  # alpha and beta blocks
    assert seqn["1"] == 0  # forced: not counted as a fallback
    assert seqn["0"] <= 0.001 * updates, seqn
    assert 0.05 * updates < seqn["2"] < updates, seqn


@pytest.mark.parametrize("which", ["multi_s2_c", "uni_mu_alpha"])
def test_rats_slice_overflow_is_an_error(mamba, which):
    """The rats scalar-block Slice evaluates its shrink candidates four at a time
    (samplers.h slice_uni_cand / slice_multi_cand) and stops at the same cap as the sequential
    loop: an infinite width (every candidate NaN) is reported as MMB_E_STATE."""
    S = mamba.model.rats_scheme_reference()
    if which == "multi_s2_c":
        S[0] = mamba.Slice("s2_c", np.inf)
    else:
        S[2] = mamba.Slice(["mu_alpha", "s2_alpha"], [np.inf, 10.0], mamba.Univariate)
    m = rats(mamba, S)
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.rats_init_matrix(3), seed=2)
    with pytest.raises(RuntimeError, match=r"error -4 .*Slice: 3 update\(s\) in iterations 1\.\.1"):
        eng.run(1, burnin=0, thin=1)


def test_restart_and_sharding(mamba, oracle):
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    init = mamba.model.rats_init_ls(128, seed=3)
    e1 = mamba.Engine(m)
    e1.init_chains(init, seed=5)
    full = e1.run(150, burnin=30, thin=3)
    e2 = mamba.Engine(m)
    e2.init_chains(init, seed=5)
    a = e2.run(70, burnin=30, thin=3)             # split past AMM's switch at m = 2d + 1 = 61
    b = e2.run(80, burnin=30, thin=3)
    np.testing.assert_array_equal(np.concatenate([a, b]), full)
    e3 = mamba.Engine(m)
    e3.init_chains(init[64:], chain_offset=64, seed=5)
    np.testing.assert_array_equal(e3.run(150, burnin=30, thin=3), full[:, :, 64:])


@pytest.mark.parametrize("how", ["window", "host_roundtrip", "file"])
def test_rats_carried_proposal_resume_after_switch(mamba, oracle, tmp_path, how):
    """AMM's carried proposal (samplers.h, tag = host epoch << 32 | iteration) after the
    adaptive switch (m > 2d = 60, amm.jl:72-76): 256 chains x 200 iterations split at 100
    (i) into two mmb_run windows with no host write (the carried proposal is reused),
    (ii) with a values + tune + iter round trip through the host in between (the epoch
    changes: the first resumed update recomputes SigmaLm z2 by the direct matvec from the
    factor restored by mmb_set_tune's slot -> position conversion), (iii) through a file
    checkpoint into a fresh engine (mcmc.jl:3-16).  Each equals the uninterrupted run bit for
    bit and the oracle bit for bit."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    init = mamba.model.rats_init_ls(256, seed=12)
    eng, full, st, do = both(mamba, oracle, m, init, 200, 100, 2, seed=21)
    np.testing.assert_array_equal(full, do)
    m1 = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    e1 = mamba.Engine(m1)
    e1.init_chains(init, seed=21)
    a = e1.run(100, burnin=100, thin=2)
    assert a is None
    tune_mid = e1.tune()
    amm = [o for o, s in zip(np.cumsum([0] + [len_ for len_ in mamba_tune_lens(mamba, m1)]), m1.samplers)
           if s.kind == mamba.abi.MMB_SAMPLER_AMM]
    # m = 100 > 2d: past the switch; most chains hold a valid (full-rank) factor whose carried
    # proposal the next window uses (the others are rank deficient: SigmaLm is kept, amm.jl:88-90)
    assert all((tune_mid[:, o + 1] == 100).all() and (tune_mid[:, o + 2] == 1).sum() >= 96 for o in amm)
    if how == "host_roundtrip":
        v, t, it = e1.values(), e1.tune(), e1.iter
        o, d = amm[0], 30
        bad = t.copy()
        bad[5, o + 4 + 2 * d + d * (d + 1) - 1] = bad[5, o + 4 + 2 * d + d * (d + 1) - 2]  # repeated pivot
        with pytest.raises(RuntimeError, match="not a permutation"):
            e1.set_tune(bad)                                # rejected before any state changes
        bad = t.copy()
        bad[7, o + 4 + 2 * d + d * (d + 1) - d] = 30.0      # pivot index out of range
        with pytest.raises(RuntimeError, match="not a permutation"):
            e1.set_tune(bad)
        e1.set_values(v)
        e1.set_tune(t)
        e1.set_iter(it)
        np.testing.assert_array_equal(e1.tune(), t)
        b = e1.run(100, burnin=100, thin=2)
    elif how == "file":
        m1.iter, m1.burnin = e1.iter, 0
        mc = mamba.Chains(np.empty((0, e1.pmon, 256)), m1.monitor_names, 102, 2, np.arange(1, 257), m1, e1)
        p = str(tmp_path / "rats_switch.chains")
        mamba.write(p, mc)
        e1.close()
        mc2 = mamba.read(p, model=rats(mamba, mamba.model.rats_scheme_gibbs_amm()))
        assert mc2.engine.iter == 100
        b = mc2.engine.run(100, burnin=100, thin=2)
    else:
        b = e1.run(100, burnin=100, thin=2)
    np.testing.assert_array_equal(b, full)


def mamba_tune_lens(mamba, m):
    """Canonical tune-row length of each block (engine.cpp mmb_get_tune layout)."""
    out = []
    for s in m.samplers:
        d = m.block_dim(s)
        if s.kind == mamba.abi.MMB_SAMPLER_AMWG:
            out.append(2 + 2 * d)
        elif s.kind == mamba.abi.MMB_SAMPLER_AMM:
            out.append(4 + 2 * d + d * (d + 1))
        else:
            out.append(0)
    return out


def test_device_gelman_rubin_matches_host(mamba):
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.rats_init_ls(1024, seed=1), seed=2)
    d = eng.run(400, burnin=100, thin=2, keep_device=True)
    for transform in (False, True):
        ps_dev, mp_dev = mamba.gelmandiag_sharded(eng, transform=transform, mpsrf=True)
        ps_host, mp_host = mamba.gelmandiag(d, transform=transform, mpsrf=True)
        np.testing.assert_allclose(ps_dev, ps_host, rtol=1e-8)
        assert mp_dev == pytest.approx(mp_host, rel=1e-8)


def test_mcmc_api_and_full_size_properties(mamba):
    """16384 chains (BASELINE config 3 size): finite draws, chains near the published
    rats posterior after a short run, and Mamba's Chains layout/range."""
    m = mamba.rats().setsamplers(mamba.model.rats_scheme_gibbs_amm())
    sim = mamba.mcmc(m, mamba.model.RATS_DATA, mamba.model.rats_init_ls(16384, seed=9), 300,
                     burnin=100, thin=2, chains=16384)
    assert sim.value.shape == (100, 3, 16384)
    assert list(sim.range)[:2] == [102, 104] and sim.names == ["s2_c", "mu_beta", "alpha0"]
    assert np.isfinite(sim.value).all()
    mb = sim["mu_beta"].mean()
    a0 = sim["alpha0"].mean()
    assert abs(mb - 6.183) < 0.02 and abs(a0 - 106.63) < 0.5, (mb, a0)


def logistic(mamba, nobs, ncoef, scheme=None):
    data, bt = mamba.model.logistic_data(nobs, ncoef)
    m = mamba.logistic(nobs, ncoef, 10.0)
    m.setinputs(data)
    return m.setsamplers(scheme or [mamba.NUTS("beta", dtype="analytic")]), bt


def _spd(p, seed, a, b):
    A = np.random.default_rng(seed).normal(0.0, 1.0, (p, p + 4))
    return (A @ A.T) / (p + 4) * a + b * np.eye(p)


LOGISTIC_GRAD_SCHEMES = {
    "hmc": lambda M, p: [M.HMC("beta", 0.01, 7, dtype="analytic")],
    "hmc_sigma": lambda M, p: [M.HMC("beta", 0.01, 4, _spd(p, 1, 0.2, 1.0), dtype="analytic")],  # near I
    "mala": lambda M, p: [M.MALA("beta", 2e-4, dtype="analytic")],
    "mala_sigma": lambda M, p: [M.MALA("beta", 0.5, _spd(p, 2, 1e-3, 1e-4), dtype="analytic")],
}


@pytest.mark.parametrize("name", sorted(LOGISTIC_GRAD_SCHEMES))
def test_logistic_hmc_mala_parity(mamba, oracle, name):
    """HMC / MALA (hmc.jl:72-111, mala.jl:67-86) on the batched MFMA gradient engine:
    bit-exact against the oracle (same gradient summation spec as NUTS)."""
    m, _ = logistic(mamba, 1000, 50, LOGISTIC_GRAD_SCHEMES[name](mamba, 50))
    K = 100
    init = np.random.default_rng(9).normal(0.0, 0.1, (K, 50))
    eng, dg, st, do = both(mamba, oracle, m, init, 25, 5, 1)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])
    # moves happened (not all rejected) and gradient counts are exact
    assert (np.abs(np.diff(dg, axis=0)).sum(axis=1) > 0).mean() > 0.2
    per = 8 if name == "hmc" else 5 if name == "hmc_sigma" else 2
    assert eng.grad_evals() == 25 * K * per


def test_logistic_nuts_parity(mamba, oracle):
    """Config 4 at reduced N: the batched MFMA gradient engine against the oracle's
    sequential restatement of the same summation order."""
    m, bt = logistic(mamba, 1000, 50)
    K = 100                                    # 2 chain tiles, the second partly live
    init = np.random.default_rng(8).normal(0.0, 0.1, (K, 50))
    eng, dg, st, do = both(mamba, oracle, m, init, 30, 10, 1, model_burnin=15)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])


@pytest.mark.parametrize("grad", ["analytic", "forward", "hmc", "mala"])
def test_logistic_split_identical(mamba, monkeypatch, grad):
    """A window runs its chains as independent parts on their own streams (engine.cpp
    run_logistic): draws, state, tuning and gradient counts identical to one stream for 2 and 3
    parts (unequal), at a width where the group-mode (fold) gradient kernel runs."""
    sch = {"hmc": [mamba.HMC("beta", 0.01, 7, dtype="analytic")], "mala": [mamba.MALA("beta", 2e-4, dtype="analytic")]}
    m, _ = logistic(mamba, 1000, 50, sch.get(grad) or [mamba.NUTS("beta", dtype=grad)])
    K = 301 if grad == "forward" else 1500
    init = np.random.default_rng(21).normal(0.0, 0.1, (K, 50))
    out = []
    for split in ("1", "2", "3"):
        monkeypatch.setenv("MMB_LG_SPLIT", split)
        eng = mamba.Engine(m)
        eng.init_chains(init, seed=5)
        d = eng.run(12, burnin=0, thin=1, model_burnin=6)
        out.append((d, eng.values(), eng.tune(), eng.grad_evals()))
        eng.close()
    for o in out[1:]:
        for a, b in zip(out[0], o):
            np.testing.assert_array_equal(a, b)


def test_logistic_device_gelman_rubin_matches_host(mamba):
    """p = 50 monitored values: the workgroup-per-chain-chunk Gelman-Rubin kernel."""
    m, _ = logistic(mamba, 1000, 50)
    eng = mamba.Engine(m)
    eng.init_chains(np.random.default_rng(3).normal(0.0, 0.1, (40, 50)), seed=4)
    d = eng.run(60, burnin=20, thin=1, model_burnin=20, keep_device=True)
    for transform in (False, True):
        ps_dev, mp_dev = mamba.gelmandiag_sharded(eng, transform=transform, mpsrf=True)
        ps_host, mp_host = mamba.gelmandiag(d, transform=transform, mpsrf=True)
        np.testing.assert_allclose(ps_dev, ps_host, rtol=1e-8)
        assert mp_dev == pytest.approx(mp_host, rel=1e-6)


def _summary_ref():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import summary_ref
    return summary_ref


@pytest.mark.parametrize("iters,burnin,thin,bs,K", [(400, 100, 2, 100, 1024), (375, 0, 1, 100, 300),
                                                     (60, 10, 1, 128, 257)])
def test_device_summarystats_and_quantiles(mamba, iters, burnin, thin, bs, K):
    """summarystats (stats.jl:85-94, mcse_bm mcse.jl:10-19) and quantile (stats.jl:73-80)
    from the device-kept draws vs the oracle restatement on the same draws: sums within
    rtol 1e-10 (reduction order differs), order statistics exact.  Covers batches that
    straddle chains (n % bs != 0) and batches longer than a chain (bs > n)."""
    sr = _summary_ref()
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.rats_init_ls(K, seed=5), seed=6)
    d = eng.run(iters, burnin=burnin, thin=thin, keep_device=True)
    sim = mamba.Chains(d, m.monitor_names, burnin + thin, thin, np.arange(1, K + 1), m, eng)
    got = sim.summarystats(bs)
    ref = sr.summarystats(d, bs)
    np.testing.assert_allclose(got[:, :4], ref[:, :4], rtol=1e-10)
    np.testing.assert_allclose(got[:, 4], ref[:, 4], rtol=1e-8)
    q = (0.025, 0.25, 0.5, 0.75, 0.975)
    np.testing.assert_array_equal(sim.quantile(q), sr.quantile(d, q))
    desc = sim.describe()
    assert set(desc) == {"s2_c", "mu_beta", "alpha0"} and desc["mu_beta"]["Mean"] == got[1, 0]


def test_device_summary_logistic_many_params(mamba):
    """p = 50 monitored values (one grid row per param)."""
    sr = _summary_ref()
    m, _ = logistic(mamba, 1000, 50)
    eng = mamba.Engine(m)
    eng.init_chains(np.random.default_rng(3).normal(0.0, 0.1, (40, 50)), seed=4)
    d = eng.run(80, burnin=20, thin=1, model_burnin=20, keep_device=True)
    got = mamba.summarystats_sharded(eng, batch_size=50)
    np.testing.assert_allclose(got[:, :4], sr.summarystats(d, 50)[:, :4], rtol=1e-9)
    np.testing.assert_array_equal(mamba.quantile_sharded(eng, (0.1, 0.5, 0.9)), sr.quantile(d, (0.1, 0.5, 0.9)))


@pytest.mark.parametrize("scheme", ["gibbs_amm", "reference"])
def test_checkpoint_file_resume(mamba, tmp_path, scheme):
    """write(name, mc) + read(name, ModelChains) + mcmc(mc, iters) (fileio.jl:3-12,
    mcmc.jl:3-16): a run checkpointed to a file and resumed in a fresh engine equals the
    uninterrupted run draw for draw (values, AMM moments/factors, AMWG/Slice tune, iter)."""
    sch = {"gibbs_amm": mamba.model.rats_scheme_gibbs_amm,
           "reference": mamba.model.rats_scheme_reference}[scheme]
    init = mamba.model.rats_init_ls(96, seed=4)
    m = rats(mamba, sch())
    e = mamba.Engine(m)
    e.init_chains(init, chain_offset=32, seed=11)
    full = e.run(110, burnin=20, thin=2)
    m1 = rats(mamba, sch())
    e1 = mamba.Engine(m1)
    e1.init_chains(init, chain_offset=32, seed=11)
    a = e1.run(70, burnin=20, thin=2)             # past AMM's adaptive switch (m > 2d = 60)
    m1.iter, m1.burnin = e1.iter, 20
    mc = mamba.Chains(a, m1.monitor_names, 22, 2, np.arange(33, 129), m1, e1)
    p = str(tmp_path / "rats.chains")
    mamba.write(p, mc)
    e1.close()
    m2 = rats(mamba, sch())
    mc2 = mamba.read(p, model=m2)
    assert mc2.engine.iter == 70
    mc3 = mamba.mcmc_restart(mc2, 40)
    np.testing.assert_array_equal(mc3.value, full)
    assert list(mc3.range) == list(range(22, 111, 2))


@pytest.mark.parametrize("name", ["nuts_slice", "amwg", "hmc", "mala_sigma_gibbs"])
def test_checkpoint_file_resume_line(mamba, tmp_path, name):
    """Checkpoint inside NUTS's dual-averaging burnin (model burnin 150, written at 100):
    the NUTS tune (eps, epsbar, Hbar, mu, m, init flag) and Model.burnin travel in the file."""
    init = mamba.model.line_init_matrix(256, seed=4)
    e = mamba.Engine(line(mamba, LINE_SCHEMES[name](mamba)))
    e.init_chains(init, seed=8)
    full = e.run(300, burnin=150, thin=2, model_burnin=150)
    m1 = line(mamba, LINE_SCHEMES[name](mamba))
    e1 = mamba.Engine(m1)
    e1.init_chains(init, seed=8)
    a = e1.run(100, burnin=150, thin=2, model_burnin=150)
    assert a is None
    m1.iter, m1.burnin = e1.iter, 150
    mc = mamba.Chains(np.empty((0, e1.pmon, 256)), m1.monitor_names, 152, 2, np.arange(1, 257), m1, e1)
    p = str(tmp_path / "line.chains")
    mamba.write(p, mc)
    e1.close()
    mc2 = mamba.read(p, model=line(mamba, LINE_SCHEMES[name](mamba)))
    assert mc2.model.burnin == 150 and mc2.engine.iter == 100
    b = mc2.engine.run(200, burnin=150, thin=2, model_burnin=mc2.model.burnin)
    np.testing.assert_array_equal(b, full)


@pytest.mark.parametrize("name", ["nuts", "hmc"])
def test_checkpoint_file_resume_logistic(mamba, tmp_path, name):
    """Logistic (config 4 at N=1000): the resumable NUTS / HMC machines hold no state across
    iteration boundaries beyond values + tune, so a file checkpoint resumes exactly."""
    sch = (lambda: [mamba.NUTS("beta", dtype="analytic")]) if name == "nuts" else (lambda: LOGISTIC_GRAD_SCHEMES["hmc"](mamba, 50))
    K = 100
    init = np.random.default_rng(8).normal(0.0, 0.1, (K, 50))
    m, _ = logistic(mamba, 1000, 50, sch())
    e = mamba.Engine(m)
    e.init_chains(init, seed=3)
    full = e.run(30, burnin=10, thin=1, model_burnin=15)
    m1, _ = logistic(mamba, 1000, 50, sch())
    e1 = mamba.Engine(m1)
    e1.init_chains(init, seed=3)
    a = e1.run(12, burnin=10, thin=1, model_burnin=15)
    m1.iter, m1.burnin = e1.iter, 15
    mc = mamba.Chains(a, m1.monitor_names, 11, 1, np.arange(1, K + 1), m1, e1)
    p = str(tmp_path / "lg.chains")
    mamba.write(p, mc)
    e1.close()
    m2, _ = logistic(mamba, 1000, 50, sch())
    mc2 = mamba.read(p, model=m2)
    b = mc2.engine.run(18, burnin=10, thin=1, model_burnin=mc2.model.burnin)
    np.testing.assert_array_equal(np.concatenate([mc2.value, b]), full)


@pytest.mark.parametrize("K,iters,burnin,thin,offset", [(1, 13, 3, 3, 0), (37, 21, 0, 1, 1000), (129, 17, 16, 1, 7), (64, 14, 4, 5, 0)])
def test_rats_ragged_shapes(mamba, oracle, K, iters, burnin, thin, offset):
    """Chain counts that fill neither a wave (2 chains) nor a workgroup (8 chains), windows
    that are not a multiple of the kernel's iterations per launch, a single kept draw,
    and nonzero global chain offsets."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    init = mamba.model.rats_init_ls(K, seed=6)
    eng, dg, st, do = both(mamba, oracle, m, init, iters, burnin, thin, offset=offset)
    assert dg.shape == do.shape == ((iters - burnin) // thin, 3, K)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])


@pytest.mark.parametrize("K", [1, 65])
@pytest.mark.parametrize("name", ["amm", "nuts_slice"])
def test_line_ragged_shapes(mamba, oracle, name, K):
    m = line(mamba, LINE_SCHEMES[name](mamba))
    init = mamba.model.line_init_matrix(K, seed=5)
    eng, dg, st, do = both(mamba, oracle, m, init, 71, 10, 3, offset=3, model_burnin=20)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])


def test_empty_window_leaves_state(mamba):
    """iters = 0: no kernel work, no draws, Model.iter and the chain state unchanged."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.rats_init_ls(40, seed=1), seed=3)
    eng.run(9, burnin=0, thin=1)
    v, t = eng.values(), eng.tune()
    assert eng.run(0, burnin=0, thin=1) is None
    assert eng.iter == 9
    np.testing.assert_array_equal(eng.values(), v)
    np.testing.assert_array_equal(eng.tune(), t)


def test_logistic_single_chain(mamba, oracle):
    """K = 1: one live lane of the first 16-chain MFMA tile, 63 padded chains."""
    m, _ = logistic(mamba, 1000, 50)
    init = np.random.default_rng(1).normal(0.0, 0.1, (1, 50))
    eng, dg, st, do = both(mamba, oracle, m, init, 12, 4, 2, model_burnin=6)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])


def test_logistic_nuts_parity_full(mamba, oracle):
    """Config 4 at its stated size (N = 10000, p = 50; BASELINE configs[3], nuts.jl:95-180):
    mmb_lg_rps = 160 rows per sub-range, 32 groups x 2 sub-ranges; 70 chains = one full and
    one partly filled 64-chain tile, NUTS chains idle at different steps.  Bit-exact."""
    m, _ = logistic(mamba, 10000, 50)
    K = 70
    init = np.random.default_rng(21).normal(0.0, 0.1, (K, 50))
    eng, dg, st, do = both(mamba, oracle, m, init, 8, 2, 1, model_burnin=4)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])


@pytest.mark.parametrize("sampler", ["nuts", "hmc", "mala"])
def test_logistic_forward_difference_parity(mamba, oracle, sampler):
    """The reference's default gradient on config 4's model: NUTS("beta") with no dtype is
    gradlogpdf!(...; dtype = :forward) (nuts.jl:47-56 -> simulation.jl:47-51, Calculus forward
    differences), run as p + 1 log-density columns per request through the batched MFMA kernel
    (logistic.hip lg_grad_kernel<.., LPONLY>, lg_assemble_fd).  Bit-exact against the oracle's
    restatement (oracle.c logf_grad: logf at x and at x + eps_k e_k in the same summation spec)."""
    sch = {"nuts": [mamba.NUTS("beta")], "hmc": [mamba.HMC("beta", 0.01, 3)], "mala": [mamba.MALA("beta", 2e-4)]}
    m, _ = logistic(mamba, 1000, 50, sch[sampler])
    assert m.samplers[0].gradient == mamba.abi.MMB_GRAD_FORWARD
    K = 70
    init = np.random.default_rng(41).normal(0.0, 0.1, (K, 50))
    eng, dg, st, do = both(mamba, oracle, m, init, 12, 2, 1, model_burnin=6)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])
    assert np.abs(dg[-1] - dg[0]).max() > 0


def test_logistic_forward_difference_full_size(mamba, oracle):
    """Forward differences at config 4's size (N = 10000, p = 50): 51 columns per request, group
    mode (>= 1024 columns), the 160-row sub-ranges; K = 70 NUTS chains, bit-exact vs the oracle,
    and the gradient within forward-difference error of the analytic one."""
    m, _ = logistic(mamba, 10000, 50, [mamba.NUTS("beta")])
    K = 70
    init = np.random.default_rng(42).normal(0.0, 0.1, (K, 50))
    eng, dg, st, do = both(mamba, oracle, m, init, 4, 1, 1, model_burnin=2)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])
    # the two gradients of one position agree to forward-difference accuracy
    x = st["values"][0]
    _, gf = oracle.block_logpdf(m, st["values"][0], 0, x, grad=True)
    ma, _ = logistic(mamba, 10000, 50, [mamba.NUTS("beta", dtype="analytic")])
    _, ga = oracle.block_logpdf(ma, st["values"][0], 0, x, grad=True)
    np.testing.assert_allclose(gf, ga, rtol=0, atol=1e-4 * np.abs(ga).max() + 1e-3)


@pytest.mark.parametrize("p", [53, 64])
def test_logistic_wide_parity(mamba, oracle, p):
    """53 <= p <= MMB_LG_DV: the 16-k-step first GEMM (coefficients 52..63 are part of eta)."""
    for sch in ([mamba.NUTS("beta", dtype="analytic")], [mamba.HMC("beta", 0.01, 5, dtype="analytic")]):
        m, _ = logistic(mamba, 1000, p, sch)
        K = 40
        init = np.random.default_rng(p).normal(0.0, 0.1, (K, p))
        eng, dg, st, do = both(mamba, oracle, m, init, 10, 2, 1, model_burnin=5)
        np.testing.assert_array_equal(dg, do)
        np.testing.assert_array_equal(eng.values(), st["values"])
        assert np.abs(dg[-1] - dg[0]).max() > 0


def test_logistic_group_mode_parity(mamba, oracle):
    """Wide gradient steps (>= MMB_LG_FOLD_MIN = 1024 running chains, engine.cpp) run one
    workgroup per (group, tile) that forms the group's (P0 + P1) itself; narrower steps one
    workgroup per sub-range.  NUTS with 1100 chains switches between the two as chains idle,
    HMC with 1024 chains at N = 10000 (160-row sub-ranges) stays in group mode: bit-exact."""
    m, _ = logistic(mamba, 1000, 50)
    K = 1100
    init = np.random.default_rng(31).normal(0.0, 0.1, (K, 50))
    eng, dg, st, do = both(mamba, oracle, m, init, 6, 1, 1, model_burnin=3)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])
    m, _ = logistic(mamba, 10000, 50, [mamba.HMC("beta", 0.005, 2, dtype="analytic")])
    K = 1024
    init = np.random.default_rng(32).normal(0.0, 0.1, (K, 50))
    eng, dg, st, do = both(mamba, oracle, m, init, 2, 0, 1)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    assert eng.grad_evals() == 2 * K * 3


def test_logistic_full_size_properties(mamba):
    """Config 4 at full size: N = 10000, p = 50, 4096 chains.  Finite draws, every update
    completed without hitting the depth cap, gradient count consistent with the tree
    depths, and Gelman-Rubin PSRF < 1.1 on all 50 coefficients after burnin."""
    m, _ = logistic(mamba, 10000, 50)
    K = 4096
    eng = mamba.Engine(m)
    eng.init_chains(np.random.default_rng(5).normal(0.0, 0.1, (K, 50)), seed=6)
    d = eng.run(200, burnin=100, thin=1, model_burnin=100, keep_device=True)
    assert d.shape == (100, 50, K) and np.isfinite(d).all()
    ns = eng.nuts_stats()
    assert ns["updates"] == 200 * K and ns["depth_cap_hits"] == 0
    # a depth-j tree evaluates at least j leapfrog gradients (one per doubling)
    assert eng.grad_evals() >= ns["depth_sum"] and 1.0 <= ns["depth_sum"] / ns["updates"] <= 10.0
    psrf, _ = mamba.gelmandiag_sharded(eng)
    assert (psrf[:, 0] < 1.1).all(), psrf[:, 0].max()


@pytest.mark.parametrize("form", ["uni", "multi"])
def test_slice_shrink_overflow_is_an_error(mamba, form):
    """An infinite Slice width makes every candidate NaN (lower = -Inf, upper = NaN), which
    s2's InverseGamma support rejects: the reference's shrink loop (slice.jl:78-88,103-113)
    never ends.  The kernel stops after MMB_SLICE_MAX_SHRINK rejections and mmb_run reports
    MMB_E_STATE instead of keeping an out-of-slice draw silently."""
    Fm = mamba.Univariate if form == "uni" else mamba.Multivariate
    m = line(mamba, [mamba.AMWG("beta", 1.0), mamba.Slice("s2", np.inf, Fm)])
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.line_init_matrix(3, seed=1), seed=2)
    with pytest.raises(RuntimeError, match=r"error -4 .*Slice: 3 update\(s\) in iterations 1\.\.1"):
        eng.run(1, burnin=0, thin=1)
    # a finite width on the same engine and chains still runs
    m2 = line(mamba, [mamba.AMWG("beta", 1.0), mamba.Slice("s2", 3.0, Fm)])
    e2 = mamba.Engine(m2)
    e2.init_chains(mamba.model.line_init_matrix(3, seed=1), seed=2)
    assert np.isfinite(e2.run(5, burnin=0, thin=1)).all()


@pytest.mark.parametrize("how", ["init_all", "unique_id"])
def test_gr_allreduce_rccl_one_gpu(mamba, how):
    """mmb_comm_init + mmb_range_allreduce + mmb_gr_allreduce (gelmandiag.jl:11-25)
    at ngpu = 1, through both communicator forms (ncclCommInitAll; ncclCommInitRank with a
    unique id): the RCCL sums equal the engine's own partials bit for bit (a one-rank SUM is
    the identity) and the PSRF equals the host gelmandiag of the same draws."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.rats_init_ls(512, seed=3), seed=4)
    d = eng.run(240, burnin=40, thin=2, keep_device=True)
    comm = (mamba.Comm([eng]) if how == "init_all"
            else mamba.Comm([eng], nranks=1, rank0=0, uid=mamba.Comm.unique_id()))
    mm = comm.range_allreduce()
    np.testing.assert_array_equal(mm, eng.gr_range())
    for transform in (False, True):
        ps, mp = mamba.gelmandiag_rccl(comm, transform=transform, mpsrf=True)
        ps_h, mp_h = mamba.gelmandiag(d, transform=transform, mpsrf=True)
        np.testing.assert_allclose(ps, ps_h, rtol=1e-8)
        assert mp == pytest.approx(mp_h, rel=1e-8)
    kinds = np.array([1, 0, 0], dtype=np.int32)
    shift = np.array([3.6, 6.0, 100.0])
    np.testing.assert_array_equal(comm.gr_allreduce(kinds, shift), eng.gr_partials(kinds, shift))
    comm.close()


def test_gr_allreduce_agreement_fails_together(mamba):
    """The collective's agreement step (engine.cpp comm_agree): a process whose engines hold
    too few kept draws fails with MMB_E_STATE *after* joining one MAX all-reduce (its peers
    do not block), and the RCCL group is closed afterwards: the next collectives on the
    same communicator still work."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.rats_init_ls(128, seed=3), seed=4)
    eng.run(12, burnin=10, thin=2, keep_device=True)        # one kept draw per chain
    assert eng.num_kept() == 1
    comm = mamba.Comm([eng], nranks=1, rank0=0, uid=mamba.Comm.unique_id())
    mm = comm.range_allreduce()                               # needs >= 1: fine
    np.testing.assert_array_equal(mm, eng.gr_range())
    with pytest.raises(RuntimeError, match=r"error -4 .*need >= 2 device-kept draws"):
        comm.gr_allreduce(np.zeros(3, np.int32), np.zeros(3))
    d = eng.run(40, burnin=0, thin=2, keep_device=True)
    np.testing.assert_array_equal(comm.range_allreduce(), eng.gr_range())
    kinds, shift = np.array([1, 0, 0], np.int32), np.array([3.6, 6.0, 100.0])
    np.testing.assert_array_equal(comm.gr_allreduce(kinds, shift), eng.gr_partials(kinds, shift))
    comm.close()
    assert d.shape[0] == 20


def test_gr_allreduce_stage_failure_reaches_the_collective(mamba, monkeypatch):
    """A rank whose agreement contribution cannot be staged (injected: MMB_TEST_COMM_STAGE_FAIL)
    still joins the agreement all-reduce, and what it contributes is the failure flag the slot
    is armed with -- never the "agree" a previous successful call left there -- so its peers
    skip the collective instead of waiting in it; the communicator keeps working afterwards."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    eng = mamba.Engine(m)
    eng.init_chains(mamba.model.rats_init_ls(128, seed=3), seed=4)
    eng.run(40, burnin=0, thin=2, keep_device=True)
    comm = mamba.Comm([eng], nranks=1, rank0=0, uid=mamba.Comm.unique_id())
    kinds, shift = np.array([1, 0, 0], np.int32), np.array([3.6, 6.0, 100.0])
    ok = comm.gr_allreduce(kinds, shift)                      # leaves a successful agreement behind
    monkeypatch.setenv("MMB_TEST_COMM_STAGE_FAIL", "1")
    with pytest.raises(RuntimeError, match=r"error -3 .*agreement staging.*saw flag 2"):
        comm.gr_allreduce(kinds, shift)
    monkeypatch.delenv("MMB_TEST_COMM_STAGE_FAIL")
    np.testing.assert_array_equal(comm.gr_allreduce(kinds, shift), ok)
    comm.close()


def test_rats_scale_total_on_one_gpu(mamba, oracle):
    """The 8-GPU configuration's 131 072 chains (8 x 16 384, BASELINE configs[4]) in ONE engine:
    rank 5's shard run alone (its chain range, chain_offset = 5 x 16 384) reproduces its
    columns bit for bit -- a chain's draws depend only on its global id, so the weak-scaling
    shards of bench.py compute exactly the single-engine result -- and the first chains
    match the oracle."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    K, S, r = 131072, 16384, 5
    init = mamba.model.rats_init_ls(K, seed=21)
    e = mamba.Engine(m)
    e.init_chains(init, seed=8)
    d = e.run(24, burnin=0, thin=4)
    assert d.shape == (6, 3, K) and np.isfinite(d).all()
    vals = e.values()
    e5 = mamba.Engine(m)
    e5.init_chains(init[r * S:(r + 1) * S], chain_offset=r * S, seed=8)
    np.testing.assert_array_equal(e5.run(24, burnin=0, thin=4), d[:, :, r * S:(r + 1) * S])
    np.testing.assert_array_equal(e5.values(), vals[r * S:(r + 1) * S])
    st = oracle.new_state(m, init[:32])
    do = oracle.run(m, st, 24, burnin=0, thin=4, seed=8, chain_offset=0, nthreads=8)
    np.testing.assert_array_equal(d[:, :, :32], do)


def test_gradient_choice_validated(mamba):
    """mmb_gradient (include/mamba_hip.h): the analytic gradient is not available on the node IR
    and is refused at mmb_create; the reference's default NUTS(:beta) (dtype=:forward) on
    logistic now runs its forward differences on the device (test_logistic_forward_difference_*)."""
    A = mamba.abi
    m = mamba.logistic(200, 5, 10.0)
    m.setsamplers([mamba.NUTS("beta")])
    assert m.samplers[0].gradient == A.MMB_GRAD_FORWARD
    ir = mamba.ir
    mi = ir.seeds_model().setinputs(ir.SEEDS)
    mi.setsamplers([mamba.NUTS(["alpha0", "alpha1", "alpha2", "alpha12"], dtype="analytic"), mamba.AMWG("b", 0.01),
                    mamba.AMWG("s2", 0.1)])
    mi.init_matrix([ir.seeds_inits()[0]], 1)
    with pytest.raises(RuntimeError, match="gradient"):
        mamba.Engine(mi)
    with pytest.raises(mamba.samplers.ArgumentError):
        mamba.NUTS("beta", dtype="central")
