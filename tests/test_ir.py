"""Node IR on the CPU: the lowering of Mamba Model DAGs, the oracle's
restatement of the IR semantics pinned against (i) the hand-lowered line and rats models,
(ii) an independent scipy evaluation of logpdf! (simulation.jl:77-90) for every supported
family and transform, (iii) libm lgamma, and the Calculus forward-difference gradient."""
import math

import numpy as np
import pytest
from scipy import stats
from scipy.special import expit, gammaln

RATS_BLOCKS = None


def ir_line(mamba, scheme):
    m = mamba.ir.line_model()
    m.setinputs(mamba.model.LINE_DATA)
    return m.setsamplers(scheme)


def test_lgamma_vs_libm(oracle):
    xs = np.concatenate([np.geomspace(1e-3, 1e4, 400), [0.5, 1.0, 1.5, 2.0, 2.5, 9.999, 10.0, 10.001]])
    for x in xs:
        want = math.lgamma(x)
        assert oracle.L.orc_lgamma(x) == pytest.approx(want, rel=1e-14, abs=1e-14), x


def test_ir_line_equals_hand_lowered_line(mamba, oracle):
    scheme = [mamba.AMWG(["beta", "s2"], 1.0), mamba.Slice("s2", 3.0)]
    m = ir_line(mamba, scheme)
    init = mamba.model.line_init_matrix(16, seed=3)
    V = m.init_matrix([{"y": [1.0, 3, 3, 3, 5], "beta": init[k, :2], "s2": init[k, 2]} for k in range(16)], 16)
    h = mamba.line().setinputs(mamba.model.LINE_DATA).setsamplers(scheme)
    np.testing.assert_array_equal(V, init)
    for k in range(16):
        x = np.array([V[k, 0], V[k, 1], np.log(V[k, 2])])
        assert oracle.block_logpdf(m, V[k], 0, x) == pytest.approx(oracle.block_logpdf(h, init[k], 0, x), rel=1e-13)
        assert oracle.block_logpdf(m, V[k], 1, [V[k, 2]]) == pytest.approx(
            oracle.block_logpdf(h, init[k], 1, [V[k, 2]]), rel=1e-13)
    assert m.monitor_names == ["beta[1]", "beta[2]", "s2"]


def test_ir_rats_equals_hand_lowered_rats(mamba, oracle):
    scheme = mamba.model.rats_scheme_reference()
    m = mamba.ir.rats_model().setinputs(mamba.ir.rats_inputs()).setsamplers(scheme)
    h = mamba.rats().setinputs(mamba.model.RATS_DATA).setsamplers(scheme)
    init = mamba.model.rats_init_ls(8, seed=4)
    # canonical orders: IR = declaration order (alpha, mu_alpha, s2_alpha, beta, mu_beta, s2_beta, s2_c)
    names = ["s2_c", "alpha", "mu_alpha", "s2_alpha", "beta", "mu_beta", "s2_beta"]
    sl = {"s2_c": slice(0, 1), "alpha": slice(1, 31), "mu_alpha": slice(31, 32), "s2_alpha": slice(32, 33),
          "beta": slice(33, 63), "mu_beta": slice(63, 64), "s2_beta": slice(64, 65)}
    inits = [{**{n: init[k, sl[n]] for n in names}, "y": mamba.model.RATS_Y} for k in range(8)]
    V = m.init_matrix(inits, 8)
    assert m.monitor_names == ["alpha0", "mu_beta", "s2_c"]
    rng = np.random.default_rng(1)
    for k in range(8):
        for b, s in enumerate(scheme):
            xh = np.concatenate([init[k, sl[p]] for p in s.params])
            xh = xh + rng.normal(0, 0.05, xh.size) * np.abs(xh)
            lp_h = oracle.block_logpdf(h, init[k], b, np.log(xh) if s.kind == mamba.abi.MMB_SAMPLER_AMWG and
                                       s.params[0].startswith("s2") else xh)
            lp_i = oracle.block_logpdf(m, V[k], b, xh)
            assert lp_i == pytest.approx(lp_h, rel=1e-12), (k, s)


# ---- every family and transform against scipy (the reference's logpdf! semantics) ----------

def zoo(mamba):
    ir = mamba.ir
    return ir.Model(
        obs_bin=ir.Stochastic(1, lambda nn, p: ir.Binomial(nn, p), False),
        obs_poi=ir.Stochastic(1, lambda lam, t: ir.Poisson(lam * t), False),
        obs_ber=ir.Stochastic(1, lambda p: ir.Bernoulli(p[1]), False),
        p=ir.Stochastic(1, lambda a, b: ir.Beta(a, b)),
        lam=ir.Stochastic(1, lambda g, th: ir.Gamma(g, th)),
        g=ir.Stochastic(lambda: ir.Exponential(2.0)),
        th=ir.Stochastic(lambda: ir.InverseGamma(3.0, 2.0)),
        a=ir.Stochastic(lambda: ir.Uniform(0.5, 4.0)),
        b=ir.Stochastic(lambda m0: ir.Normal(m0, 2.0)),
        m0=ir.Stochastic(lambda: ir.Normal(3.0, 1.0)))


ZOO_DATA = {"nn": [10.0, 12, 7, 20], "t": [1.0, 2.5, 0.5, 4.0, 1.5]}
ZOO_FIXED = {"obs_bin": [3.0, 0, 7, 11], "obs_poi": [0.0, 4, 1, 9, 2], "obs_ber": [1.0, 0, 1]}


def zoo_ref_lp(blockparams, v, transform):
    """logpdf!(m, x, block, transform) by scipy: params \\ targets, then targets."""
    p, lam, g, th, a, b, m0 = v["p"], v["lam"], v["g"], v["th"], v["a"], v["b"], v["m0"]
    node = {
        "obs_bin": lambda: stats.binom.logpmf(ZOO_FIXED["obs_bin"], ZOO_DATA["nn"], p).sum(),
        "obs_poi": lambda: stats.poisson.logpmf(ZOO_FIXED["obs_poi"], lam * np.asarray(ZOO_DATA["t"])).sum(),
        "obs_ber": lambda: stats.bernoulli.logpmf(ZOO_FIXED["obs_ber"], p[0]).sum(),
        "p": lambda: (stats.beta.logpdf(p, a, b) + (np.log(p * (1 - p)) if tr("p") else 0)).sum(),
        "lam": lambda: (stats.gamma.logpdf(lam, g, scale=th) + (np.log(lam) if tr("lam") else 0)).sum(),
        "g": lambda: stats.expon.logpdf(g, scale=2.0) + (np.log(g) if tr("g") else 0),
        "th": lambda: stats.invgamma.logpdf(th, 3.0, scale=2.0) + (np.log(th) if tr("th") else 0),
        "a": lambda: stats.uniform.logpdf(a, 0.5, 3.5) + (np.log((a - 0.5) * (4 - a) / 3.5) if tr("a") else 0),
        "b": lambda: stats.norm.logpdf(b, m0, 2.0),
        "m0": lambda: stats.norm.logpdf(m0, 3.0, 1.0),
    }
    children = {"p": ["obs_bin", "obs_ber"], "lam": ["obs_poi"], "g": ["lam"], "th": ["lam"], "a": ["p"],
                "b": ["p"], "m0": ["b"]}

    def tr(n):
        return transform and n in blockparams

    targets = {c for q in blockparams for c in children[q]}
    order = ["obs_bin", "obs_poi", "obs_ber", "p", "lam", "g", "th", "a", "b", "m0"]
    topo = ["g", "th", "a", "m0", "lam", "b", "obs_poi", "p", "obs_bin", "obs_ber"]
    assert set(topo) == set(order)
    lp = 0.0
    for n in [q for q in blockparams if q not in targets] + [t for t in topo if t in targets]:
        lp += float(node[n]())
    return lp


def test_ir_families_vs_scipy(mamba, oracle):
    m = zoo(mamba).setinputs(ZOO_DATA)
    schemes = [mamba.AMWG(["p", "a"], 0.1), mamba.Slice(["lam", "g", "th"], 1.0, transform=True),
               mamba.Slice(["b", "m0"], 1.0), mamba.NUTS(["g", "th", "lam"])]
    m.setsamplers(schemes)
    rng = np.random.default_rng(7)
    inits = []
    for k in range(6):
        inits.append({**ZOO_FIXED, "p": rng.uniform(0.05, 0.95, 4), "lam": rng.gamma(2.0, 1.0, 5),
                      "g": rng.gamma(2.0, 1.0), "th": rng.gamma(2.0, 1.0), "a": rng.uniform(0.6, 3.9),
                      "b": rng.normal(3, 1), "m0": rng.normal(3, 1)})
    V = m.init_matrix(inits, 6)
    names = ["p", "lam", "g", "th", "a", "b", "m0"]
    off = {n: m.nodes[n].offset for n in names}
    ln = {n: m.nodes[n].dim for n in names}
    links = {"p": (expit, lambda x: np.log(x / (1 - x))), "lam": (np.exp, np.log), "g": (np.exp, np.log),
             "th": (np.exp, np.log), "a": (lambda y: 3.5 * expit(y) + 0.5, lambda x: np.log((x - 0.5) / (4 - x))),
             "b": (lambda y: y, lambda x: x), "m0": (lambda y: y, lambda x: x)}
    for k in range(6):
        vals = {n: V[k, off[n]:off[n] + ln[n]] for n in names}
        vals = {n: (v if ln[n] > 1 else float(v[0])) for n, v in vals.items()}
        for bi, s in enumerate(schemes):
            trf = s.kind != mamba.abi.MMB_SAMPLER_SLICE or bool(s.transform)
            new = {n: vals[n] * (1.0 + rng.normal(0, 0.02, np.shape(vals[n]))) for n in s.params}
            x = np.concatenate([np.atleast_1d(links[n][1](new[n]) if trf else new[n]) for n in s.params])
            got = oracle.block_logpdf(m, V[k], bi, x)
            v2 = dict(vals)
            v2.update({n: (np.atleast_1d(links[n][0](links[n][1](np.asarray(new[n])))) if trf else
                           np.atleast_1d(new[n])) for n in s.params})
            v2 = {n: (np.asarray(v) if np.size(v) > 1 else float(np.ravel(v)[0])) for n, v in v2.items()}
            want = zoo_ref_lp(s.params, v2, trf)
            assert got == pytest.approx(want, rel=1e-11, abs=1e-10), (k, s.params)
    # out of support -> -Inf, and the early exit leaves it there
    x = np.array([0.5, 0.5, 0.5, 5.0])   # a = 5 is outside Uniform(0.5, 4) (AMWG block uses link: use Slice)
    ms = zoo(mamba).setinputs(ZOO_DATA).setsamplers([mamba.Slice(["p", "a"], 1.0)])
    Vs = ms.init_matrix(inits, 1)
    assert oracle.block_logpdf(ms, Vs[0], 0, x) == -np.inf


def test_ir_forward_difference_gradient(mamba, oracle):
    m = mamba.ir.surgical_model().setinputs(mamba.ir.SURGICAL)
    m.setsamplers([mamba.NUTS("b"), mamba.Slice(["mu", "s2"], 1.0)])
    inits = [{"r": mamba.ir.SURGICAL["r"], "b": np.linspace(-3, -2, 12), "s2": 0.3, "mu": -2.5}]
    V = m.init_matrix(inits, 1)
    x = np.linspace(-3.2, -1.9, 12)
    lp, g = oracle.block_logpdf(m, V[0], 0, x, grad=True)
    assert lp == oracle.block_logpdf(m, V[0], 0, x)
    for k in range(12):  # Calculus :forward, epsilon = sqrt(eps) * max(1, |x|), bit for bit
        e = 2.0 ** -26 * max(1.0, abs(x[k]))
        xp = x.copy()
        xp[k] = x[k] + e
        assert g[k] == (oracle.block_logpdf(m, V[0], 0, xp) - lp) / e
    # against the analytic gradient (loose: forward differences)
    p = expit(x)
    mu, s2 = -2.5, 0.3
    r, n = np.asarray(mamba.ir.SURGICAL["r"], float), np.asarray(mamba.ir.SURGICAL["n"], float)
    ga = r - n * p - (x - mu) / s2
    np.testing.assert_allclose(g, ga, rtol=1e-5, atol=1e-4)


def test_ir_lowering_structure(mamba):
    m = mamba.ir.seeds_model().setinputs(mamba.ir.SEEDS)
    m.setsamplers([mamba.AMM(["alpha0", "alpha1", "alpha2", "alpha12"], 0.01 * np.eye(4)), mamba.AMWG("b", 0.01),
                   mamba.AMWG("s2", 0.1)])
    m.init_matrix(mamba.ir.seeds_inits(), 2)
    ir = m.ir()
    assert m.nvalues == 4 + 21 + 1
    assert m.monitor_names == ["alpha0", "alpha1", "alpha2", "alpha12", "s2"]
    ids = {n: i for i, n in enumerate(m.order)}
    terms = [[ir.blocks[b].term[t] for t in range(ir.blocks[b].nterms)] for b in range(3)]
    # params \ targets in block order (their own priors), then the targets (simulation.jl:82-88)
    assert terms[0] == [ids[a] for a in ("alpha0", "alpha1", "alpha2", "alpha12")] + [ids["r"]]
    assert [s.targets for s in m.samplers] == [["r"], ["r"], ["b"]]
    assert terms[1] == [ids["b"], ids["r"]] and terms[2] == [ids["s2"], ids["b"]]
    assert [ir.blocks[2].trans[t] for t in range(2)] == [1, 0]


def test_ir_lowering_errors(mamba):
    ir = mamba.ir
    m = ir.seeds_model().setinputs(ir.SEEDS)
    with pytest.raises(mamba.ArgumentError, match="Gibbs"):
        m.setsamplers([mamba.Gibbs("s2")])
    with pytest.raises(mamba.ArgumentError, match="not a Stochastic node"):
        m.setsamplers([mamba.AMWG("nope", 1.0)])
    m.setsamplers([mamba.AMWG("r", 1.0)])
    with pytest.raises(mamba.ArgumentError, match="cannot be sampled"):
        m.init_matrix(ir.seeds_inits(), 2)
    with pytest.raises(mamba.ArgumentError, match="missing initial value"):
        m.setsamplers([mamba.AMWG("s2", 1.0)]).init_matrix([{"s2": 1.0}], 1)
    big = ir.Model(v=ir.Stochastic(1, lambda: ir.Normal(0, 1)))
    big.setinputs({}).setsamplers([mamba.AMWG("v", 1.0)])
    with pytest.raises(mamba.ArgumentError, match="at most 32"):
        big.init_matrix([{"v": np.zeros(40)}], 1)
    bad = ir.Model(v=ir.Stochastic(1, lambda s: ir.Uniform(0, s)), s=ir.Stochastic(lambda: ir.Gamma(1, 1)))
    bad.setinputs({}).setsamplers([mamba.AMWG("v", 1.0), mamba.AMWG("s", 1.0)])
    with pytest.raises(mamba.ArgumentError, match="Uniform bounds"):
        bad.init_matrix([{"v": np.ones(3), "s": 2.0}], 1)
    mm = ir.Model(y=ir.Stochastic(1, lambda mu, x: ir.MvNormal(mu * x, 1.0), False),
                  mu=ir.Stochastic(1, lambda: ir.Normal(0, 1)))
    mm.setinputs({"x": [1.0, 2, 3]}).setsamplers([mamba.AMWG("mu", 1.0)])
    with pytest.raises(mamba.ArgumentError, match="length"):
        mm.init_matrix([{"y": [1.0, 2, 3], "mu": [0.0, 1.0]}], 1)
    # code-word operands are 24 bits: a pool offset >= 2^24 would carry into the opcode
    W = mamba.ir._Lowering.word
    assert W(5, (1 << 24) - 1) == (5 << 24) | 0xffffff
    for bad_arg in (1 << 24, -1):
        with pytest.raises(mamba.ArgumentError, match="24 bits"):
            W(5, bad_arg)


def test_ir_create_validates_before_touching_the_device(mamba):
    """mmb_create_ir checks every code word / range on the host (no GPU here)."""
    import ctypes as C
    lib = mamba.abi.lib()
    m = mamba.ir.pumps_model().setinputs(mamba.ir.PUMPS)
    m.setsamplers([mamba.Slice(["alpha", "beta"], 1.0, mamba.Univariate), mamba.Slice("theta", 1.0, mamba.Univariate)])
    m.init_matrix([{"y": mamba.ir.PUMPS["y"], "alpha": 1.0, "beta": 1.0, "theta": np.ones(10)}], 1)
    h = C.c_void_p()
    sp = m.spec()
    assert lib.mmb_create(C.byref(sp), 0, C.byref(h)) == -1            # IR needs mmb_create_ir
    ir = m.ir()
    keep = m._ir_keep["code"].copy()
    try:
        m._ir_keep["code"][0] = (3 << 24) | 1000                        # VALI out of the state row
        assert lib.mmb_create_ir(C.byref(sp), C.byref(ir), 0, C.byref(h)) == -1
        assert b"invalid code" in lib.mmb_last_error(None)
    finally:
        m._ir_keep["code"][:] = keep
    sp.blocks[0].sampler = mamba.abi.MMB_SAMPLER_GIBBS
    assert lib.mmb_create_ir(C.byref(sp), C.byref(ir), 0, C.byref(h)) == -2


def _jit_source(mamba, m):
    import ctypes as C
    lib = mamba.abi.lib()
    spec, irm = m.spec(), m.ir()
    n = lib.mmb_ir_jit_source_text(C.byref(spec), C.byref(irm), None, 0)
    buf = C.create_string_buffer(n + 1)
    lib.mmb_ir_jit_source_text(C.byref(spec), C.byref(irm), buf, n + 1)
    return buf.value.decode()


def test_ir_specialised_source_is_straight_line(mamba):
    """mmb_create_ir's specialisation (csrc/ir_jit.cpp): the rats model with the reference scheme
    as HIP source -- y's MvNormal over the 150 observations with its mean alpha[rat] + beta[rat] *
    (x[j] - xbar) as four statements (two gathers, a data load, a multiply-add pair in the
    interpreter's order), one function per node and one case per block, no code-word dispatch,
    the sweep kernel instantiated for the scheme's sampler kinds only (Slice + AMWG)."""
    ir = mamba.ir
    m = ir.rats_model().setinputs(ir.rats_inputs()).setsamplers(mamba.model.rats_scheme_reference())
    m.init_matrix([{**mamba.model.RATS_INITS[k % 2], "y": mamba.model.RATS_Y} for k in range(2)], 2)
    src = _jit_source(mamba, m)
    assert "ir_code" not in src and "mmb_jit_block_lp" in src
    assert src.count("case ") >= len(m.samplers)
    kinds = 0
    for s in m.samplers:
        kinds |= 1 << s.kind
    assert f"sweep_body<MMB_MODEL_IR, {kinds}u>" in src
    # the y node's mean: gather alpha, gather beta, the data column, t3 * t4, t2 + t5
    assert "const double t5 = t3 * t4;" in src and "const double t6 = t2 + t5;" in src
    assert "d_iso(150, sig, ss)" in src


def test_ir_specialised_kernel_compiles_without_a_device(mamba):
    """hipRTC compiles the specialised kernel on the CPU build host (mmb_ir_jit_prebuild: the
    same validation as mmb_create_ir, then compile into the code-object cache)."""
    import ctypes as C
    ir = mamba.ir
    m = ir.line_model().setinputs(mamba.model.LINE_DATA).setsamplers([mamba.AMWG(["beta", "s2"], 1.0)])
    v = mamba.model.line_init_matrix(2, seed=1)
    m.init_matrix([{"y": [1.0, 3, 3, 3, 5], "beta": v[k, :2], "s2": v[k, 2]} for k in range(2)], 2)
    lib = mamba.abi.lib()
    buf = C.create_string_buffer(8192)
    rc = lib.mmb_ir_jit_prebuild(C.byref(m.spec()), C.byref(m.ir()), buf, len(buf))
    assert rc == 0, buf.value.decode()
    assert buf.value.decode().startswith(("cache hit", "compiled in"))
