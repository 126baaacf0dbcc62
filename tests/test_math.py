"""Pin the shared RNG / elementary-function layer (mmb_math.h) independently:
Philox4x32-10 against Random123's known-answer vectors and rocRAND's engine
(tests/golden/philox_kat.json), exp/log/log1p/sincos against libm (numpy)."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_philox_known_answers(oracle):
    kat = json.load(open(os.path.join(GOLD, "philox_kat.json")))
    for case in kat["random123"] + kat["rocrand"]:
        assert oracle.philox(case["ctr"], case["key"]) == case["out"]


def ulps(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    ia = a.view(np.int64)
    ib = b.view(np.int64)
    ia = np.where(ia < 0, np.int64(-0x8000000000000000) - ia, ia)
    ib = np.where(ib < 0, np.int64(-0x8000000000000000) - ib, ib)
    return np.abs(ia - ib)


@pytest.mark.parametrize("fn,npf,gen", [
    ("orc_log", np.log, lambda r: np.exp(r.uniform(-700, 700, 20000))),
    ("orc_log", np.log, lambda r: r.uniform(0.5, 2.0, 20000)),
    ("orc_exp", np.exp, lambda r: r.uniform(-740, 709, 20000)),
    ("orc_exp", np.exp, lambda r: r.uniform(-1, 1, 20000)),
    ("orc_log1p", np.log1p, lambda r: np.exp(r.uniform(-40, 3, 20000))),
    ("orc_exp_neg", np.exp, lambda r: r.uniform(-745, 0, 20000)),
    ("orc_exp_neg", np.exp, lambda r: -np.exp(r.uniform(-60, 0, 20000))),
])
def test_elementary_within_one_ulp(oracle, fn, npf, gen):
    x = gen(np.random.default_rng(7))
    f = getattr(oracle.L, fn)
    got = np.array([f(float(v)) for v in x])
    ref = npf(x)
    bad = ulps(got, ref)
    tol = 2 if fn == "orc_log1p" else 1
    assert bad.max() <= tol, (x[bad.argmax()], got[bad.argmax()], ref[bad.argmax()])


def test_elementary_special_values(oracle):
    L = oracle.L
    assert L.orc_log(0.0) == -np.inf and np.isnan(L.orc_log(-1.0)) and L.orc_log(np.inf) == np.inf
    assert L.orc_log(1.0) == 0.0 and L.orc_exp(0.0) == 1.0
    assert L.orc_exp(800.0) == np.inf and L.orc_exp(-800.0) == 0.0 and L.orc_exp(-np.inf) == 0.0
    assert np.isnan(L.orc_exp(np.nan))
    # logistic-term kernels (x <= 0, t in [0, 1])
    assert L.orc_exp_neg(0.0) == 1.0 and L.orc_exp_neg(-800.0) == 0.0 and L.orc_exp_neg(-np.inf) == 0.0
    assert np.isnan(L.orc_exp_neg(np.nan)) and L.orc_exp_neg(-745.1) == 5e-324
    assert abs(L.orc_log(5e-324) - np.log(5e-324)) < 1e-12  # subnormal path


def test_sincos2pi(oracle):
    import ctypes as C
    u = np.random.default_rng(3).random(20000)
    s = C.c_double()
    c = C.c_double()
    err = 0.0
    for v in u:
        oracle.L.orc_sincos2pi(float(v), C.byref(s), C.byref(c))
        err = max(err, abs(s.value - np.sin(2 * np.pi * v)), abs(c.value - np.cos(2 * np.pi * v)))
    assert err < 2e-15


def test_uniform_and_normal_streams(oracle):
    L = oracle.L
    u = np.array([L.orc_uniform(11, 5, 3, 2, 1, k) for k in range(40000)])
    assert 0.0 <= u.min() and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.006 and abs(u.var() - 1 / 12) < 0.002
    z = np.array([L.orc_normal(11, 5, 3, 2, 0, k) for k in range(40000)])
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02
    assert abs(np.mean(z**3)) < 0.05 and abs(np.mean(z**4) - 3) < 0.15
    # distinct streams per (chain, iter, block, substream)
    assert L.orc_uniform(11, 5, 3, 2, 1, 0) != L.orc_uniform(11, 6, 3, 2, 1, 0)
    assert L.orc_uniform(11, 5, 3, 2, 1, 0) != L.orc_uniform(11, 5, 4, 2, 1, 0)
    assert L.orc_uniform(11, 5, 3, 2, 1, 0) != L.orc_uniform(11, 5, 3, 3, 1, 0)


@pytest.mark.parametrize("a", [1.0, 2.501, 15.001, 75.001])
def test_gamma_marsaglia_tsang(oracle, a):
    g = np.array([oracle.L.orc_gamma(a, 99, c, 1, 0) for c in range(20000)])
    se = np.sqrt(a / 20000)
    assert abs(g.mean() - a) < 5 * se
    assert abs(g.var() / a - 1) < 0.06


def test_logistic_row_accuracy(oracle):
    """mmb_logistic_row (config-4 per-row terms): lin = y*eta - max(eta, 0), a = 1 + exp(-|eta|)
    and res = y - invlogit(eta), against an 80-bit long-double evaluation; lp = lin - log(a)
    (taken once per lane through mmb_lg_lane_lp)."""
    import ctypes as C
    r = np.random.default_rng(11)
    eta = np.concatenate([r.normal(0, 3, 20000), r.uniform(-745, 745, 2000), [0.0, -0.0, 1e-300, -1e-300, 40.0, -40.0]])
    out = {y: [np.empty(eta.size) for _ in range(4)] for y in (0.0, 1.0)}
    lin, a, rs = C.c_double(), C.c_double(), C.c_double()
    for y in (0.0, 1.0):
        o = out[y]
        for k, e in enumerate(eta):
            oracle.L.orc_logistic_row(float(e), y, C.byref(lin), C.byref(a), C.byref(rs))
            o[0][k], o[1][k], o[2][k] = lin.value, a.value, rs.value
            o[3][k] = oracle.L.orc_lg_lane_lp(lin.value, a.value, 0)
    E = eta.astype(np.longdouble)
    t = np.exp(-np.abs(E))
    sp = np.maximum(E, 0) + np.log1p(t)
    sig = np.where(E >= 0, 1 / (1 + t), t / (1 + t))
    for y in (0.0, 1.0):
        got_lin, got_a, got_res, got_lp = out[y]
        assert np.array_equal(got_lin, (y * eta - np.maximum(eta, 0)))
        assert np.abs(got_a - (1 + t).astype(np.float64)).max() <= 2.3e-16
        ref = (y * E - sp).astype(np.float64)
        # absolute error of the per-row lp (a = 1 + t rounds t below 2^-53 away; the row terms
        # are summed, so absolute error is the measure): <= 2^-52 relative to max(|lp|, 1)
        assert (np.abs(got_lp - ref) / np.maximum(np.abs(ref), 1.0)).max() <= 4.5e-16
        assert np.abs(got_res - (y - sig).astype(np.float64)).max() <= 2.3e-16


def test_lane_product_renormalisation_is_exact(oracle):
    """The lane product P 2^E of the (1 + t) factors does not depend on when it is renormalised
    (power-of-two scaling is exact): log of a 4000-factor product (overflows without it)."""
    import ctypes as C
    r = np.random.default_rng(5)
    f = 1.0 + r.uniform(0, 1, 4000)
    P, E = 1.0, 0
    for v in f:
        P = P * v
        m, e = np.frexp(P)          # P = m 2^e, m in [0.5, 1)
        P, E = m * 2.0, E + int(e) - 1
    got = oracle.L.orc_lg_lane_lp(0.0, P, E)
    ref = -float(np.sum(np.log(f.astype(np.longdouble))))
    assert abs(got - ref) <= 1e-9 * abs(ref)
    # every fourth factor instead of every factor: the same bits
    P2, E2 = 1.0, 0
    for k, v in enumerate(f):
        P2 = P2 * v
        if k % 4 == 3:
            m, e = np.frexp(P2)
            P2, E2 = m * 2.0, E2 + int(e) - 1
    assert oracle.L.orc_lg_lane_lp(0.0, P2, E2) == got
