"""Adversarial GPU parity for the round-4 fast paths:

* the 32-lane pivoted Cholesky's optimistic pass + post-hoc check + checked redo (samplers.h
  pchol32) on crafted matrices -- exact and high-word diagonal ties, zero / negative pivots at
  step 0 and mid-factorization, NaN and +inf entries, magnitudes of 2^+-750 and subnormals --
  against the oracle's dpstf2 restatement (oracle.c orc_pchol; amm.jl:87 cholfact(..., Val{true})
  = LAPACK dpstf2 for n < 64): rank, factor and pivot order bit for bit, and the redo must fire;
* the same cases reached through the AMM update itself: rats tune rows written by mmb_set_tune
  so that the moment matrix Mvv - Mv Mv' (amm.jl:81-90) has ties, huge entries, NaN and negative
  pivots; draws, values, tune and the factorization counters equal the oracle's;
* the lane-parallel AMWG decision (samplers.h amwg_lanes) with accept uniforms placed a few ulps
  to 2^-12 off each coordinate's threshold exp(d_j) (MMB_AMWG_PROBE=1, mmb_math.h
  mmb_amwg_probe_factor, kernels and oracle alike): both certain and uncertain decisions occur,
  and every mode (default, MMB_AMWG_EXACT=1) equals the oracle bit for bit (amwg.jl:99-115)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rats(mamba, scheme):
    m = mamba.rats()
    m.setinputs(mamba.model.RATS_DATA)
    return m.setsamplers(scheme)


def spd(rng, d, scale=1.0):
    A = rng.normal(0.0, 1.0, (d, d + 3))
    return scale * (A @ A.T) / d


def crafted(d, rng):
    """(label, matrix) pairs; lower triangles are what the device reads, the oracle gets the
    symmetric matrix."""
    out = []
    for i in range(4):
        out.append(("spd", spd(rng, d)))
    out.append(("tie_exact_identity", np.eye(d) * 2.0 ** 100))
    out.append(("tie_exact_scaled", np.eye(d) * 3.0))
    S = spd(rng, d)
    np.fill_diagonal(S, S.diagonal().max() * 1.5)  # every diagonal equal, off-diagonals random
    out.append(("tie_exact_dense", S))
    S = np.eye(d) * (1.0 + np.arange(d) * 2.0 ** -40)  # high words equal, low words ordered
    out.append(("tie_highword_ascending", S))
    out.append(("tie_highword_descending", np.eye(d) * (1.0 + np.arange(d)[::-1] * 2.0 ** -40)))
    S = spd(rng, d)
    k = int(np.argmax(S.diagonal()))
    j = (k + 3) % d
    S[j, j] = np.nextafter(S[k, k], 0.0)  # one ulp below the maximum: the high words tie
    out.append(("tie_highword_one_ulp", S))
    out.append(("zero_matrix", np.zeros((d, d))))
    out.append(("negative_diag", -np.eye(d)))
    S = spd(rng, d)
    S[0, 0] = -1.0
    out.append(("negative_pivot_candidate", S))
    v = 2.0 ** rng.integers(-3, 4, d)
    out.append(("rank1_exact_zero_remainder", np.outer(v, v)))  # step 1's remaining diagonal is 0
    B = spd(rng, d // 2 + 1)[: d // 2, : d // 2]
    S = np.zeros((d, d))
    h = d // 2
    S[:h, :h] = S[h:2 * h, h:2 * h] = S[:h, h:2 * h] = S[h:2 * h, :h] = B  # duplicated rows
    if d % 2:
        S[-1, -1] = 1.0
    out.append(("duplicated_rows", S))
    S = spd(rng, d)
    S[2, 2] = np.nan
    out.append(("nan_diag", S))
    S = spd(rng, d)
    S[d - 1, 1] = np.nan
    out.append(("nan_offdiag", S))
    S = spd(rng, d)
    S[1, 1] = np.inf
    out.append(("inf_diag", S))
    out.append(("huge_2p750", spd(rng, d, 2.0 ** 750)))
    out.append(("tiny_2m750", spd(rng, d, 2.0 ** -750)))
    D = np.diag(2.0 ** np.where(np.arange(d) % 2 == 0, 370.0, -370.0))
    out.append(("mixed_scales", D @ spd(rng, d) @ D))
    out.append(("subnormal", spd(rng, d, 2.0 ** -1060)))
    S = spd(rng, d)
    S[4, 4] = -0.0
    out.append(("negative_zero_diag", S))
    S = spd(rng, d)
    S[0, 0] = 2.0 ** -710  # a tiny (positive) pivot candidate below the fast range
    S[0, 1:] = S[1:, 0] = 0.0
    out.append(("tiny_pivot", S))
    return out


@pytest.mark.parametrize("d", [30, 17, 5])
def test_pchol_probe_matches_dpstf2(mamba, oracle, d):
    rng = np.random.default_rng(100 + d)
    cases = crafted(d, rng)
    S = np.stack([c[1] for c in cases])
    rank, redone, L, piv = mamba.abi.debug_pchol(S)
    must_redo = ("tie_exact", "tie_highword", "nan", "inf", "huge", "tiny", "mixed", "subnormal")
    for c, (label, M) in enumerate(cases):
        ro, Lo, po = oracle.pchol(np.tril(M) + np.tril(M, -1).T)
        assert rank[c] == ro, (label, rank[c], ro)
        if ro == d:
            Lo = Lo.reshape(d, d)
            np.testing.assert_array_equal(piv[c], po, err_msg=label)
            np.testing.assert_array_equal(L[c], Lo, err_msg=label)
        if label.startswith(must_redo) and not (label == "tie_exact_scaled" and d == 1):
            assert redone[c] == 1, (label, d)
        if label == "spd":
            assert redone[c] == 0, label
    assert rank[[i for i, c in enumerate(cases) if c[0] == "rank1_exact_zero_remainder"][0]] == 1


def _amm_tune_slices(mamba, m):
    """Per AMM block: (offset in the tune row, d)."""
    out, off = [], 0
    for s in m.samplers:
        d = m.block_dim(s)
        if s.kind == mamba.abi.MMB_SAMPLER_AMM:
            out.append((off, d))
            off += 4 + 2 * d + d * (d + 1)
        elif s.kind == mamba.abi.MMB_SAMPLER_AMWG:
            off += 2 + 2 * d
    return out


def _craft_tune(tune, off, d, kind, rng):
    """Write an AMM tune row (adapt, m, valid, alias, Mv, Mvv, Ls, piv) so that the next adaptive
    update's moment matrix Mvv' - Mv' Mv'^T has the wanted structure: with m = 2^30 the weight
    1 - p of the new draw is 2^-30, so against entries of 2^100 (or Mv = 0) the draw's contribution
    rounds away and the crafted structure survives exactly."""
    T = d * (d + 1) // 2
    tri = lambda i: i * (i + 1) // 2  # noqa: E731
    t = tune[off:off + 4 + 2 * d + 2 * T]
    t[0], t[1], t[2], t[3] = 1.0, float(2 ** 30), 0.0, 0.0
    Mv = t[4:4 + d]
    Mvv = t[4 + d:4 + d + T]
    Mv[:] = 0.0
    Mvv[:] = 0.0
    big = 2.0 ** 100
    if kind == "tie_exact":
        for i in range(d):
            Mvv[tri(i) + i] = big
    elif kind == "tie_highword":
        for i in range(d):
            Mvv[tri(i) + i] = big * (1.0 + ((i * 7) % d) * 2.0 ** -40)
    elif kind == "huge":
        A = rng.normal(0.0, 1.0, (d, d + 3))
        S = (A @ A.T) / d * 2.0 ** 750
        for i in range(d):
            Mvv[tri(i):tri(i) + i + 1] = S[i, :i + 1]
    elif kind == "nan":
        for i in range(d):
            Mvv[tri(i) + i] = big
        Mvv[tri(d - 2) + 3] = np.nan
    elif kind == "negative":
        for i in range(d):
            Mvv[tri(i) + i] = -big
    elif kind == "dup":  # duplicated rows: exact zero remainders after the first pivot of a pair
        for i in range(d):
            for k in range(i + 1):
                Mvv[tri(i) + k] = big if (i // 2 == k // 2) else 0.0
    else:
        raise ValueError(kind)


KINDS = ["tie_exact", "tie_highword", "huge", "nan", "negative", "dup"]


def test_amm_crafted_moments_match_oracle(mamba, oracle):
    """Rats Gibbs+AMM with each chain's AMM tune rows crafted (mmb_set_tune; the oracle's tune
    row the same): the factorizations of the first adaptive updates meet ties, huge entries, NaN,
    negative and exactly-zero pivots.  Draws, values, tune and the AMM counters equal the oracle's;
    the checked redo fires."""
    m = rats(mamba, mamba.model.rats_scheme_gibbs_amm())
    K = 6 * 64
    init = mamba.model.rats_init_ls(16384, seed=1000)[:K]
    rng = np.random.default_rng(7)
    eng = mamba.Engine(m)
    eng.init_chains(init, seed=91)
    st = oracle.new_state(m, init)
    tune = eng.tune()
    np.testing.assert_array_equal(tune, st["tune"][:, :st["tl"]])
    for c in range(K):
        kind = KINDS[c % len(KINDS)]
        for off, d in _amm_tune_slices(mamba, m):
            _craft_tune(tune[c], off, d, kind, rng)
    eng.set_tune(tune)
    st["tune"][:, :st["tl"]] = tune
    oracle.amm_stats(reset=True)
    dg = eng.run(6, burnin=0, thin=1)
    do = oracle.run(m, st, 6, burnin=0, thin=1, seed=91, nthreads=8)
    np.testing.assert_array_equal(dg, do)
    np.testing.assert_array_equal(eng.values(), st["values"])
    tg, to = eng.tune(), st["tune"][:, :st["tl"]]
    np.testing.assert_array_equal(np.isnan(tg), np.isnan(to))
    np.testing.assert_array_equal(np.nan_to_num(tg, nan=0.0), np.nan_to_num(to, nan=0.0))
    sg, so = eng.amm_stats(), oracle.amm_stats(reset=True)
    for b in sg:
        assert (sg[b]["updates"], sg[b]["full_rank"], sg[b]["rank_sum"]) == \
            (so[b]["updates"], so[b]["full_rank"], so[b]["rank_sum"]), (b, sg[b], so[b])
        assert sg[b]["redo"] > 0, sg[b]
        assert 0 < sg[b]["full_rank"] < sg[b]["updates"]


def test_amwg_near_threshold_uniforms_match_oracle(mamba, oracle, monkeypatch):
    """Reference rats scheme with MMB_AMWG_PROBE=1: each alpha / beta coordinate's accept uniform
    is exp(d_j)(1 + k 2^-52), |k| from 0 to 2^40 (mmb_amwg_probe_factor), so decisions sit a few
    ulps from the threshold.  The lane-parallel decision must either be certain and right or fall
    back; both happen, and default and sequential-only runs equal the oracle bit for bit."""
    monkeypatch.setenv("MMB_AMWG_PROBE", "1")
    m = rats(mamba, mamba.model.rats_scheme_reference())
    init = mamba.model.rats_init_matrix(512)
    iters = 40
    st = oracle.new_state(m, init)
    do = oracle.run(m, st, iters, burnin=0, thin=1, seed=5, nthreads=8)
    seq = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MMB_AMWG_EXACT", mode)
        eng = mamba.Engine(m)
        eng.init_chains(init, seed=5)
        dg = eng.run(iters, burnin=0, thin=1)
        np.testing.assert_array_equal(dg, do)
        np.testing.assert_array_equal(eng.values(), st["values"])
        np.testing.assert_array_equal(eng.tune(), st["tune"][:, :st["tl"]])
        seq[mode] = eng.amwg_stats()["sequential_updates"]
    updates = 2 * init.shape[0] * iters
    # mode 0 of the probe (half the block updates) is decided lane-parallel, mode 1 falls back
    assert 0.1 * updates < seq["0"] < 0.9 * updates, seq
    # without the probe the same run takes the same draws from Philox: the probe changed them
    monkeypatch.delenv("MMB_AMWG_PROBE")
    monkeypatch.setenv("MMB_AMWG_EXACT", "0")
    eng = mamba.Engine(m)
    eng.init_chains(init, seed=5)
    assert not np.array_equal(eng.run(iters, burnin=0, thin=1), do)
