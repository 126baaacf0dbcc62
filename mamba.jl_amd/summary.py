"""Posterior summaries of the device-kept draws, pooled over all chains of all GPUs.

summarystats(c; etype=:bm) (src/output/stats.jl:85-94) and quantile(c)
(src/output/stats.jl:73-80) reduce the n x p x chains draw array per param over
iterations AND chains.  The per-element work runs on the GPU (summary.hip):

* mmb_chain_summary gives, per chain and param, shifted sums and the batch-means terms
  of mcse_bm (src/output/mcse.jl:10-19) for the batches of vec(x) lying inside the chain,
  plus the chain's pieces of the batches it shares with its neighbours.  This module
  joins the pieces (locally, then across GPUs with one all-gather of the few unjoined
  ones), all-reduces the sums and applies the reference formulas:
    Mean = mean(x), SD = std(x), Naive SE = sem(x) = SD/sqrt(N),
    MCSE = sem(batch means of size `bs`), ESS = min((SD/MCSE)^2, n)   [n = iterations]
* quantile: exact order statistics by radix select (mmb_order_hist, 8 passes of one byte,
  counts all-reduced across GPUs), then Julia 0.5 Base.quantile's interpolation
  (index = 1 + (N-1)q, r = (1-h) v[lo] + h v[hi]; recalled from Julia Base, not vendored).

The cross-GPU reductions are callbacks (`allreduce_sum`, `allgather`), identity on one
engine; bench.py / tests pass torch.distributed ones (RCCL or gloo).
"""
import numpy as np

from .samplers import ArgumentError

F_S1, F_Q, F_B1, F_B2, F_NFULL, F_HSUM, F_HCNT, F_TSUM, F_TCNT = range(9)
QUANTILES = (0.025, 0.25, 0.5, 0.75, 0.975)


def _pieces(parts, kg, n, bs):
    """The (batch id, sums[p], count) pieces of batches a chain shares with a neighbour."""
    hmask = parts[:, 0, F_HCNT] > 0
    tmask = parts[:, 0, F_TCNT] > 0
    ids = np.concatenate([(kg[hmask] * n) // bs, (kg[tmask] * n + n - 1) // bs])
    sums = np.concatenate([parts[hmask, :, F_HSUM], parts[tmask, :, F_TSUM]])
    cnts = np.concatenate([parts[hmask, 0, F_HCNT], parts[tmask, 0, F_TCNT]])
    return ids.astype(np.int64), sums, cnts


def _join(ids, sums, cnts, bs):
    """Join pieces by batch id -> (complete batch deviations d_b, unjoined pieces)."""
    p = sums.shape[1] if sums.ndim == 2 else 0
    if ids.size == 0:
        return np.zeros((0, p)), (ids, sums.reshape(0, p), cnts)
    uniq, inv = np.unique(ids, return_inverse=True)
    tot = np.zeros((uniq.size, p))
    np.add.at(tot, inv, sums)
    cnt = np.bincount(inv, weights=cnts, minlength=uniq.size)
    done = cnt == bs
    if np.any(cnt > bs):
        raise RuntimeError("summary: a batch received more than batch_size elements")
    return tot[done] / bs, (uniq[~done], tot[~done], cnt[~done])


def pool_summary(parts, kg, n, bs, shift, allreduce_sum=None, allgather=None):
    """Pool K x p x MMB_SUMMARY_FIELDS chain partials (global chain ids kg, computed with
    `shift`) into the p x 5 summarystats table [Mean, SD, Naive SE, MCSE, ESS]."""
    parts = np.asarray(parts, dtype=np.float64)
    kg = np.asarray(kg, dtype=np.int64)
    K, p, _ = parts.shape
    sums = np.concatenate([parts[:, :, f].sum(0) for f in (F_S1, F_Q, F_B1, F_B2, F_NFULL)] + [[K]])
    d, left = _join(*_pieces(parts, kg, n, bs), bs)
    if allgather is not None:  # the unjoined pieces of every rank (a few per rank)
        allp = allgather(left)
        ids = np.concatenate([a[0] for a in allp])
        sm = np.concatenate([a[1].reshape(-1, p) for a in allp])
        ct = np.concatenate([a[2] for a in allp])
        d2, left = _join(ids, sm, ct, bs)
    else:
        d2 = np.zeros((0, p))
    if allreduce_sum is not None:
        sums = np.asarray(allreduce_sum(sums), dtype=np.float64)
    # pieces joined locally are rank-local sums; those joined from the gather are identical on
    # every rank and are added after the all-reduce
    loc = np.concatenate([d.sum(0), (d * d).sum(0), [d.shape[0]]])
    if allreduce_sum is not None:
        loc = np.asarray(allreduce_sum(loc), dtype=np.float64)
    S1, Q, D1, D2, NF = (sums[i * p:(i + 1) * p] for i in range(5))
    M = int(round(sums[5 * p]))
    D1 = D1 + loc[:p] + d2.sum(0)
    D2 = D2 + loc[p:2 * p] + (d2 * d2).sum(0)
    mb = NF + loc[2 * p] + d2.shape[0]
    N = n * M
    m = N // bs
    if m < 2:  # mcse.jl:13-16
        raise ArgumentError(f"iterations are < {2 * bs} and batch size is > {N // 2}")
    if not np.all(mb == m):
        raise RuntimeError(f"summary: joined {mb} batches, expected {m}")
    mean = shift + S1 / N
    sd = np.sqrt((Q - S1 * S1 / N) / (N - 1))
    sem = sd / np.sqrt(N)
    mcse = np.sqrt((D2 - D1 * D1 / m) / (m - 1) / m)
    ess = np.minimum((sd / mcse) ** 2, n)                  # stats.jl:92 (n = iterations)
    return np.stack([mean, sd, sem, mcse, ess], axis=1)


def _global_chains(engine, allreduce_sum):
    K = engine.K
    tot = float(allreduce_sum(np.array([float(K)]))[0]) if allreduce_sum is not None else float(K)
    return int(round(tot))


def summarystats_sharded(engine, batch_size=100, allreduce_sum=None, allgather=None, allreduce_minmax=None):
    """summarystats(c; etype=:bm) over every chain of every rank, from device-kept draws.
    Two device passes: shifted by the mid-range (-> global mean), then by the mean."""
    n = engine.num_kept()
    mm = engine.gr_range()
    lo, hi = mm[:, 0].copy(), mm[:, 1].copy()
    if allreduce_minmax is not None:
        lo, hi = allreduce_minmax(lo, hi)
    mid = 0.5 * (lo + hi)
    M = _global_chains(engine, allreduce_sum)
    # chains are concatenated in global chain order when sharded, local order alone
    base = engine.chain_offset if allgather is not None else 0
    s1 = engine.chain_summary(mid, batch_size, base)[:, :, F_S1].sum(0)
    if allreduce_sum is not None:
        s1 = np.asarray(allreduce_sum(s1), dtype=np.float64)
    mu = mid + s1 / (n * M)
    kg = base + np.arange(engine.K)
    parts = engine.chain_summary(mu, batch_size, base)
    return pool_summary(parts, kg, n, batch_size, mu, allreduce_sum, allgather)


# ---- exact order statistics by radix select --------------------------------------------
def key_to_double(key):
    key = np.asarray(key, dtype=np.uint64)
    top = np.uint64(1) << np.uint64(63)
    u = np.where(key & top, key & ~top, ~key)
    return u.view(np.float64)


def order_stats(engine, param, ranks, allreduce_sum=None):
    """Exact 0-based order statistics `ranks` of the pooled draws of `param`."""
    ranks = [int(r) for r in ranks]
    prefix = [0] * len(ranks)
    rem = list(ranks)
    for ps in range(8):
        uniq = sorted(set(prefix))
        counts = {}
        for c0 in range(0, len(uniq), 16):
            chunk = uniq[c0:c0 + 16]
            h = engine.order_hist(param, np.array(chunk, dtype=np.uint64), ps)
            if allreduce_sum is not None:
                h = np.asarray(allreduce_sum(h.astype(np.float64))).round().astype(np.uint64)
            for u, row in zip(chunk, h):
                counts[u] = np.cumsum(row.astype(np.int64))
        for t in range(len(ranks)):
            cum = counts[prefix[t]]
            if rem[t] >= cum[-1]:
                raise ArgumentError(f"rank {ranks[t]} out of range")
            dgt = int(np.searchsorted(cum, rem[t], side="right"))
            rem[t] -= int(cum[dgt - 1]) if dgt > 0 else 0
            prefix[t] = (prefix[t] << 8) | dgt
    return key_to_double(np.array(prefix, dtype=np.uint64))


def quantile_sharded(engine, q=QUANTILES, allreduce_sum=None):
    """quantile(c; q) (stats.jl:73-80) pooled over iterations and all chains: p x len(q)."""
    n = engine.num_kept()
    N = n * _global_chains(engine, allreduce_sum)
    q = np.asarray(q, dtype=np.float64)
    index = 1.0 + (N - 1) * q                      # Julia 0.5 quantile!: 1-based
    lo = np.floor(index).astype(np.int64)
    hi = np.ceil(index).astype(np.int64)
    h = index - lo
    ranks = sorted(set((lo - 1).tolist()) | set((hi - 1).tolist()))
    out = np.empty((engine.pmon, q.size))
    for j in range(engine.pmon):
        v = dict(zip(ranks, order_stats(engine, j, ranks, allreduce_sum)))
        for t in range(q.size):
            a, b = v[lo[t] - 1], v[hi[t] - 1]
            out[j, t] = a if index[t] == lo[t] else (1.0 - h[t]) * a + h[t] * b
    return out
