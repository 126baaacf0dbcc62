"""Posterior summaries: summarystats / mcse_bm / quantile.

CPU tests: the oracle restatement (oracle/summary_ref.py) pinned by hand-checkable
cases; the host pooling of the device partials (mamba.jl_amd/summary.py) against it,
fed by an engine-shaped host shard whose partials/histograms restate the kernels'
contracts (include/mamba_hip.h mmb_chain_summary / mmb_order_hist); and the sharded
path at world size 2 over gloo, with the rank boundary inside a batch.  The device
kernels themselves are checked in tests/test_gpu_parity.py.
"""
import math
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import summary_ref  # noqa: E402


def _keys(x):
    """The order-preserving uint64 key of a double (summary.hip os_key)."""
    u = np.ascontiguousarray(x, dtype=np.float64).view(np.uint64)
    top = np.uint64(1) << np.uint64(63)
    return np.where(u & top, ~u, u | top)


class HostSummaryShard:
    """Engine-shaped view of n x p x k draws of global chains [off, off + k)."""

    def __init__(self, draws, chain_offset=0):
        self.d = np.asarray(draws, dtype=np.float64)
        self.pmon, self.K = self.d.shape[1], self.d.shape[2]
        self.chain_offset = chain_offset

    def num_kept(self):
        return self.d.shape[0]

    def gr_range(self):
        return np.stack([self.d.min(axis=(0, 2)), self.d.max(axis=(0, 2))], axis=1)

    def chain_summary(self, shift, batch_size=100, chain_base=0):
        return summary_ref.chain_partials(self.d, chain_base + np.arange(self.K), batch_size, shift)

    def order_hist(self, param, prefixes, npass):
        k = _keys(self.d[:, param, :].ravel())
        dsh = np.uint64(56 - 8 * npass)
        dg = (k >> dsh) & np.uint64(255)
        hi = k >> (dsh + np.uint64(8)) if npass else np.zeros_like(k)
        out = np.zeros((len(prefixes), 256), dtype=np.uint64)
        for t, pf in enumerate(prefixes):
            sel = hi == np.uint64(pf)
            out[t] = np.bincount(dg[sel].astype(np.int64), minlength=256)
        return out


def make_draws(n=375, p=3, m=10, seed=11):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, p, m)).cumsum(0) * 0.05 + rng.normal(size=(1, p, m))  # autocorrelated
    d[:, 1, :] = np.exp(d[:, 1, :]) * 30.0
    d[:, 2, :] -= 100.0                      # all negative
    d[::7, 0, :] = 0.25                      # ties
    return d


# ---- the oracle, pinned ---------------------------------------------------------------
def test_mcse_bm_batch_constant_series():
    """A series constant within each batch: mcse_bm = std(batch values)/sqrt(m) exactly."""
    vals = np.array([1.0, 4.0, -2.0, 0.5, 3.0])
    x = np.repeat(vals, 100)
    assert summary_ref.mcse_bm(x) == pytest.approx(vals.std(ddof=1) / math.sqrt(5), rel=1e-15)
    with pytest.raises(ValueError, match="iterations are < 200"):
        summary_ref.mcse_bm(np.ones(199))


def test_summarystats_ref_against_numpy():
    d = make_draws()
    ss = summary_ref.summarystats(d)
    for j in range(d.shape[1]):
        v = d[:, j, :].ravel(order="F")
        assert ss[j, 0] == pytest.approx(v.mean(), rel=1e-13)
        assert ss[j, 1] == pytest.approx(v.std(ddof=1), rel=1e-12)
        assert ss[j, 2] == pytest.approx(v.std(ddof=1) / math.sqrt(v.size), rel=1e-12)
        mb = v[:v.size // 100 * 100].reshape(-1, 100).mean(1)
        assert ss[j, 3] == pytest.approx(mb.std(ddof=1) / math.sqrt(mb.size), rel=1e-11)
        assert ss[j, 4] == min((ss[j, 1] / ss[j, 3]) ** 2, d.shape[0])


def test_quantile_ref_against_numpy_linear():
    d = make_draws()
    q = (0.0, 0.025, 0.25, 0.5, 0.75, 0.975, 1.0)
    got = summary_ref.quantile(d, q)
    for j in range(d.shape[1]):
        np.testing.assert_allclose(got[j], np.quantile(d[:, j, :].ravel(), q), rtol=1e-15, atol=0)


# ---- host pooling of the device partials ----------------------------------------------
@pytest.mark.parametrize("n,bs,m", [(375, 100, 8), (1000, 100, 5), (50, 100, 9), (7, 3, 11), (200, 100, 2)])
def test_pool_summary_single_engine(mamba, n, bs, m):
    d = make_draws(n=n, m=m, seed=n + m)
    got = mamba.summarystats_sharded(HostSummaryShard(d), batch_size=bs)
    ref = summary_ref.summarystats(d, bs)
    np.testing.assert_allclose(got[:, :4], ref[:, :4], rtol=1e-10)
    np.testing.assert_allclose(got[:, 4], ref[:, 4], rtol=1e-8)


def test_pool_summary_too_few_batches(mamba):
    with pytest.raises(mamba.ArgumentError, match="iterations are < 200"):
        mamba.summarystats_sharded(HostSummaryShard(make_draws(n=30, m=3)), batch_size=100)


def test_quantile_by_radix_select(mamba):
    d = make_draws(n=301, m=7)
    q = (0.025, 0.25, 0.5, 0.75, 0.975, 0.0, 1.0)
    got = mamba.quantile_sharded(HostSummaryShard(d), q)
    np.testing.assert_array_equal(got, summary_ref.quantile(d, q))
    ranks = [0, 5, 1000, d.shape[0] * d.shape[2] - 1]
    s = np.sort(d[:, 2, :].ravel())
    np.testing.assert_array_equal(mamba.summary.order_stats(HostSummaryShard(d), 2, ranks), s[ranks])


# ---- sharded: world size 2 over gloo ---------------------------------------------------
def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import _mamba_path
        mb = _mamba_path.load()
        d = make_draws()
        m = d.shape[2]
        lo, hi = (0, 3) if rank == 0 else (3, m)  # uneven; boundary at flat 3*375: mid-batch
        shard = HostSummaryShard(d[:, :, lo:hi], chain_offset=lo)

        def ar_sum(x):
            t = torch.tensor(np.asarray(x, dtype=np.float64))
            dist.all_reduce(t)
            return t.numpy()

        def ar_minmax(a, b):
            t = torch.tensor(np.concatenate([-a, b]), dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t = t.numpy()
            return -t[:len(a)], t[len(a):]

        def gather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out

        ss = mb.summarystats_sharded(shard, 100, allreduce_sum=ar_sum, allgather=gather, allreduce_minmax=ar_minmax)
        qs = mb.quantile_sharded(shard, allreduce_sum=ar_sum)
        if rank == 0:
            q.put((ss, qs))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_summary_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ss, qs = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = make_draws()
    ref = summary_ref.summarystats(d)
    np.testing.assert_allclose(ss[:, :4], ref[:, :4], rtol=1e-10)
    np.testing.assert_allclose(ss[:, 4], ref[:, 4], rtol=1e-8)
    np.testing.assert_array_equal(qs, summary_ref.quantile(d))
