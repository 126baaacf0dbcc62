"""Multi-process (gloo, world size 2) test of the sharded Gelman-Rubin reduction.

The N>1 data path has exactly one exchange (gelmandiag.jl:11-25): each
rank reduces its chains' kept draws to the L-vector of sufficient statistics, the
ranks all-reduce it (SUM) plus the link-function range (MAX), and the PSRF comes out
of the global sums.  Here each rank holds a host shard with the engine's GR interface
(the device kernel gr_stats_kernel computes the same per-chain quantities; its parity
with this host form is tests/test_gpu_parity.py::test_device_gelman_rubin_matches_host).
The collectives are the ones bench.py issues over RCCL, run over gloo on CPU.
test_library_partials_two_processes (-m gpu) runs the same exchange over the library's own
device partials: two processes, each an engine over its shard of global chains on the one
GPU of the box (RCCL refuses two ranks on one device, so the exchange is gloo there).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class HostShard:
    """Engine-shaped view of n x p x k draws (global chains [off, off+k))."""

    def __init__(self, draws):
        self.d = np.asarray(draws, dtype=np.float64)
        self.pmon = self.d.shape[1]

    def num_kept(self):
        return self.d.shape[0]

    def gr_range(self):
        return np.stack([self.d.min(axis=(0, 2)), self.d.max(axis=(0, 2))], axis=1)

    def gr_partials(self, kinds, shift):
        x = self.d.copy()
        for j, kd in enumerate(kinds):
            if kd == 1:
                x[:, j, :] = np.log(x[:, j, :])
            elif kd == 2:
                x[:, j, :] = np.log(x[:, j, :] / (1 - x[:, j, :]))
        n, p, m = x.shape
        mean = x.mean(0)                                   # p x m
        dv = x - mean
        S2 = np.einsum("ijk,ilk->jlk", dv, dv) / (n - 1)  # p x p x m
        phi = (mean - np.asarray(shift)[:, None]).T       # m x p
        s2 = np.stack([np.diag(S2[:, :, k]) for k in range(m)])
        return np.concatenate([[m], phi.sum(0), (phi.T @ phi).ravel(), S2.sum(2).ravel(),
                               (s2 ** 2).sum(0), (s2 * phi).sum(0), (s2 * phi ** 2).sum(0)])


def make_draws(n=200, p=3, m=16, seed=5):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, p, m)) + rng.normal(scale=0.3, size=(1, p, m))
    d[:, 0, :] = np.exp(d[:, 0, :])                 # positive -> log link
    d[:, 2, :] = 1.0 / (1.0 + np.exp(-d[:, 2, :]))  # unit interval -> logit link
    return d


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import _mamba_path
        mb = _mamba_path.load()
        d = make_draws()
        m = d.shape[2]
        lo, hi = rank * m // world, (rank + 1) * m // world
        shard = HostShard(d[:, :, lo:hi])

        def ar_sum(x):
            t = torch.tensor(x, dtype=torch.float64)
            dist.all_reduce(t)
            return t.numpy()

        def ar_minmax(a, b):
            t = torch.tensor(np.concatenate([-a, b]), dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t = t.numpy()
            return -t[:len(a)], t[len(a):]

        out = {}
        for tr in (False, True):
            psrf, mp_ = mb.gelmandiag_sharded(shard, allreduce_sum=ar_sum, allreduce_minmax=ar_minmax,
                                              transform=tr, mpsrf=True)
            out[tr] = (psrf, mp_)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_sharded_gelman_rubin_gloo(world):
    import _mamba_path
    mb = _mamba_path.load()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = make_draws()
    for tr in (False, True):
        ref, ref_mp = mb.gelmandiag(d, transform=tr, mpsrf=True)
        psrf, mp_ = res[tr]
        np.testing.assert_allclose(psrf, ref, rtol=1e-10)
        np.testing.assert_allclose(mp_, ref_mp, rtol=1e-9)


def test_sharded_equals_single_process():
    """World size 1 through the same code path (identity collectives)."""
    import _mamba_path
    mb = _mamba_path.load()
    d = make_draws(m=9)
    for tr in (False, True):
        psrf, _ = mb.gelmandiag_sharded(HostShard(d), transform=tr)
        ref, _ = mb.gelmandiag(d, transform=tr)
        np.testing.assert_allclose(psrf, ref, rtol=1e-10)


def _gpu_worker(rank, world, port, q, K):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import _mamba_path
        mb = _mamba_path.load()
        m = mb.rats()
        m.setinputs(mb.model.RATS_DATA)
        m.setsamplers(mb.model.rats_scheme_gibbs_amm())
        init = mb.model.rats_init_ls(world * K, seed=7)[rank * K:(rank + 1) * K]
        eng = mb.Engine(m, device=0)
        eng.init_chains(init, seed=11, chain_offset=rank * K)
        d = eng.run(120, burnin=40, thin=2, keep_device=True)

        def ar_sum(x):
            t = torch.tensor(x, dtype=torch.float64)
            dist.all_reduce(t)
            return t.numpy()

        def ar_minmax(a, b):
            t = torch.tensor(np.concatenate([-a, b]), dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t = t.numpy()
            return -t[:len(a)], t[len(a):]

        out = {tr: mb.gelmandiag_sharded(eng, allreduce_sum=ar_sum, allreduce_minmax=ar_minmax,
                                         transform=tr, mpsrf=True) for tr in (False, True)}
        q.put((rank, d, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_library_partials_two_processes():
    """Two processes x one engine each (global chains [r K, (r+1) K), chain_offset = r K):
    mmb_gr_range / mmb_gr_partials of each shard, exchanged by all-reduce, give the PSRF of
    the host gelmandiag over all 2K chains' draws (gelmandiag.jl:11-25)."""
    import _mamba_path
    mb = _mamba_path.load()
    world, K = 2, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q, K)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (d, o)) for r, d, o in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = np.concatenate([res[r][0] for r in range(world)], axis=2)
    assert d.shape == (40, 3, world * K)
    for tr in (False, True):
        ref, ref_mp = mb.gelmandiag(d, transform=tr, mpsrf=True)
        for r in range(world):
            psrf, mp_ = res[r][1][tr]
            np.testing.assert_allclose(psrf, ref, rtol=1e-8)
            np.testing.assert_allclose(mp_, ref_mp, rtol=1e-8)
