"""mcmc() driver, Engine wrapper and Chains container.

Mirrors src/model/mcmc.jl: `mcmc(m, inputs, inits, iters; burnin, thin, chains)`
(mcmc.jl:19-33) and the restart form `mcmc(mc, iters)` (mcmc.jl:3-16).  The chain
fan-out (`pmap2(mcmc_worker!, ...)`, mcmc.jl:52) is one HIP engine per GPU holding a
contiguous shard of global chain ids; draws come back in Mamba's Chains layout
(n x p x chains, src/output/chains.jl:5-11).
"""
import ctypes as C

import numpy as np

from . import abi
from .samplers import ArgumentError


class Engine:
    """One libmambahip engine (one GPU, one shard of chains)."""

    def __init__(self, model, device=0):
        self.lib = abi.lib()
        self.model = model
        self.spec = model.spec()
        h = C.c_void_p()
        if model.kind == abi.MMB_MODEL_IR:  # generic node IR (ir.py)
            self.ir = model.ir()
            rc = self.lib.mmb_create_ir(C.byref(self.spec), C.byref(self.ir), int(device), C.byref(h))
        else:
            rc = self.lib.mmb_create(C.byref(self.spec), int(device), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"mmb_create failed ({abi.ERRORS.get(rc, rc)}): "
                               f"{self.lib.mmb_last_error(None).decode()}")
        self.h = h
        for name, arr in zip(model.input_names, model.data_arrays()):
            self._chk(self.lib.mmb_set_data(self.h, name.encode(), abi.dptr(arr), arr.size))
        self.P = self.lib.mmb_num_values(self.h)
        self.pmon = self.lib.mmb_num_monitored(self.h)
        self.K = 0

    def _chk(self, rc):
        return abi.check(rc, self.h)

    def close(self):
        if getattr(self, "h", None):
            self.lib.mmb_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def init_chains(self, init, chain_offset=0, seed=1):
        init = np.ascontiguousarray(init, dtype=np.float64)
        self.K = init.shape[0]
        self.chain_offset = int(chain_offset)
        self.seed = int(seed)
        self._chk(self.lib.mmb_init_chains(self.h, abi.dptr(init), self.K, int(chain_offset),
                                           C.c_uint64(int(seed))))

    def run(self, iters, burnin=0, thin=1, model_burnin=None, draws=True, keep_device=False,
            time_kernels=False):
        a = abi.RunArgs()
        a.iters, a.burnin, a.thin = int(iters), int(burnin), int(thin)
        a.model_burnin = int(burnin if model_burnin is None else model_burnin)
        a.keep_device = int(keep_device)
        a.time_kernels = int(time_kernels)
        it0 = self.iter
        kept = lambda t: (t - burnin) // thin if t > burnin else 0  # noqa: E731
        nk = kept(it0 + iters) - kept(it0)
        out = None
        if draws and nk > 0:
            out = np.empty((nk, self.pmon, self.K), order="F")
            a.draws = abi.dptr(out)
        self._chk(self.lib.mmb_run(self.h, C.byref(a)))
        return out

    def reserve_draws(self, nkept):
        """Allocate the device draw buffer for windows keeping up to `nkept` iterations now
        (mmb_reserve_draws), so a later run does not allocate inside a timed window."""
        self._chk(self.lib.mmb_reserve_draws(self.h, int(nkept)))

    @property
    def iter(self):
        return self.lib.mmb_iter(self.h)

    def set_iter(self, it):
        self._chk(self.lib.mmb_set_iter(self.h, int(it)))

    def values(self):
        v = np.empty((self.K, self.P))
        self._chk(self.lib.mmb_get_values(self.h, abi.dptr(v)))
        return v

    def set_values(self, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        self._chk(self.lib.mmb_set_values(self.h, abi.dptr(v)))

    def tune(self):
        n = self.lib.mmb_tune_len(self.h)
        t = np.empty((self.K, max(n, 1)))
        if n > 0:
            self._chk(self.lib.mmb_get_tune(self.h, abi.dptr(t)))
        return t[:, :n]

    def set_tune(self, t):
        t = np.ascontiguousarray(t, dtype=np.float64)
        if t.size:
            self._chk(self.lib.mmb_set_tune(self.h, abi.dptr(t)))

    def num_kept(self):
        return self.lib.mmb_num_kept(self.h)

    def draws(self):
        nk = self.num_kept()
        out = np.empty((nk, self.pmon, self.K), order="F")
        if nk:
            self._chk(self.lib.mmb_get_draws(self.h, abi.dptr(out)))
        return out

    def sync(self):
        self._chk(self.lib.mmb_sync(self.h))

    def kernel_time(self):
        ms = C.c_double()
        n = C.c_int64()
        u = C.c_int64()
        self.lib.mmb_kernel_time(self.h, C.byref(ms), C.byref(n), C.byref(u))
        return ms.value, n.value, u.value

    def grad_evals(self):
        n = C.c_int64()
        self._chk(self.lib.mmb_grad_evals(self.h, C.byref(n)))
        return n.value

    def nuts_stats(self):
        """NUTS tree statistics since init_chains (mmb_nuts_stats): completed updates,
        updates stopped by the depth cap (reference: unbounded), mean final tree depth."""
        v = (C.c_int64 * 3)()
        self._chk(self.lib.mmb_nuts_stats(self.h, v))
        return {"updates": v[0], "depth_cap_hits": v[1], "depth_sum": v[2]}

    def amm_stats(self):
        """AMM factorization counters since init_chains (mmb_amm_stats), one dict per AMM block
        (keyed by block index): adaptive updates (cholfact calls, amm.jl:87), full-rank ones
        (rank(F) == n: SigmaLm replaced, amm.jl:88-90), the rank sum, the factorization steps
        the device executed (per wavefront of two chains on the 32-lane kernels) and the updates
        whose optimistic pass was redone by the checked one."""
        v = (C.c_int64 * (abi.MMB_MAX_BLOCKS * abi.MMB_AMM_STATS))()
        self._chk(self.lib.mmb_amm_stats(self.h, v))
        out = {}
        for b, blk in enumerate(self.model.samplers):
            if getattr(blk, "kind", None) != abi.MMB_SAMPLER_AMM:
                continue
            r = v[b * abi.MMB_AMM_STATS:(b + 1) * abi.MMB_AMM_STATS]
            out[b] = {"updates": r[0], "full_rank": r[1], "rank_sum": r[2], "steps_sum": r[3], "redo": r[4]}
        return out

    def amwg_stats(self):
        """AMWG block updates since init_chains that ran the sequential coordinate loop
        (mmb_amwg_stats) rather than the lane-parallel decision of every coordinate."""
        v = (C.c_int64 * 1)()
        self._chk(self.lib.mmb_amwg_stats(self.h, v))
        return {"sequential_updates": v[0]}

    def chain_order(self):
        """The lane-group slot -> chain table of the last window (mmb_chain_order): the 32-lane
        kernels pair chains whose AMM factorization stops alike; results do not depend on it."""
        out = np.empty(self.K, dtype=np.int32)
        if self.K:
            self._chk(self.lib.mmb_chain_order(self.h, out.ctypes.data_as(C.POINTER(C.c_int32))))
        return out

    def ir_jit(self):
        """Node-IR engines: (True, info) when the specialised kernel runs (mmb_create_ir compiled
        the model with hipRTC or found it in the cache), (False, reason) for the interpreter."""
        buf = C.create_string_buffer(4096)
        r = self.lib.mmb_ir_jit_info(self.h, buf, len(buf))
        if r < 0:
            self._chk(r)
        return bool(r), buf.value.decode()

    def state_bytes(self):
        b = C.c_double()
        self.lib.mmb_state_bytes(self.h, C.byref(b))
        return b.value

    # Gelman-Rubin partial sums of the device-kept draws (for the cross-GPU all-reduce)
    def gr_range(self):
        mm = np.empty(2 * self.pmon)
        self._chk(self.lib.mmb_gr_range(self.h, abi.dptr(mm)))
        return mm.reshape(self.pmon, 2)

    def gr_partials(self, link, shift):
        link = np.ascontiguousarray(link, dtype=np.int32)
        shift = np.ascontiguousarray(shift, dtype=np.float64)
        out = np.empty(self.lib.mmb_gr_len(self.h))
        self._chk(self.lib.mmb_gr_partials(self.h, link.ctypes.data_as(C.POINTER(C.c_int32)),
                                           abi.dptr(shift), abi.dptr(out)))
        return out

    # posterior-summary partials of the device-kept draws (summary.py pools them)
    def chain_summary(self, shift, batch_size=100, chain_base=0):
        shift = np.ascontiguousarray(shift, dtype=np.float64)
        out = np.empty((self.K, self.pmon, abi.MMB_SUMMARY_FIELDS))
        self._chk(self.lib.mmb_chain_summary(self.h, abi.dptr(shift), int(batch_size), int(chain_base),
                                             abi.dptr(out)))
        return out

    def order_hist(self, param, prefixes, npass):
        pre = np.ascontiguousarray(prefixes, dtype=np.uint64)
        out = np.empty((pre.size, 256), dtype=np.uint64)
        u64 = C.POINTER(C.c_uint64)
        self._chk(self.lib.mmb_order_hist(self.h, int(param), int(pre.size), pre.ctypes.data_as(u64), int(npass),
                                          out.ctypes.data_as(u64)))
        return out


class Chains:
    """Chains / ModelChains (src/output/chains.jl:5-11, modelchains.jl): value is
    n x p x chains, names the monitored nodes, range = start:thin:stop."""

    def __init__(self, value, names, start, thin, chains, model=None, engine=None):
        self.value = value
        self.names = list(names)
        self.start, self.thin = int(start), int(thin)
        self.chains = np.asarray(chains)
        self.model = model
        self.engine = engine

    @property
    def range(self):
        n = self.value.shape[0]
        return range(self.start, self.start + n * self.thin, self.thin)

    def __getitem__(self, name):
        return self.value[:, self.names.index(name), :]

    def _device_engine(self):
        eng = self.engine
        if eng is None or eng.h is None or eng.num_kept() != self.value.shape[0] or self.value.shape[0] == 0:
            raise ArgumentError("summaries run on the device-kept draws: sample with keep_device=True "
                                "(the engine holds the last window's draws)")
        return eng

    def summarystats(self, batch_size=100):
        """summarystats(c; etype=:bm) (stats.jl:85-94): p x [Mean, SD, Naive SE, MCSE, ESS]."""
        from .summary import summarystats_sharded
        return summarystats_sharded(self._device_engine(), batch_size)

    def quantile(self, q=(0.025, 0.25, 0.5, 0.75, 0.975)):
        """quantile(c; q) (stats.jl:73-80), pooled over iterations and chains: p x len(q)."""
        from .summary import quantile_sharded
        return quantile_sharded(self._device_engine(), q)

    def describe(self, q=(0.025, 0.25, 0.5, 0.75, 0.975), batch_size=100):
        """describe(c) (stats.jl:42-52): summarystats and quantiles per monitored name."""
        ss = self.summarystats(batch_size)
        qs = self.quantile(q)
        labels = ["Mean", "SD", "Naive SE", "MCSE", "ESS"]
        return {nm: {**{lb: float(ss[j, i]) for i, lb in enumerate(labels)},
                     **{f"{100 * x}%": float(qs[j, t]) for t, x in enumerate(q)}}
                for j, nm in enumerate(self.names)}


def mcmc(model, inputs, inits, iters, burnin=0, thin=1, chains=1, verbose=False, device=0,
         chain_offset=0, seed=1, keep_device=False):
    """mcmc(m, inputs, inits, iters; burnin, thin, chains) (mcmc.jl:19-33)."""
    if not iters > burnin:
        raise ArgumentError("burnin is greater than or equal to iters")
    model.setinputs(inputs)
    init = model.init_matrix(inits, chains)
    model.burnin = burnin
    eng = Engine(model, device)
    eng.init_chains(init, chain_offset=chain_offset, seed=seed)
    draws = eng.run(iters, burnin=burnin, thin=thin, model_burnin=burnin, keep_device=keep_device)
    if draws is None:
        draws = np.empty((0, eng.pmon, eng.K))
    model.iter = eng.iter
    return Chains(draws, model.monitor_names, burnin + thin, thin,
                  np.arange(chain_offset + 1, chain_offset + chains + 1), model, eng)


def mcmc_restart(mc, iters, verbose=False):
    """mcmc(mc::ModelChains, iters) (mcmc.jl:3-16): continue from model.states."""
    eng, model = mc.engine, mc.model
    last = mc.range[-1] if mc.value.shape[0] else mc.start - mc.thin
    if last != (model.iter // mc.thin) * mc.thin:
        raise ArgumentError("chain is missing its last iteration")
    draws = eng.run(iters, burnin=last, thin=mc.thin, model_burnin=model.burnin)
    model.iter = eng.iter
    value = np.concatenate([mc.value, draws], axis=0) if draws is not None else mc.value
    return Chains(value, mc.names, mc.start, mc.thin, mc.chains, model, eng)


_CKPT_KIND = "mamba_amd.ModelChains/1"


def write(name, c):
    """write(name, c::AbstractChains) (fileio.jl:10-12): save the chains and, for a
    ModelChains with a live engine, the resumable model state (ModelState values + tune,
    Model.iter, Philox seed, global chain offset, Model.burnin).  The file is a plain
    .npz (no pickled objects): `read(name, model=...)` restores an engine on any device
    and `mcmc_restart` then continues exactly where the writer stopped."""
    arrays = dict(kind=np.array(_CKPT_KIND), value=np.asarray(c.value, dtype=np.float64),
                  names=np.array(c.names, dtype=np.str_), start=np.int64(c.start),
                  thin=np.int64(c.thin), chains=np.asarray(c.chains, dtype=np.int64))
    eng = c.engine
    if eng is not None and getattr(eng, "h", None) is not None and eng.K > 0:
        arrays.update(values=eng.values(), tune=eng.tune(), iter=np.int64(eng.iter),
                      seed=np.uint64(eng.seed), chain_offset=np.int64(eng.chain_offset),
                      model_burnin=np.int64(getattr(c.model, "burnin", 0)))
    with open(name, "wb") as f:  # np.savez would append ".npz" to a bare name
        np.savez(f, **arrays)


def read(name, model=None, device=0):
    """read(name, ModelChains) (fileio.jl:3-8): load chains written by `write`.  With
    `model` (the same Model, inputs set, as the writer's: closures are not serialised),
    the saved state is restored into a new engine on `device`, ready for
    `mcmc_restart(mc, iters)`.  Raises TypeError if the file holds no chains."""
    with np.load(name, allow_pickle=False) as z:
        if "kind" not in z.files or str(z["kind"]) != _CKPT_KIND:
            raise TypeError(f'read("{name}", ModelChains): not a chains file')
        d = {k: z[k] for k in z.files}
    eng = None
    if model is not None:
        if "values" not in d:
            raise ArgumentError("file holds no model state to resume from")
        vals = d["values"]
        eng = Engine(model, device)
        if vals.shape[1] != eng.P:
            eng.close()
            raise ArgumentError(f"saved state has {vals.shape[1]} values per chain, model has {eng.P}")
        eng.init_chains(vals, chain_offset=int(d["chain_offset"]), seed=int(d["seed"]))
        eng.set_tune(d["tune"])
        eng.set_iter(int(d["iter"]))
        model.burnin = int(d["model_burnin"])
        model.iter = int(d["iter"])
    return Chains(d["value"], [str(x) for x in d["names"]], int(d["start"]), int(d["thin"]),
                  d["chains"], model, eng)
