"""ctypes binding of oracle/liboracle.so — the CPU restatement used as the CHECKER.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return LIB


class Oracle:
    def __init__(self):
        import _mamba_path
        self.abi = _mamba_path.load().abi
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(ORACLE_DIR, "oracle.c")):
            build_oracle()
        L = C.CDLL(LIB)
        D, I64, P = C.POINTER(C.c_double), C.c_int64, C.POINTER(self.abi.ModelSpec)
        DD = C.POINTER(C.POINTER(C.c_double))
        L.orc_tune_len.restype = I64
        L.orc_tune_len.argtypes = [P, DD, C.POINTER(I64)]
        L.orc_init_tune.argtypes = [P, DD, C.POINTER(I64), D, I64]
        L.orc_run.argtypes = [P, DD, C.POINTER(I64), I64, I64, C.c_uint64, D, D, I64, I64, I64, I64,
                              I64, D, C.c_int]
        L.orc_block_logpdf.restype = C.c_double
        L.orc_block_logpdf.argtypes = [P, DD, C.POINTER(I64), D, C.c_int, D]
        L.orc_block_logpdf_grad.restype = C.c_double
        L.orc_block_logpdf_grad.argtypes = [P, DD, C.POINTER(I64), D, C.c_int, D, D]
        L.orc_pivoted_cholesky.argtypes = [C.c_int, D, D, C.POINTER(C.c_int)]
        for f in ("orc_log", "orc_exp", "orc_log1p", "orc_exp_neg"):
            getattr(L, f).restype = C.c_double
            getattr(L, f).argtypes = [C.c_double]
        L.orc_sincos2pi.argtypes = [C.c_double, D, D]
        L.orc_logistic_row.argtypes = [C.c_double, C.c_double, D, D, D]
        L.orc_lg_lane_lp.restype = C.c_double
        L.orc_lg_lane_lp.argtypes = [C.c_double, C.c_double, C.c_int]
        L.orc_philox.argtypes = [C.POINTER(C.c_uint32)] * 3
        for f in ("orc_uniform", "orc_normal"):
            getattr(L, f).restype = C.c_double
            getattr(L, f).argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_set_ir.argtypes = [C.c_void_p]
        L.orc_lgamma.restype = C.c_double
        L.orc_lgamma.argtypes = [C.c_double]
        L.orc_ir_elem_lp.restype = C.c_double
        L.orc_ir_elem_lp.argtypes = [C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, C.c_int,
                                     C.c_double, C.c_double]
        L.orc_gamma.restype = C.c_double
        L.orc_gamma.argtypes = [C.c_double, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_amm_stats.argtypes = [C.POINTER(C.c_int64)]
        L.orc_amm_stats_reset.argtypes = []
        self.L = L

    def _ir(self, model):
        """Node-IR models: hand the lowered mmb_ir_model to the oracle (orc_set_ir)."""
        if model.kind == self.abi.MMB_MODEL_IR:
            self.L.orc_set_ir(C.addressof(model.ir()))

    @staticmethod
    def _data(model):
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in model.data_arrays()]
        ptrs = (C.POINTER(C.c_double) * len(arrs))(*[a.ctypes.data_as(C.POINTER(C.c_double)) for a in arrs])
        ns = (C.c_int64 * len(arrs))(*[a.size for a in arrs])
        return arrs, ptrs, ns

    def new_state(self, model, init):
        self._ir(model)
        spec = model.spec()
        arrs, ptrs, ns = self._data(model)
        K = init.shape[0]
        tl = self.L.orc_tune_len(C.byref(spec), ptrs, ns)
        if tl < 0:
            raise ValueError(f"oracle rejected spec ({tl})")
        tune = np.zeros((K, max(tl, 1)))
        rc = self.L.orc_init_tune(C.byref(spec), ptrs, ns, tune.ctypes.data_as(C.POINTER(C.c_double)), K)
        assert rc == 0
        return {"values": np.ascontiguousarray(init, dtype=np.float64).copy(), "tune": tune, "tl": tl,
                "iter": 0}

    def run(self, model, state, iters, burnin=0, thin=1, model_burnin=None, chain_offset=0, seed=1,
            nthreads=1, draws=True):
        self._ir(model)
        spec = model.spec()
        arrs, ptrs, ns = self._data(model)
        K = state["values"].shape[0]
        it0 = state["iter"]
        kept = lambda t: (t - burnin) // thin if t > burnin else 0  # noqa: E731
        nk = kept(it0 + iters) - kept(it0)
        pmon = len(model.monitor_names)
        dr = np.zeros((max(nk, 1), pmon, K)) if draws else None
        rc = self.L.orc_run(C.byref(spec), ptrs, ns, K, chain_offset, C.c_uint64(seed),
                            state["values"].ctypes.data_as(C.POINTER(C.c_double)),
                            state["tune"].ctypes.data_as(C.POINTER(C.c_double)),
                            it0, iters, burnin, thin, burnin if model_burnin is None else model_burnin,
                            dr.ctypes.data_as(C.POINTER(C.c_double)) if draws else None, nthreads)
        assert rc == 0, rc
        state["iter"] = it0 + iters
        if not draws or nk == 0:
            return None
        # [n][p][K] -> Mamba Chains order n x p x K
        return np.asfortranarray(dr[:nk])

    def block_logpdf(self, model, values, block, x, grad=False):
        self._ir(model)
        spec = model.spec()
        arrs, ptrs, ns = self._data(model)
        v = np.ascontiguousarray(values, dtype=np.float64)
        xx = np.ascontiguousarray(x, dtype=np.float64)
        dp = C.POINTER(C.c_double)
        if grad:
            g = np.zeros_like(xx)
            lp = self.L.orc_block_logpdf_grad(C.byref(spec), ptrs, ns, v.ctypes.data_as(dp), block,
                                              xx.ctypes.data_as(dp), g.ctypes.data_as(dp))
            return lp, g
        return self.L.orc_block_logpdf(C.byref(spec), ptrs, ns, v.ctypes.data_as(dp), block, xx.ctypes.data_as(dp))

    def amm_stats(self, reset=False):
        """Per-block AMM counters since the last reset: (cholfact calls, rank == n, rank sum)."""
        v = (C.c_int64 * (8 * 3))()
        self.L.orc_amm_stats(v)
        if reset:
            self.L.orc_amm_stats_reset()
        return {b: {"updates": v[3 * b], "full_rank": v[3 * b + 1], "rank_sum": v[3 * b + 2]}
                for b in range(8) if v[3 * b]}

    def pchol(self, S):
        d = S.shape[0]
        S = np.ascontiguousarray(S, dtype=np.float64)
        L = np.zeros((d, d))
        piv = np.zeros(d, dtype=np.int32)
        dp = C.POINTER(C.c_double)
        r = self.L.orc_pivoted_cholesky(d, S.ctypes.data_as(dp), L.ctypes.data_as(dp),
                                        piv.ctypes.data_as(C.POINTER(C.c_int)))
        return r, L, piv

    def philox(self, ctr, key):
        c = (C.c_uint32 * 4)(*ctr)
        k = (C.c_uint32 * 2)(*key)
        o = (C.c_uint32 * 4)()
        self.L.orc_philox(c, k, o)
        return list(o)
