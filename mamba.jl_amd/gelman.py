"""Gelman, Rubin and Brooks diagnostic (src/output/gelmandiag.jl:3-60), sharded.

The device reduces each chain's kept draws to the sufficient statistics of
gelmandiag (Engine.gr_partials); those L-vectors are summed over GPUs with one
RCCL all-reduce (torch.distributed, backend "nccl"); this module turns the global
sums into the PSRF / upper limit / MPSRF exactly as gelmandiag.jl does.

L-vector layout for p monitored params (phi = chain mean - shift):
  [m, sum phi (p), sum phi phi' (p*p), sum S2 (p*p), sum s2^2 (p), sum s2*phi (p), sum s2*phi^2 (p)]
"""
import ctypes as C

import numpy as np
from scipy import stats

from . import abi


def link_kinds(minmax):
    """link(c) (src/output/chains.jl:237-246): log for positive, logit if also < 1."""
    kinds = []
    for lo, hi in minmax:
        kinds.append(0 if not lo > 0.0 else (2 if hi < 1.0 else 1))
    return np.array(kinds, dtype=np.int32)


def psrf_from_sums(sums, n, p, alpha=0.05, mpsrf=False):
    sums = np.asarray(sums, dtype=np.float64)
    o = 0
    m = sums[o]; o += 1
    A1 = sums[o:o + p]; o += p
    A2 = sums[o:o + p * p].reshape(p, p); o += p * p
    A3 = sums[o:o + p * p].reshape(p, p); o += p * p
    A4 = sums[o:o + p]; o += p
    A5 = sums[o:o + p]; o += p
    A6 = sums[o:o + p]
    if m < 2:
        raise ValueError("less than 2 chains supplied to gelman diagnostic")
    W = A3 / m
    mphi = A1 / m
    covpsi = (A2 - m * np.outer(mphi, mphi)) / (m - 1)
    B = n * covpsi
    w, b = np.diag(W), np.diag(B)
    s2sum = np.diag(A3)
    phi2sum = np.diag(A2)
    var_w = ((A4 - s2sum**2 / m) / (m - 1)) / m
    var_b = (2.0 / (m - 1)) * b**2
    cov_s2_phi2 = (A6 - s2sum * phi2sum / m) / (m - 1)
    cov_s2_phi = (A5 - s2sum * A1 / m) / (m - 1)
    var_wb = (n / m) * (cov_s2_phi2 - 2.0 * mphi * cov_s2_phi)
    V = ((n - 1) / n) * w + ((m + 1) / (m * n)) * b
    var_V = ((n - 1)**2 * var_w + ((m + 1) / m)**2 * var_b + (2.0 * (n - 1) * (m + 1) / m) * var_wb) / n**2
    df = 2.0 * V**2 / var_V
    B_df = m - 1
    W_df = 2.0 * w**2 / var_w
    R_fixed = (n - 1) / n
    R_random_scale = (m + 1) / (m * n)
    q = 1.0 - alpha / 2.0
    psrf = np.empty((p, 2))
    for i in range(p):
        corr = (df[i] + 3.0) / (df[i] + 1.0)
        R_random = R_random_scale * b[i] / w[i]
        psrf[i, 0] = np.sqrt(corr * (R_fixed + R_random))
        if not np.isnan(R_random):
            R_random *= stats.f.ppf(q, B_df, W_df[i])
        psrf[i, 1] = np.sqrt(corr * (R_fixed + R_random))
    mp = None
    if mpsrf:
        try:
            np.linalg.cholesky(W)
            mp = R_fixed + R_random_scale * float(np.max(np.real(np.linalg.eigvals(np.linalg.solve(W, B)))))
        except np.linalg.LinAlgError:
            mp = float("nan")
    return psrf, mp


def gelmandiag_sharded(engine, allreduce_sum=None, allreduce_minmax=None, transform=False,
                       alpha=0.05, mpsrf=False):
    """PSRF over all chains of all ranks.  `allreduce_sum(x)` / `allreduce_minmax(lo, hi)`
    perform the cross-GPU reductions (identity on a single engine)."""
    p = engine.pmon
    mm = engine.gr_range()
    lo, hi = mm[:, 0].copy(), mm[:, 1].copy()
    if allreduce_minmax is not None:
        lo, hi = allreduce_minmax(lo, hi)
    kinds = link_kinds(zip(lo, hi)) if transform else np.zeros(p, dtype=np.int32)
    mid = 0.5 * (lo + hi)
    shift = mid.copy()
    shift[kinds == 1] = np.log(mid[kinds == 1])
    shift[kinds == 2] = np.log(mid[kinds == 2] / (1.0 - mid[kinds == 2]))
    local = engine.gr_partials(kinds, shift)
    tot = allreduce_sum(local) if allreduce_sum is not None else local
    n = engine.num_kept()
    return psrf_from_sums(tot, n, p, alpha=alpha, mpsrf=mpsrf)


def gelmandiag(chains, alpha=0.05, mpsrf=False, transform=False):
    """Host gelmandiag on an n x p x m array (reference formula, gelmandiag.jl:3-60)."""
    psi = np.asarray(chains.value if hasattr(chains, "value") else chains, dtype=np.float64)
    n, p, m = psi.shape
    if m < 2:
        raise ValueError("less than 2 chains supplied to gelman diagnostic")
    if transform:
        psi = psi.copy()
        for j in range(p):
            x = psi[:, j, :]
            if x.min() > 0:
                psi[:, j, :] = np.log(x / (1 - x)) if x.max() < 1 else np.log(x)
    means = psi.mean(0)                               # p x m
    S2 = np.einsum("ijk,ilk->jlk", psi - means, psi - means) / (n - 1)
    phi = means.T                                     # m x p
    s2 = np.stack([np.diag(S2[:, :, k]) for k in range(m)])
    sums = np.concatenate([[m], phi.sum(0), (phi.T @ phi).ravel(), S2.sum(2).ravel(),
                           (s2**2).sum(0), (s2 * phi).sum(0), (s2 * phi**2).sum(0)])
    return psrf_from_sums(sums, n, p, alpha=alpha, mpsrf=mpsrf)


class Comm:
    """The library's own RCCL communicator (include/mamba_hip.h mmb_comm_*): the one
    cross-GPU collective of the path, reachable from any C caller.

    Comm([e0, e1, ...])                       one process driving all its GPUs (ncclCommInitAll)
    Comm([e], nranks=N, rank0=r, uid=bytes)   one process per GPU; rank 0 makes `uid` with
                                              Comm.unique_id() and the caller broadcasts it
    """

    def __init__(self, engines, nranks=None, rank0=0, uid=None):
        self.lib = abi.lib()
        self.engines = list(engines)
        n = len(self.engines)
        nranks = n if nranks is None else int(nranks)
        arr = (C.c_void_p * n)(*[e.h for e in self.engines])
        idp = None
        if uid is not None:
            if len(uid) != abi.MMB_COMM_ID_BYTES:
                raise ValueError(f"unique id must be {abi.MMB_COMM_ID_BYTES} bytes")
            idp = (C.c_uint8 * abi.MMB_COMM_ID_BYTES)(*uid)
        h = C.c_void_p()
        abi.check(self.lib.mmb_comm_init(arr, n, nranks, int(rank0), idp, C.byref(h)), self.engines[0].h)
        self.h = h

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * abi.MMB_COMM_ID_BYTES)()
        abi.check(abi.lib().mmb_comm_id(buf))
        return bytes(buf)

    def range_allreduce(self):
        """Global [min, max] per monitored param over every chain of every rank (p x 2)."""
        p = self.engines[0].pmon
        out = np.empty(2 * p)
        abi.check(self.lib.mmb_range_allreduce(self.h, abi.dptr(out)), self.engines[0].h)
        return out.reshape(p, 2)

    def gr_allreduce(self, kinds, shift):
        """Global Gelman-Rubin sufficient statistics (mmb_gr_len doubles)."""
        kinds = np.ascontiguousarray(kinds, dtype=np.int32)
        shift = np.ascontiguousarray(shift, dtype=np.float64)
        out = np.empty(self.lib.mmb_gr_len(self.engines[0].h))
        abi.check(self.lib.mmb_gr_allreduce(self.h, kinds.ctypes.data_as(C.POINTER(C.c_int32)), abi.dptr(shift),
                                            abi.dptr(out)), self.engines[0].h)
        return out

    def close(self):
        if getattr(self, "h", None):
            self.lib.mmb_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gelmandiag_rccl(comm, transform=False, alpha=0.05, mpsrf=False):
    """gelmandiag over every chain of every rank of `comm`, all reductions inside the
    library (RCCL): one MAX all-reduce for the range, one SUM all-reduce of the sums."""
    eng = comm.engines[0]
    mm = comm.range_allreduce()
    kinds = link_kinds(mm) if transform else np.zeros(eng.pmon, dtype=np.int32)
    mid = 0.5 * (mm[:, 0] + mm[:, 1])
    shift = mid.copy()
    shift[kinds == 1] = np.log(mid[kinds == 1])
    shift[kinds == 2] = np.log(mid[kinds == 2] / (1.0 - mid[kinds == 2]))
    tot = comm.gr_allreduce(kinds, shift)
    return psrf_from_sums(tot, eng.num_kept(), eng.pmon, alpha=alpha, mpsrf=mpsrf)
