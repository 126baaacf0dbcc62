"""ctypes mirror of include/mamba_hip.h and the loader of libmambahip.so.

The product path is the HIP engine only: if the shared library is missing (not
built, or built without a GPU-capable runtime) every entry point raises
RuntimeError -- there is no CPU fallback.
"""
import ctypes as C
import os

MMB_MAX_BLOCKS = 8
MMB_AMM_STATS = 5
MMB_MAX_NODES_PER_BLOCK = 4

MMB_MODEL_LINE, MMB_MODEL_RATS, MMB_MODEL_LOGISTIC, MMB_MODEL_IR = 1, 2, 3, 4
MMB_SAMPLER_AMWG, MMB_SAMPLER_AMM, MMB_SAMPLER_NUTS, MMB_SAMPLER_SLICE, MMB_SAMPLER_GIBBS = 1, 2, 3, 4, 5
MMB_SAMPLER_HMC, MMB_SAMPLER_MALA = 6, 7
MMB_ABI_VERSION = 9
MMB_GRAD_DEFAULT, MMB_GRAD_FORWARD, MMB_GRAD_ANALYTIC = 0, 1, 2
MMB_SUMMARY_FIELDS, MMB_ORDER_MAX_TARGETS = 10, 16
MMB_ADAPT_ALL, MMB_ADAPT_BURNIN, MMB_ADAPT_NONE = 0, 1, 2
MMB_SLICE_MULTIVARIATE, MMB_SLICE_UNIVARIATE = 0, 1
MMB_LINE_BETA, MMB_LINE_S2 = 0, 1
(MMB_RATS_S2_C, MMB_RATS_ALPHA, MMB_RATS_MU_ALPHA, MMB_RATS_S2_ALPHA, MMB_RATS_BETA, MMB_RATS_MU_BETA,
 MMB_RATS_S2_BETA) = range(7)
MMB_LOGISTIC_BETA = 0

# node IR (include/mamba_hip.h)
(MMB_IR_NORMAL, MMB_IR_ISONORMAL, MMB_IR_INVGAMMA, MMB_IR_GAMMA, MMB_IR_EXPONENTIAL, MMB_IR_UNIFORM, MMB_IR_BETA,
 MMB_IR_BINOMIAL, MMB_IR_POISSON, MMB_IR_BERNOULLI, MMB_IR_LOGICAL) = range(1, 12)
IR_OP = {"end": 0, "const": 1, "val": 2, "vali": 3, "valg": 4, "data": 5, "datas": 6,
         "+": 16, "-": 17, "*": 18, "/": 19,
         "neg": 32, "exp": 33, "log": 34, "sqrt": 35, "invlogit": 36, "logit": 37, "abs": 38}
MMB_IR_MAX_STACK, MMB_IR_MAX_TERMS, MMB_IR_MAX_VALUES = 16, 16, 512

ERRORS = {-1: "invalid argument", -2: "unsupported model/scheme", -3: "HIP runtime error",
          -4: "call out of order", -5: "out of memory", -6: "RCCL error"}
MMB_COMM_ID_BYTES = 128


class BlockSpec(C.Structure):
    _fields_ = [("sampler", C.c_int32), ("nnodes", C.c_int32),
                ("nodes", C.c_int32 * MMB_MAX_NODES_PER_BLOCK), ("adapt", C.c_int32),
                ("form", C.c_int32), ("transform", C.c_int32), ("batchsize", C.c_int32),
                ("target", C.c_double), ("beta", C.c_double), ("scale", C.c_double),
                ("dim", C.c_int32), ("ntuning", C.c_int32), ("tuning", C.POINTER(C.c_double)),
                ("epsilon", C.c_double), ("nsteps", C.c_int32), ("gradient", C.c_int32)]


class ModelSpec(C.Structure):
    _fields_ = [("model", C.c_int32), ("nblocks", C.c_int32),
                ("blocks", BlockSpec * MMB_MAX_BLOCKS), ("nobs", C.c_int32), ("ncoef", C.c_int32),
                ("prior_sd", C.c_double), ("reserved", C.c_int32 * 8)]


class IrNode(C.Structure):
    _fields_ = [("family", C.c_int32), ("fixed", C.c_int32), ("off", C.c_int32), ("len", C.c_int32),
                ("expr", C.c_int32 * 3), ("cterm", C.c_int32), ("lo", C.c_double), ("hi", C.c_double)]


class IrBlock(C.Structure):
    _fields_ = [("nterms", C.c_int32), ("term", C.c_int32 * MMB_IR_MAX_TERMS),
                ("trans", C.c_int32 * MMB_IR_MAX_TERMS)]


class IrModel(C.Structure):
    _fields_ = [("nvalues", C.c_int32), ("nnodes", C.c_int32), ("nodes", C.POINTER(IrNode)),
                ("ncode", C.c_int32), ("code", C.POINTER(C.c_int32)), ("nconst", C.c_int32),
                ("consts", C.POINTER(C.c_double)), ("npool", C.c_int64), ("pool", C.POINTER(C.c_double)),
                ("nmon", C.c_int32), ("mon", C.POINTER(C.c_int32)), ("stack", C.c_int32),
                ("blocks", IrBlock * MMB_MAX_BLOCKS)]


class RunArgs(C.Structure):
    _fields_ = [("iters", C.c_int64), ("burnin", C.c_int64), ("thin", C.c_int64),
                ("model_burnin", C.c_int64), ("draws", C.POINTER(C.c_double)),
                ("keep_device", C.c_int32), ("time_kernels", C.c_int32)]


PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MMB_LIB") or os.path.join(PKG_DIR, "lib", "libmambahip.so")
_lib = None


def _declare(lib):
    P, D, I64, I32 = C.c_void_p, C.POINTER(C.c_double), C.c_int64, C.c_int32
    sig = {
        "mmb_abi_version": (C.c_int, []),
        "mmb_create": (C.c_int, [C.POINTER(ModelSpec), C.c_int, C.POINTER(C.c_void_p)]),
        "mmb_create_ir": (C.c_int, [C.POINTER(ModelSpec), C.POINTER(IrModel), C.c_int, C.POINTER(C.c_void_p)]),
        "mmb_destroy": (None, [P]),
        "mmb_last_error": (C.c_char_p, [P]),
        "mmb_set_data": (C.c_int, [P, C.c_char_p, D, I64]),
        "mmb_num_values": (C.c_int, [P]),
        "mmb_num_monitored": (C.c_int, [P]),
        "mmb_init_chains": (C.c_int, [P, D, I64, I64, C.c_uint64]),
        "mmb_run": (C.c_int, [P, C.POINTER(RunArgs)]),
        "mmb_iter": (I64, [P]),
        "mmb_set_iter": (C.c_int, [P, I64]),
        "mmb_get_values": (C.c_int, [P, D]),
        "mmb_set_values": (C.c_int, [P, D]),
        "mmb_tune_len": (I64, [P]),
        "mmb_get_tune": (C.c_int, [P, D]),
        "mmb_set_tune": (C.c_int, [P, D]),
        "mmb_num_kept": (I64, [P]),
        "mmb_get_draws": (C.c_int, [P, D]),
        "mmb_reserve_draws": (C.c_int, [P, I64]),
        "mmb_gr_range": (C.c_int, [P, D]),
        "mmb_gr_len": (I64, [P]),
        "mmb_gr_partials": (C.c_int, [P, C.POINTER(I32), D, D]),
        "mmb_chain_summary": (C.c_int, [P, D, I64, I64, D]),
        "mmb_order_hist": (C.c_int, [P, C.c_int, C.c_int, C.POINTER(C.c_uint64), C.c_int, C.POINTER(C.c_uint64)]),
        "mmb_sync": (C.c_int, [P]),
        "mmb_kernel_time": (C.c_int, [P, D, C.POINTER(I64), C.POINTER(I64)]),
        "mmb_state_bytes": (C.c_int, [P, D]),
        "mmb_grad_evals": (C.c_int, [P, C.POINTER(I64)]),
        "mmb_nuts_stats": (C.c_int, [P, C.POINTER(I64)]),
        "mmb_amm_stats": (C.c_int, [P, C.POINTER(I64)]),
        "mmb_amwg_stats": (C.c_int, [P, C.POINTER(I64)]),
        "mmb_chain_order": (C.c_int, [P, C.POINTER(C.c_int32)]),
        "mmb_debug_pchol": (C.c_int, [C.c_int, I64, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                      C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
        "mmb_ir_jit_info": (C.c_int, [P, C.c_char_p, I64]),
        "mmb_ir_jit_prebuild": (C.c_int, [C.POINTER(ModelSpec), C.POINTER(IrModel), C.c_char_p, I64]),
        "mmb_ir_jit_source_text": (C.c_int, [C.POINTER(ModelSpec), C.POINTER(IrModel), C.c_char_p, I64]),
        "mmb_comm_id": (C.c_int, [C.POINTER(C.c_uint8)]),
        "mmb_comm_init": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8), C.POINTER(P)]),
        "mmb_range_allreduce": (C.c_int, [P, D]),
        "mmb_gr_allreduce": (C.c_int, [P, C.POINTER(I32), D, D]),
        "mmb_comm_destroy": (None, [P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def lib():
    """Load libmambahip.so (the HIP engine).  Raises if it is missing: no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP engine not built: {LIB_PATH} missing (run __graft_entry__.build())")
        try:  # pin the HIP runtime torch ships, if torch is present (single runtime per process)
            import torch  # noqa: F401
        except Exception:
            pass
        _lib = _declare(C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL))
        if _lib.mmb_abi_version() != MMB_ABI_VERSION:
            raise RuntimeError("libmambahip.so ABI version mismatch")
    return _lib


def check(rc, eng=None):
    if rc != 0:
        msg = lib().mmb_last_error(eng)
        raise RuntimeError(f"mamba_hip error {rc} ({ERRORS.get(rc, '?')}): "
                           f"{msg.decode() if msg else ''}")
    return rc


def debug_pchol(S, device=0):
    """mmb_debug_pchol: the device's 32-lane pivoted Cholesky (samplers.h pchol32, the AMM update's
    cholfact(Hermitian(S), :U, Val{true})) on matrices S [n, d, d] (lower triangles read).  Returns
    (rank [n], redone [n], L [n, d, d] with L[c, e, k] = element e's factor entry at step k (zero
    unless full rank), piv [n, d] the pivot order)."""
    import numpy as np
    S = np.asarray(S, dtype=np.float64)
    n, d = S.shape[0], S.shape[1]
    tri = lambda i: i * (i + 1) // 2  # noqa: E731
    P = np.zeros((n, 480))
    for i in range(d):
        P[:, tri(i):tri(i) + i + 1] = S[:, i, :i + 1]
    Lp = np.zeros((n, 480))
    pos = np.zeros((n, 32), dtype=np.int32)
    info = np.zeros((n, 2), dtype=np.int32)
    i32 = C.POINTER(C.c_int32)
    check(lib().mmb_debug_pchol(device, n, d, dptr(P), dptr(Lp), pos.ctypes.data_as(i32), info.ctypes.data_as(i32)))
    L = np.zeros((n, d, d))
    piv = np.zeros((n, d), dtype=np.int32)
    for c in range(n):
        if info[c, 0] != d:
            continue
        for e in range(d):
            t = pos[c, e]
            L[c, e, :t + 1] = Lp[c, tri(t):tri(t) + t + 1]
            piv[c, t] = e
    return info[:, 0].copy(), info[:, 1].copy(), L, piv


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))
