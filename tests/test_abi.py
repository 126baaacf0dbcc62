"""C ABI boundary checks that run without a GPU: the library loads, exports every
symbol include/mamba_hip.h declares, the ctypes structs match the header layout, and
argument validation (ArgumentError semantics of the reference) happens host-side."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mamba_hip.h")


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*]+\s+)+\**(mmb_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol(mamba):
    lib = mamba.abi.lib()
    out = subprocess.check_output(["nm", "-D", "--defined-only", mamba.abi.LIB_PATH]).decode()
    exported = set(re.findall(r" T (mmb_\w+)", out))
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    assert lib.mmb_abi_version() == mamba.abi.MMB_ABI_VERSION == 9


def test_struct_layout_matches_header(mamba):
    src = """
#include <stddef.h>
#include <stdio.h>
#include "mamba_hip.h"
int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(mmb_block_spec), sizeof(mmb_model_spec),
 sizeof(mmb_run_args), offsetof(mmb_block_spec, tuning), offsetof(mmb_model_spec, prior_sd),
 offsetof(mmb_run_args, keep_device), offsetof(mmb_block_spec, epsilon), offsetof(mmb_block_spec, nsteps));
 return 0;}
"""
    d = "/tmp/mmb_layout"
    os.makedirs(d, exist_ok=True)
    open(f"{d}/t.c", "w").write(src)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", f"{d}/t", f"{d}/t.c"])
    got = list(map(int, subprocess.check_output([f"{d}/t"]).split()))
    a = mamba.abi
    want = [C.sizeof(a.BlockSpec), C.sizeof(a.ModelSpec), C.sizeof(a.RunArgs), a.BlockSpec.tuning.offset,
            a.ModelSpec.prior_sd.offset, a.RunArgs.keep_device.offset, a.BlockSpec.epsilon.offset,
            a.BlockSpec.nsteps.offset]
    assert got == want


def test_create_validates_before_touching_the_device(mamba):
    lib = mamba.abi.lib()
    m = mamba.line()
    m.setsamplers([mamba.AMWG(["beta", "s2"], 1.0)])
    sp = m.spec()
    sp.blocks[0].dim = 7                      # wrong block length
    h = C.c_void_p()
    assert lib.mmb_create(C.byref(sp), 0, C.byref(h)) == -1
    assert b"unlisted length" in lib.mmb_last_error(None)
    r = mamba.rats()
    r.setsamplers([mamba.NUTS("alpha")])                       # NUTS not lowered for rats
    assert lib.mmb_create(C.byref(r.spec()), 0, C.byref(h)) == -2
    r.setsamplers([mamba.Slice(["alpha", "mu_alpha"], 1.0)])   # mixed vector/scalar block
    assert lib.mmb_create(C.byref(r.spec()), 0, C.byref(h)) == -2
    r.setsamplers([mamba.HMC("alpha", 0.1, 5)])                # HMC not lowered for rats
    assert lib.mmb_create(C.byref(r.spec()), 0, C.byref(h)) == -2
    m.setsamplers([mamba.MALA(["beta", "s2"], 0.1, np.eye(3))])
    sp = m.spec()
    sp.blocks[0].ntuning = 4                                   # Sigma of the wrong size
    assert lib.mmb_create(C.byref(sp), 0, C.byref(h)) == -1
    assert b"Sigma dimension" in lib.mmb_last_error(None)
    m.setsamplers([mamba.HMC(["beta", "s2"], 0.1, 3, -np.eye(3))])
    assert lib.mmb_create(C.byref(m.spec()), 0, C.byref(h)) == -1   # cholfact: not PD
    lg = mamba.logistic(10, 3)
    lg.setsamplers([mamba.AMWG("beta", 1.0)])                  # logistic lowers NUTS/HMC/MALA only
    assert lib.mmb_create(C.byref(lg.spec()), 0, C.byref(h)) == -2


def test_python_argument_errors(mamba):
    with pytest.raises(mamba.ArgumentError, match="adapt must be one of"):
        mamba.AMWG("alpha", 1.0, adapt="sometimes")
    m = mamba.rats()
    with pytest.raises(mamba.ArgumentError, match="length\\(sigma\\) differs"):
        m.setsamplers([mamba.AMWG("alpha", [1.0, 2.0])])
    with pytest.raises(mamba.ArgumentError, match="Sigma dimension"):
        m.setsamplers([mamba.AMM("alpha", np.eye(3))])
    with pytest.raises(mamba.ArgumentError, match="Sigma dimension"):
        mamba.line().setsamplers([mamba.HMC(["beta", "s2"], 0.1, 10, np.eye(2))])
    with pytest.raises(mamba.ArgumentError, match="unsupported dtype"):
        mamba.MALA("beta", 0.1, dtype="backward")
    with pytest.raises(mamba.ArgumentError, match="burnin is greater"):
        mamba.mcmc(m.setsamplers([mamba.Gibbs("s2_c")]), mamba.model.RATS_DATA, mamba.model.RATS_INITS, 10,
                   burnin=10)
    with pytest.raises(mamba.ArgumentError, match="fewer initial values"):
        m.setinputs(mamba.model.RATS_DATA).init_matrix(mamba.model.RATS_INITS, 3)


def test_chains_file_round_trip(mamba, tmp_path):
    """write/read (fileio.jl:3-12) of chains without engine state: plain .npz, no pickle."""
    val = np.random.default_rng(0).normal(size=(7, 3, 4))
    c = mamba.Chains(val, ["s2_c", "mu_beta", "alpha0"], 1002, 2, np.arange(1, 5))
    p = str(tmp_path / "sim.chains")
    mamba.write(p, c)
    r = mamba.read(p)
    np.testing.assert_array_equal(r.value, val)
    assert r.names == c.names and r.start == 1002 and r.thin == 2
    assert list(r.range) == list(c.range)
    np.testing.assert_array_equal(r.chains, c.chains)
    with pytest.raises(mamba.ArgumentError):  # no model state saved
        mamba.read(p, model=mamba.rats())
    bad = str(tmp_path / "bad.npz")
    np.savez(bad, value=val)
    with pytest.raises(TypeError):
        mamba.read(bad)


def test_comm_init_validates_before_touching_the_device(mamba):
    """mmb_comm_init rejects bad rank layouts on the host (no GPU, no RCCL call here)."""
    lib = mamba.abi.lib()
    h = C.c_void_p()
    assert lib.mmb_comm_init(None, 1, 1, 0, None, C.byref(h)) == -1
    arr = (C.c_void_p * 1)(None)
    assert lib.mmb_comm_init(arr, 0, 1, 0, None, C.byref(h)) == -1
    assert lib.mmb_comm_init(arr, 1, 1, 0, None, C.byref(h)) == -1          # null engine
    assert lib.mmb_range_allreduce(None, None) == -1
    assert lib.mmb_gr_allreduce(None, None, None, None) == -1
    assert lib.mmb_reserve_draws(None, 8) == -1
    lib.mmb_comm_destroy(None)


def test_julia_shim_binds_declared_symbols():
    """julia/MambaHIP.jl (the ccall shim, not runnable here) binds only entry points the
    header declares and the library exports, and covers the ones a mcmc_master! branch needs."""
    src = open(os.path.join(ROOT, "julia", "MambaHIP.jl")).read()
    bound = set(re.findall(r"ccall\(\(:(mmb_\w+), libmambahip\)", src))
    declared = set(declared_symbols())
    assert bound and not (bound - declared), bound - declared
    need = {"mmb_create", "mmb_set_data", "mmb_init_chains", "mmb_run", "mmb_get_values", "mmb_get_tune",
            "mmb_set_tune", "mmb_set_iter", "mmb_comm_init", "mmb_gr_allreduce", "mmb_range_allreduce"}
    assert need <= bound, need - bound


def _julia_src():
    return open(os.path.join(ROOT, "julia", "MambaHIP.jl")).read()


def test_julia_shim_reads_sampler_args_from_the_registry():
    """`s.eval` is modelfx's eval'd wrapper (src/samplers/sampler.jl:22-24, src/utils.jl:3-12):
    it has no fields, so the shim must not try to read constructor arguments from it.  Every
    sampler constructor the engine lowers is wrapped and registers its arguments."""
    src = _julia_src()
    code = "\n".join(l.split("#")[0] for l in src.splitlines())  # comments may name s.eval
    assert not re.search(r"\b(getfield|fieldnames)\s*\(", code), "no reflection on closures"
    assert not re.search(r"captured\s*\(", code)
    uses = re.findall(r"s\.eval\b", code)
    assert uses and all(u == "s.eval" for u in uses)
    # s.eval is used only as the registry key
    for line in code.splitlines():
        if "s.eval" in line:
            assert "REGISTRY" in line, line
    for ctor in ["AMWG", "AMM", "NUTS", "Slice", "HMC", "MALA"]:
        assert re.search(rf"^{ctor}\(params.*=\s*$", code, re.M), ctor
        assert f"register(Mamba.{ctor}(params" in code, ctor
    assert "register(Sampler(params, f, GibbsTune())" in code
    # lower goes through block_spec, which returns nothing for an unregistered sampler
    blk = code[code.index("function block_spec"):code.index("function lower(")]
    assert "r === nothing && return nothing" in blk


def test_julia_shim_sizes_draws_like_mcmc_worker():
    """mcmc_worker! allocates Chains(last(window), p, start=burnin+thin, thin=thin)
    (src/model/mcmc.jl:70-71) = length(burnin+thin:thin:last(window)) rows
    (src/output/chains.jl:5-11); the shim must allocate the same and check it equals the
    engine's kept count before handing the pointer to mmb_run."""
    code = _julia_src()
    rc = code[code.index("function run_chains!"):]
    rc = rc[:rc.index("\nend\n")]
    assert re.search(r"Chains\(last\(window\), length\(pnames\), start=burnin \+ thin, thin=thin", rc)
    assert "size(sim.value, 1) == nkept" in rc
    assert "Ptr{Float64}(C_NULL)" in rc          # a window that keeps nothing: no pointer into []
    assert "first(filter" not in rc


def test_julia_chains_rows_equal_kept_count():
    """The invariant the shim's guard checks, over windows mcmc() and mcmc(mc, iters) produce:
    first run 1:iters, and a restart whose burnin is last(mc) with last(mc) the last kept
    iteration (mcmc.jl:3-16: last(mc) == div(iter, thin) * thin)."""
    cases = []
    for iters in (1, 7, 60, 1000):
        for burnin in (0, 3, 250):
            for thin in (1, 2, 3, 7):
                if iters > burnin:
                    cases.append((1, iters, burnin, thin))
    for it0 in (10, 11, 1000, 1001):
        for thin in (1, 2, 3):
            last_kept = (it0 // thin) * thin
            cases.append((it0 + 1, it0 + 37, last_kept, thin))
    for first, last, burnin, thin in cases:
        rows = len(range(burnin + thin, last + 1, thin))
        kept = sum(1 for i in range(first, last + 1) if i > burnin and (i - burnin) % thin == 0)
        assert rows == kept, (first, last, burnin, thin)


def _julia_fields(src, name):
    m = re.search(rf"^immutable {name}\b(.*?)^end", src, re.M | re.S)
    assert m, name
    body = re.sub(r"#.*", "", m.group(1))
    return re.findall(r"(\w+)::([\w{},]+)", body)


def _c_fields(name):
    txt = open(HDR).read()
    m = re.search(r"typedef struct \{([^{}]*)\}\s*" + name + ";", txt)
    assert m, name
    body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
    out = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        typ, names = re.match(r"((?:const\s+)?\w+\s*\**)\s*(.*)", decl).groups()
        for nm in names.split(","):
            nm = nm.strip()
            star = nm.count("*") + typ.count("*")
            nm = nm.strip("* ")
            arr = re.match(r"(\w+)\[(\w+)\]", nm)
            out.append((arr.group(1) if arr else nm, typ.replace("const", "").strip(" *"), star,
                        arr.group(2) if arr else None))
    return out


JL_C = {"Int32": "int32_t", "Int64": "int64_t", "Float64": "double", "IrBlock": "mmb_ir_block"}


@pytest.mark.parametrize("jl,c", [("IrNode", "mmb_ir_node"), ("IrBlock", "mmb_ir_block"),
                                  ("IrModel", "mmb_ir_model"), ("BlockSpec", "mmb_block_spec")])
def test_julia_structs_match_header(jl, c):
    """The Julia shim's immutable structs (ccall'd by reference) have the header's fields in
    the header's order with the same C types: the node-IR lowering (lower_ir ->
    mmb_create_ir) and the block specs reach the library with the right layout."""
    jf, cf = _julia_fields(_julia_src(), jl), _c_fields(c)
    arrays = {"MMB_IR_MAX_TERMS": 16, "MMB_MAX_BLOCKS": 8, "MMB_MAX_NODES_PER_BLOCK": 4}
    assert [n for n, _ in jf] == [n for n, *_ in cf], (jf, cf)
    for (jn, jt), (cn, ct, star, arr) in zip(jf, cf):
        if star:
            assert jt.startswith("Ptr{"), (jn, jt, ct)
        elif arr:
            n = arrays.get(arr, int(arr) if arr.isdigit() else None)
            inner = re.match(r"NTuple\{(\d+),(\w+)\}", jt)
            assert inner and int(inner.group(1)) == n, (jn, jt, arr)
            assert JL_C.get(inner.group(2)) == ct, (jn, jt, ct)
        else:
            assert JL_C.get(jt) == ct, (jn, jt, ct)


def test_julia_ir_lowering_present():
    """the shim lowers any other DAG to the node IR through the reference's
    own node functions (node.eval on a tracer Model) and term lists (keys(m, :target, b))."""
    code = "\n".join(l.split("#")[0] for l in _julia_src().splitlines())
    for needle in ["function lower_ir_(m::Model)", "node.eval(tm)", "m[k].eval(tm)", "keys(m, :target, b)",
                   "keys(m, :dependent)", "ccall((:mmb_create_ir, libmambahip)", "irl = lower_ir(m)"]:
        assert needle in code, needle
