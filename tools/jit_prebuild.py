"""Compile the node-IR specialised kernels (csrc/ir_jit.cpp, hipRTC) of every IR model the GPU
tests and bench.py create, into the in-tree cache (mamba.jl_amd/lib/jit, next to the library),
on the CPU -- a build step like the library itself, so no GPU run pays a compile.

  python tools/jit_prebuild.py [-j 3]

The cache key is a hash of the generated source (the model's structure, not its data), the
embedded headers, the options and the hipRTC version.
"""
import argparse
import ctypes as C
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def models():
    """(label, model) of every IR model the GPU tests and the bench create."""
    import _mamba_path
    mb = _mamba_path.load()
    import test_gpu_ir as T
    out = []
    for case, (name, sch) in sorted(T.CASES.items()):
        m, _ = T.example(mb, name, 2, scheme=sch(mb) if sch else None)
        out.append((case, m))
    for name in ["seeds", "pumps", "surgical", "dyes", "salm", "blocker"]:
        m, _ = T.example(mb, name, 2)
        out.append((name, m))
    ir = mb.ir
    m = ir.rats_model().setinputs(ir.rats_inputs()).setsamplers(mb.model.rats_scheme_reference())
    m.init_matrix([{**mb.model.RATS_INITS[k % 2], "y": mb.model.RATS_Y} for k in range(2)], 2)
    out.append(("rats_ir_reference", m))
    m = ir.seeds_model().setinputs(ir.SEEDS)
    m.setsamplers([mb.AMM(["alpha0", "alpha1", "alpha2", "alpha12"], 0.01 * np.eye(4)), mb.AMWG("b", 0.01),
                   mb.AMWG("s2", 0.1)])
    m.init_matrix([ir.seeds_inits()[k % 2] for k in range(2)], 2)
    out.append(("seeds_ir_bench", m))
    return out


def build_one(i):
    import _mamba_path
    mb = _mamba_path.load()
    label, m = models()[i]
    lib = mb.abi.lib()
    spec, irm = m.spec(), m.ir()
    buf = C.create_string_buffer(8192)
    t0 = time.time()
    rc = lib.mmb_ir_jit_prebuild(C.byref(spec), C.byref(irm), buf, len(buf))
    return label, rc, time.time() - t0, buf.value.decode()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=3)  # hipRTC compiles take several GB each
    a = ap.parse_args()
    n = len(models())
    import multiprocessing as mp
    with ProcessPoolExecutor(a.j, mp_context=mp.get_context("spawn")) as ex:  # no fork of a HIP process
        res = list(ex.map(build_one, range(n)))
    bad = 0
    for label, rc, dt, info in res:
        print(f"{label:24s} rc={rc} {dt:6.1f}s {info.splitlines()[0] if info else ''}")
        if rc != 0:
            bad += 1
            print(info)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
