"""Build libmambahip.so (hipcc, gfx950) in-tree: mamba.jl_amd/lib/libmambahip.so.

Device code is compiled with -ffp-contract=off: together with mmb_math.h this makes
every per-lane arithmetic path bit-identical to the CPU oracle.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "lib", "libmambahip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
SOURCES = ["sweep.hip", "gr.hip", "nuts.hip", "engine.cpp"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-I", os.path.join(ROOT, "include")]


def _compile(src, objdir):
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    cmd = [HIPCC, *FLAGS, "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose=False):
    objdir = os.path.join(PKG, "lib", "obj")
    os.makedirs(objdir, exist_ok=True)
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    with ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir), srcs))
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
