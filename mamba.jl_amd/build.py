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
SOURCES = ["sweep.hip", "line_amm.hip", "gr.hip", "logistic.hip", "summary.hip", "engine.cpp"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-mllvm", "-pragma-unroll-threshold=100000",  # pchol32's 30 steps stay fully unrolled
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-I", os.path.join(ROOT, "include")]


def _deps_mtime(src):
    """Newest of the source and every header it may include (csrc/*.h, include/*.h)."""
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    inc = os.path.join(ROOT, "include")
    hdrs += [os.path.join(inc, f) for f in os.listdir(inc) if f.endswith(".h")]
    return max(os.path.getmtime(x) for x in [os.path.join(CSRC, src), *hdrs, __file__])


def _compile(src, objdir, defines=()):
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) > _deps_mtime(src) and not os.environ.get("MMB_REBUILD"):
        return obj  # up to date (same flags: the object directory is per define set)
    cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines], "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose=False, out=OUT, defines=()):
    """defines: extra -D flags (experiments, e.g. MMB_SWEEP_WAVES=3) -> separate obj dir."""
    tag = "_".join(d.replace("=", "") for d in defines)
    objdir = os.path.join(PKG, "lib", "obj" + ("_" + tag if tag else ""))
    os.makedirs(objdir, exist_ok=True)
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    with ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir, defines), srcs))
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out, "-L/opt/rocm/lib", "-lrccl",
           "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print("built", out)
    return out


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
