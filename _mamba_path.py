"""Register the package directory `mamba.jl_amd/` as the importable module `mamba_amd`."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "mamba.jl_amd")


def load():
    if "mamba_amd" in sys.modules:
        return sys.modules["mamba_amd"]
    spec = importlib.util.spec_from_file_location(
        "mamba_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mamba_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
