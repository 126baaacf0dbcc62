"""mamba_amd — MI355X-native many-chain MCMC engine for Mamba.jl's sampler hot path.

Python host mirror of the reference's model-based sampler API (src/samplers/*.jl,
src/model/mcmc.jl) over the C ABI of include/mamba_hip.h (libmambahip.so).  Every
sampling call runs the hand-written HIP kernels; there is no CPU fallback.

The package directory is `mamba.jl_amd/`; import it as `mamba_amd` via
`_mamba_path.load()` (the dot in the directory name is not importable directly).
"""
from . import abi, gelman, ir, model, samplers, summary  # noqa: F401
from .gelman import Comm, gelmandiag, gelmandiag_rccl, gelmandiag_sharded, psrf_from_sums  # noqa: F401
from .summary import pool_summary, quantile_sharded, summarystats_sharded  # noqa: F401
from .mcmc import Chains, Engine, mcmc, mcmc_restart, read, write  # noqa: F401
from .model import line, logistic, rats  # noqa: F401
from .samplers import (AMM, AMWG, HMC, MALA, NUTS, ArgumentError, Gibbs, Multivariate, Sampler,  # noqa: F401
                       Slice, Univariate)

__version__ = "0.1.0"
