"""Sampler constructors mirroring Mamba.jl's model-based sampler API.

Each constructor returns a `Sampler` (src/Mamba.jl:119-124: params, eval, tune,
targets) whose `eval` is a lowered HIP block update instead of a Julia closure.
Argument meaning, defaults and validation errors follow the reference:

  AMWG(params, sigma; adapt=:all, batchsize=50, target=0.44)   src/samplers/amwg.jl:47-61
  AMM(params, Sigma; adapt=:all, beta=0.05, scale=2.38)        src/samplers/amm.jl:45-59
  NUTS(params; dtype=:forward, target=0.6)                     src/samplers/nuts.jl:47-56
  Slice(params, width, Univariate|Multivariate; transform=false) src/samplers/slice.jl:47-58
  HMC(params, epsilon, L[, Sigma]; dtype=:forward)            src/samplers/hmc.jl:47-65
  MALA(params, epsilon[, Sigma]; dtype=:forward)              src/samplers/mala.jl:43-58
  Gibbs(params)  -- a user `Sampler(params, f)` whose f is the node's conjugate full
                    conditional (doc/tutorial/line.jl:27-45); lowered per model.
"""
import numpy as np

from . import abi

Univariate = "Univariate"
Multivariate = "Multivariate"


class ArgumentError(ValueError):
    """Julia ArgumentError raised by the reference's validators."""


def _params(params):
    if isinstance(params, str):
        return [params]
    return list(params)


def _adapt(adapt):
    adapt = str(adapt).lstrip(":")
    if adapt not in ("all", "burnin", "none"):
        raise ArgumentError("adapt must be one of :all, :burnin, or :none")
    return {"all": abi.MMB_ADAPT_ALL, "burnin": abi.MMB_ADAPT_BURNIN, "none": abi.MMB_ADAPT_NONE}[adapt]


class Sampler:
    def __init__(self, params, kind, adapt=abi.MMB_ADAPT_ALL, tuning=None, **kw):
        self.params = _params(params)
        self.kind = kind
        self.adapt = adapt
        self.tuning = None if tuning is None else np.atleast_1d(np.asarray(tuning, dtype=np.float64))
        self.form = kw.pop("form", abi.MMB_SLICE_MULTIVARIATE)
        self.transform = int(kw.pop("transform", False))
        self.batchsize = int(kw.pop("batchsize", 50))
        self.target = float(kw.pop("target", 0.44))
        self.beta = float(kw.pop("beta", 0.05))
        self.scale = float(kw.pop("scale", 2.38))
        self.epsilon = float(kw.pop("epsilon", 0.0))
        self.nsteps = int(kw.pop("nsteps", 0))
        self.gradient = int(kw.pop("gradient", abi.MMB_GRAD_DEFAULT))
        if kw:
            raise ArgumentError(f"unsupported sampler arguments {sorted(kw)}")
        self.targets = []

    def validate(self, dim):
        """validate(v) (amwg.jl:37-42, amm.jl:35-40, slice.jl:37-42)"""
        t = self.tuning
        if self.kind == abi.MMB_SAMPLER_AMWG and not (t.size == 1 or t.size == dim):
            raise ArgumentError(f"length(sigma) differs from variate length {dim}")
        if self.kind == abi.MMB_SAMPLER_AMM and t.size != dim * dim:
            raise ArgumentError(f"Sigma dimension differs from variate length {dim}")
        if self.kind == abi.MMB_SAMPLER_SLICE and not (t.size == 1 or t.size == dim):
            raise ArgumentError(f"length(width) differs from variate length {dim}")
        if self.kind in (abi.MMB_SAMPLER_HMC, abi.MMB_SAMPLER_MALA) and t is not None and t.size != dim * dim:
            raise ArgumentError(f"Sigma dimension differs from variate length {dim}")

    def __repr__(self):
        names = {1: "AMWG", 2: "AMM", 3: "NUTS", 4: "Slice", 5: "Gibbs", 6: "HMC", 7: "MALA"}
        return f"{names[self.kind]}({self.params})"


def AMWG(params, sigma, adapt="all", batchsize=50, target=0.44):
    return Sampler(params, abi.MMB_SAMPLER_AMWG, _adapt(adapt), sigma, batchsize=batchsize,
                   target=target)


def AMM(params, Sigma, adapt="all", beta=0.05, scale=2.38):
    S = np.asarray(Sigma, dtype=np.float64)
    if S.ndim != 2 or S.shape[0] != S.shape[1]:
        raise ArgumentError("Sigma must be a square matrix")
    # column-major, as Julia stores it
    return Sampler(params, abi.MMB_SAMPLER_AMM, _adapt(adapt), S.ravel(order="F"), beta=beta,
                   scale=scale)


def NUTS(params, dtype="forward", target=0.6):
    return Sampler(params, abi.MMB_SAMPLER_NUTS, abi.MMB_ADAPT_BURNIN, None, target=target,
                   gradient=_dtype(dtype))


def _dtype(dtype):
    """logpdfgrad! scheme (sampler.jl:97-111 -> simulation.jl:47-51, Calculus): "forward" (the
    reference's default) -> MMB_GRAD_FORWARD: Calculus forward differences (line, node IR; the
    logistic kernel has none: mmb_create refuses it with MMB_E_UNSUPPORTED, so a reference-default
    NUTS(:beta) on logistic is never silently given another gradient); "analytic" -> the
    hand-derived gradient (line, logistic: the config-4 kernel's batched MFMA gradient).
    Calculus' :central / :complex are not on the device."""
    d = str(dtype).lstrip(":")
    if d == "forward":
        return abi.MMB_GRAD_FORWARD
    if d == "analytic":
        return abi.MMB_GRAD_ANALYTIC
    if d in ("central", "complex"):
        raise ArgumentError(f"dtype :{d} is not supported on the device (forward or analytic)")
    raise ArgumentError(f"unsupported dtype {dtype}")


def _sigma(Sigma):
    if Sigma is None:
        return None  # SigmaL = I (UniformScaling)
    S = np.asarray(Sigma, dtype=np.float64)
    if S.ndim != 2 or S.shape[0] != S.shape[1]:
        raise ArgumentError("Sigma must be a square matrix")
    return S.ravel(order="F")


def HMC(params, epsilon, L, Sigma=None, dtype="forward"):
    """HMC(params, epsilon, L[, Sigma]; dtype) -- hmc.jl:47-55; tune [epsilon, L] (HMCTune)."""
    g = _dtype(dtype)
    if int(L) != L:
        raise ArgumentError("L must be an integer")
    return Sampler(params, abi.MMB_SAMPLER_HMC, abi.MMB_ADAPT_NONE, _sigma(Sigma), epsilon=epsilon,
                   nsteps=int(L), gradient=g)


def MALA(params, epsilon, Sigma=None, dtype="forward"):
    """MALA(params, epsilon[, Sigma]; dtype) -- mala.jl:43-51; tune [epsilon] (MALATune)."""
    g = _dtype(dtype)
    return Sampler(params, abi.MMB_SAMPLER_MALA, abi.MMB_ADAPT_NONE, _sigma(Sigma), epsilon=epsilon, gradient=g)


def Slice(params, width, form=Multivariate, transform=False):
    f = {Univariate: abi.MMB_SLICE_UNIVARIATE, Multivariate: abi.MMB_SLICE_MULTIVARIATE}.get(form)
    if f is None:
        raise ArgumentError("form must be Univariate or Multivariate")
    return Sampler(params, abi.MMB_SAMPLER_SLICE, abi.MMB_ADAPT_NONE, width, form=f,
                   transform=transform)


def Gibbs(params):
    return Sampler(params, abi.MMB_SAMPLER_GIBBS, abi.MMB_ADAPT_NONE, None)
