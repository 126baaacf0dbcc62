"""Lowered models: the Model/Stochastic/Logical DAGs the HIP engine supports.

A Julia `Model(...)` (src/model/model.jl:5-27) is a DAG of user closures that the
GPU cannot run; the build lowers a fixed set of models to hand-written fused
log-density kernels.  Each `Model` here records what the engine
needs from the reference's DAG machinery:

  * the Stochastic nodes that can form sampling blocks, their lengths and whether
    their distribution is a PositiveDistribution (link = log,
    src/distributions/transformdistribution.jl:66-78);
  * the canonical unlisted value layout (ModelState.value, initialization.jl:25);
  * the monitored names in Chains order (names(m, true), model.jl:231-239);
  * the required inputs (setinputs!, initialization.jl:30-40).

  line      doc/tutorial/line.jl:5-25      y ~ MvNormal(xmat*beta, sqrt(s2))
  rats      doc/examples/rats.jl:48-97     hierarchical growth model, 30 rats x 5 weeks
  logistic  build-defined     y ~ Bernoulli(invlogit(X*beta)), beta ~ MvNormal(p, sd)
"""
import numpy as np

from . import abi
from .samplers import ArgumentError


class Node:
    def __init__(self, name, nid, offset, dim, positive):
        self.name, self.id, self.offset, self.dim, self.positive = name, nid, offset, dim, positive


class Model:
    def __init__(self, kind, nodes, nvalues, monitor_names, inputs, nobs=0, ncoef=0, prior_sd=0.0):
        self.kind = kind
        self.nodes = {n.name: n for n in nodes}
        self.nvalues = nvalues
        self.monitor_names = monitor_names
        self.input_names = inputs
        self.nobs, self.ncoef, self.prior_sd = nobs, ncoef, prior_sd
        self.samplers = []
        self.inputs = None
        self.iter = 0
        self.burnin = 0
        self._keep = []

    # ---- setsamplers! (initialization.jl:42-48) ----
    def setsamplers(self, samplers):
        out = []
        for s in samplers:
            if len(s.params) > abi.MMB_MAX_NODES_PER_BLOCK:
                raise ArgumentError("too many nodes in one block")
            for p in s.params:
                if p not in self.nodes:
                    raise ArgumentError(f"{p} is not a Stochastic node of this model")
            s.validate(self.block_dim(s))
            out.append(s)
        if not 1 <= len(out) <= abi.MMB_MAX_BLOCKS:
            raise ArgumentError(f"need 1..{abi.MMB_MAX_BLOCKS} sampling blocks")
        self.samplers = out
        return self

    def block_dim(self, s):
        return sum(self.nodes[p].dim for p in s.params)

    # ---- setinputs! ----
    def setinputs(self, inputs):
        data = {}
        for key in self.input_names:
            if key not in inputs:
                raise ArgumentError(f"missing inputs for node : {key}")
            data[key] = np.ascontiguousarray(np.asarray(inputs[key], dtype=np.float64).ravel())
        self.inputs = data
        return self

    # ---- inits (dict per chain) -> canonical K x P ----
    def init_matrix(self, inits, chains):
        if isinstance(inits, np.ndarray):
            a = np.ascontiguousarray(inits, dtype=np.float64)
            if a.ndim != 2 or a.shape[1] != self.nvalues or a.shape[0] < chains:
                raise ArgumentError("fewer initial values than chains")
            return np.ascontiguousarray(a[:chains])
        if len(inits) < chains:
            raise ArgumentError("fewer initial values than chains")
        out = np.empty((chains, self.nvalues))
        for k in range(chains):
            d = inits[k]
            for n in self.nodes.values():
                if n.name not in d:
                    raise ArgumentError(f"missing initial value for node : {n.name}")
                v = np.asarray(d[n.name], dtype=np.float64).ravel()
                if v.size != n.dim:
                    raise ArgumentError(f"incompatible initial value for node : {n.name}")
                out[k, n.offset:n.offset + n.dim] = v
        return out

    # ---- lowering to the C ABI ----
    def spec(self):
        if not self.samplers:
            raise ArgumentError("no samplers set (setsamplers!)")
        sp = abi.ModelSpec()
        sp.model = self.kind
        sp.nblocks = len(self.samplers)
        sp.nobs, sp.ncoef, sp.prior_sd = self.nobs, self.ncoef, self.prior_sd
        keep = []
        for b, s in enumerate(self.samplers):
            bs = sp.blocks[b]
            bs.sampler = s.kind
            bs.nnodes = len(s.params)
            for a, p in enumerate(s.params):
                bs.nodes[a] = self.nodes[p].id
            bs.adapt, bs.form, bs.transform = s.adapt, s.form, s.transform
            bs.batchsize, bs.target, bs.beta, bs.scale = s.batchsize, s.target, s.beta, s.scale
            bs.dim = self.block_dim(s)
            bs.epsilon, bs.nsteps, bs.gradient = s.epsilon, s.nsteps, s.gradient
            if s.tuning is not None:
                t = np.ascontiguousarray(s.tuning, dtype=np.float64)
                keep.append(t)
                bs.ntuning = t.size
                bs.tuning = abi.dptr(t)
            else:
                bs.ntuning = 0
        self._keep = keep
        return sp

    def data_arrays(self):
        """Inputs in the order the oracle/engine expect (tests use this for the oracle)."""
        if self.inputs is None:
            raise ArgumentError("inputs must be set before inits")
        return [self.inputs[k] for k in self.input_names]


def line():
    """doc/tutorial/line.jl:5-25"""
    nodes = [Node("beta", abi.MMB_LINE_BETA, 0, 2, False), Node("s2", abi.MMB_LINE_S2, 2, 1, True)]
    return Model(abi.MMB_MODEL_LINE, nodes, 3, ["beta[1]", "beta[2]", "s2"], ["x", "y"])


def rats():
    """doc/examples/rats.jl:48-97; monitored: s2_c, mu_beta, alpha0 (rats.rst:43-46)."""
    nodes = [Node("s2_c", abi.MMB_RATS_S2_C, 0, 1, True), Node("alpha", abi.MMB_RATS_ALPHA, 1, 30, False),
             Node("mu_alpha", abi.MMB_RATS_MU_ALPHA, 31, 1, False),
             Node("s2_alpha", abi.MMB_RATS_S2_ALPHA, 32, 1, True),
             Node("beta", abi.MMB_RATS_BETA, 33, 30, False), Node("mu_beta", abi.MMB_RATS_MU_BETA, 63, 1, False),
             Node("s2_beta", abi.MMB_RATS_S2_BETA, 64, 1, True)]
    return Model(abi.MMB_MODEL_RATS, nodes, 65, ["s2_c", "mu_beta", "alpha0"], ["y", "x"])


def logistic(nobs, ncoef, prior_sd=10.0):
    nodes = [Node("beta", abi.MMB_LOGISTIC_BETA, 0, ncoef, False)]
    return Model(abi.MMB_MODEL_LOGISTIC, nodes, ncoef, [f"beta[{i + 1}]" for i in range(ncoef)],
                 ["X", "y"], nobs=nobs, ncoef=ncoef, prior_sd=prior_sd)


# ---- reference data / inits ------------------------------------------------------
LINE_DATA = {"x": [1.0, 2, 3, 4, 5], "y": [1.0, 3, 3, 3, 5]}           # line.jl:69-73

RATS_Y = [151, 199, 246, 283, 320, 145, 199, 249, 293, 354, 147, 214, 263, 312, 328,
          155, 200, 237, 272, 297, 135, 188, 230, 280, 323, 159, 210, 252, 298, 331,
          141, 189, 231, 275, 305, 159, 201, 248, 297, 338, 177, 236, 285, 350, 376,
          134, 182, 220, 260, 296, 160, 208, 261, 313, 352, 143, 188, 220, 273, 314,
          154, 200, 244, 289, 325, 171, 221, 270, 326, 358, 163, 216, 242, 281, 312,
          160, 207, 248, 288, 324, 142, 187, 234, 280, 316, 156, 203, 243, 283, 317,
          157, 212, 259, 307, 336, 152, 203, 246, 286, 321, 154, 205, 253, 298, 334,
          139, 190, 225, 267, 302, 146, 191, 229, 272, 302, 157, 211, 250, 285, 323,
          132, 185, 237, 286, 331, 160, 207, 257, 303, 345, 169, 216, 261, 295, 333,
          157, 205, 248, 289, 316, 137, 180, 219, 258, 291, 153, 200, 244, 286, 324]
RATS_DATA = {"y": RATS_Y, "x": [8.0, 15.0, 22.0, 29.0, 36.0]}           # rats.jl:4-37

RATS_INITS = [                                                           # rats.jl:101-108
    {"alpha": [250.0] * 30, "beta": [6.0] * 30, "mu_alpha": 150.0, "mu_beta": 10.0,
     "s2_c": 1.0, "s2_alpha": 1.0, "s2_beta": 1.0},
    {"alpha": [20.0] * 30, "beta": [0.6] * 30, "mu_alpha": 15.0, "mu_beta": 1.0,
     "s2_c": 10.0, "s2_alpha": 10.0, "s2_beta": 10.0},
]


def rats_init_matrix(chains):
    """Chain k uses inits[(k-1) % 2 + 1]."""
    m = rats()
    base = m.init_matrix(RATS_INITS, 2)
    return np.ascontiguousarray(base[np.arange(chains) % 2])


def rats_init_ls(chains, seed=1):
    """Config-3 inits (build-defined scheme): per-rat least-squares intercepts/slopes plus
    per-chain N(0, 3^2) / N(0, 0.3^2) jitter; hyper-parameters alternate rats.jl:101-108.
    The rats.jl constant inits (all 30 alphas equal) freeze a joint AMM + conjugate
    s2_alpha scheme: one rejected joint proposal leaves the alphas identical, the Gibbs
    draw of s2_alpha collapses to ~1e-4 and pins them."""
    y = np.asarray(RATS_Y, dtype=np.float64).reshape(30, 5)
    x = np.asarray(RATS_DATA["x"])
    xm = x - x.mean()
    a_ls = y.mean(1)
    b_ls = (y * xm).sum(1) / (xm @ xm)
    rng = np.random.default_rng(seed)
    init = rats_init_matrix(chains)
    init[:, 1:31] = a_ls + rng.normal(0.0, 3.0, (chains, 30))
    init[:, 33:63] = b_ls + rng.normal(0.0, 0.3, (chains, 30))
    return init


def line_init_matrix(chains, seed=123):
    """line.jl:81-88: beta ~ Normal(0,1) x2, s2 ~ Gamma(1,1) (numpy stream, not MT)."""
    rng = np.random.default_rng(seed)
    out = np.empty((chains, 3))
    out[:, :2] = rng.normal(0.0, 1.0, (chains, 2))
    out[:, 2] = rng.gamma(1.0, 1.0, chains)
    return out


def rats_scheme_reference():
    """rats.jl:112-116 (the published rats.rst run)."""
    from .samplers import AMWG, Slice, Univariate
    return [Slice("s2_c", 10.0), AMWG("alpha", 100.0),
            Slice(["mu_alpha", "s2_alpha"], [100.0, 10.0], Univariate),
            AMWG("beta", 1.0), Slice(["mu_beta", "s2_beta"], 1.0, Univariate)]


def rats_scheme_gibbs_amm():
    """BASELINE config 3 'mixed Gibbs+AMM' (SURVEY §8a): conjugate Gibbs on the variance /
    hyper-mean nodes, AMM on the 30-dim alpha and beta blocks with diagonal proposal
    covariances Sigma_alpha = I, Sigma_beta = 0.01 I (posterior sd ~2.7 and ~0.27)."""
    from .samplers import AMM, Gibbs
    return [Gibbs("s2_c"), AMM("alpha", np.eye(30)), Gibbs("mu_alpha"), Gibbs("s2_alpha"),
            AMM("beta", 0.01 * np.eye(30)), Gibbs("mu_beta"), Gibbs("s2_beta")]


def logistic_data(nobs=10000, ncoef=50):
    """Synthetic config 4: X ~ N(0,1) (seed 2), beta_true ~ N(0, 0.5^2) (seed 3),
    y ~ Bernoulli(invlogit(X beta_true)) (seed 4)."""
    X = np.random.default_rng(2).normal(0.0, 1.0, (nobs, ncoef))
    bt = np.random.default_rng(3).normal(0.0, 0.5, ncoef)
    p = 1.0 / (1.0 + np.exp(-(X @ bt)))
    y = (np.random.default_rng(4).random(nobs) < p).astype(np.float64)
    return {"X": X, "y": y}, bt
