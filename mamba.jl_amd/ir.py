"""Generic node IR: Mamba Model DAGs lowered for the HIP engine.

Mirrors the reference's model specification API (src/model/dependent.jl:75-152,
src/model/model.jl:5-27):

    model = ir.Model(
        r=ir.Stochastic(1, lambda alpha0, alpha1, x1, b, n:
                        ir.Binomial(n, ir.invlogit(alpha0 + alpha1 * x1 + b)), False),
        b=ir.Stochastic(1, lambda s2: ir.Normal(0, ir.sqrt(s2)), False),
        alpha0=ir.Stochastic(lambda: ir.Normal(0, 1000)), ...)

Each node function names its parents by argument name, like a Julia closure
(src/utils.jl:3-43).  It is traced once with symbolic arguments, so it is written
vectorised: arithmetic broadcasts elementwise over the node's elements (a Stochastic(1, ...)
node with a univariate distribution is elementwise, distributionstruct.jl:142-158),
`mu[batch]` gathers with a 1-based data index vector, `beta[2]` is element 2 (1-based).
Logical nodes are inlined into their Stochastic children; Stochastic nodes that no sampling
block updates are fixed (observed) and their values (from the inits, as in the reference)
go to the data pool.  The lowering produces the mmb_ir_model of include/mamba_hip.h:
per-node stack code, the block term lists of logpdf! (simulation.jl:77-90: params \\ targets
in block order, then targets in topological order) and the monitored nodes.

Supported: Normal, MvNormal(mu, sigma) (isotropic), InverseGamma, Gamma, Exponential,
Uniform (constant bounds), Beta for sampled nodes; Binomial, Poisson, Bernoulli for fixed
nodes; + - * / neg abs exp log sqrt invlogit logit, x**2; blocks of <= 32 elements.
The topological order of targets is deterministic (declaration order breaks ties); the
reference's depends on Dict hashing (model.jl:112-120), which only changes summation order.
"""
import ctypes as C
import inspect
import math

import numpy as np

from . import abi
from .model import Model as _BaseModel, Node
from .samplers import ArgumentError

# ------------------------------------------------------------------ expressions


def _e(x):
    if isinstance(x, Expr):
        return x
    if isinstance(x, (int, float, np.integer, np.floating)):
        return Const(float(x))
    raise ArgumentError(f"unsupported value in a node expression: {x!r}")


class Expr:
    def __add__(s, o): return Bin("+", s, _e(o))
    def __radd__(s, o): return Bin("+", _e(o), s)
    def __sub__(s, o): return Bin("-", s, _e(o))
    def __rsub__(s, o): return Bin("-", _e(o), s)
    def __mul__(s, o): return Bin("*", s, _e(o))
    def __rmul__(s, o): return Bin("*", _e(o), s)
    def __truediv__(s, o): return Bin("/", s, _e(o))
    def __rtruediv__(s, o): return Bin("/", _e(o), s)
    def __neg__(s): return Un("neg", s)
    def __abs__(s): return Un("abs", s)

    def __pow__(s, k):
        if k == 2:
            return Bin("*", s, s)
        raise ArgumentError("only x**2 is supported in node expressions")


class Const(Expr):
    def __init__(s, v):
        s.v = v


class Ref(Expr):
    """A closure argument: a node or an input, elementwise."""

    def __init__(s, name):
        s.name = name

    def __getitem__(s, idx):
        if isinstance(idx, Ref):
            return Gather(s.name, idx.name)
        if isinstance(idx, (int, np.integer)) and idx >= 1:
            return Elem(s.name, int(idx))
        raise ArgumentError("index a node with a 1-based integer or a data index vector")


class Elem(Expr):
    def __init__(s, name, k):
        s.name, s.k = name, k


class Gather(Expr):
    def __init__(s, name, idx):
        s.name, s.idx = name, idx


class Bin(Expr):
    def __init__(s, op, a, b):
        s.op, s.a, s.b = op, a, b


class Un(Expr):
    def __init__(s, op, a):
        s.op, s.a = op, a


def exp(x): return Un("exp", _e(x))
def log(x): return Un("log", _e(x))
def sqrt(x): return Un("sqrt", _e(x))
def invlogit(x): return Un("invlogit", _e(x))   # src/utils.jl:64
def logit(x): return Un("logit", _e(x))         # src/utils.jl:67


# ------------------------------------------------------------------ distributions

class Dist:
    def __init__(s, fam, *params):
        s.fam = fam
        s.params = [_e(p) for p in params]


def Normal(mu=0.0, sigma=1.0): return Dist(abi.MMB_IR_NORMAL, mu, sigma)
def InverseGamma(shape=1.0, scale=1.0): return Dist(abi.MMB_IR_INVGAMMA, shape, scale)
def Gamma(shape=1.0, scale=1.0): return Dist(abi.MMB_IR_GAMMA, shape, scale)
def Exponential(scale=1.0): return Dist(abi.MMB_IR_EXPONENTIAL, scale)
def Uniform(a=0.0, b=1.0): return Dist(abi.MMB_IR_UNIFORM, a, b)
def Beta(a=1.0, b=1.0): return Dist(abi.MMB_IR_BETA, a, b)
def Binomial(n, p): return Dist(abi.MMB_IR_BINOMIAL, n, p)
def Poisson(lam): return Dist(abi.MMB_IR_POISSON, lam)
def Bernoulli(p): return Dist(abi.MMB_IR_BERNOULLI, p)


def MvNormal(mu, sigma):
    """MvNormal(mu, sigma) / MvNormal(k, sigma) (zero mean): isotropic ScalMat covariance."""
    if isinstance(mu, (int, np.integer)) and not isinstance(mu, bool):
        mu = 0.0
    return Dist(abi.MMB_IR_ISONORMAL, mu, sigma)


_SAMPLEABLE = {abi.MMB_IR_NORMAL, abi.MMB_IR_ISONORMAL, abi.MMB_IR_INVGAMMA, abi.MMB_IR_GAMMA,
               abi.MMB_IR_EXPONENTIAL, abi.MMB_IR_UNIFORM, abi.MMB_IR_BETA}
_DISCRETE = {abi.MMB_IR_BINOMIAL, abi.MMB_IR_POISSON, abi.MMB_IR_BERNOULLI}
_POSITIVE = {abi.MMB_IR_INVGAMMA, abi.MMB_IR_GAMMA, abi.MMB_IR_EXPONENTIAL}


# ------------------------------------------------------------------ nodes

class _NodeDef:
    def __init__(self, kind, args, monitor):
        if args and callable(args[0]):
            dim, f, rest = 0, args[0], args[1:]
        elif len(args) >= 2 and callable(args[1]):
            dim, f, rest = int(args[0]), args[1], args[2:]
        else:
            raise ArgumentError(f"{kind}([dim,] f[, monitor])")
        if rest:
            monitor = rest[0]
        self.kind, self.dim, self.f = kind, dim, f
        self.monitor = bool(monitor)
        self.argnames = list(inspect.signature(f).parameters)


def Stochastic(*args, monitor=True):
    """Stochastic(f[, monitor]) / Stochastic(d, f[, monitor]) (dependent.jl:137-152)."""
    return _NodeDef("stochastic", args, monitor)


def Logical(*args, monitor=True):
    """Logical(f[, monitor]) / Logical(d, f[, monitor]) (dependent.jl:75-88)."""
    return _NodeDef("logical", args, monitor)


# ------------------------------------------------------------------ model

class Model(_BaseModel):
    """Model(; nodes...) (model.jl:5-27) lowered to the node IR at setinits (init_matrix)."""

    def __init__(self, **nodes):
        super().__init__(abi.MMB_MODEL_IR, [], 0, [], [])
        self.defs = dict(nodes)
        self.order = list(nodes)
        self.traced = {}
        for name, d in self.defs.items():
            if not isinstance(d, _NodeDef):
                raise ArgumentError(f"node {name} must be a Stochastic or Logical")
            out = d.f(*[Ref(a) for a in d.argnames])
            if d.kind == "stochastic":
                if not isinstance(out, Dist):
                    raise ArgumentError(f"Stochastic node {name} must return a distribution")
            else:
                out = _e(out)
            self.traced[name] = out
        self.stoch = [n for n in self.order if self.defs[n].kind == "stochastic"]
        # Stochastic nodes are the candidate block parameters (dims known at setinits)
        self.nodes = {n: Node(n, i, 0, 0, self.traced[n].fam in _POSITIVE) for i, n in enumerate(self.order)
                      if self.defs[n].kind == "stochastic"}
        self.compiled = False
        self.inputs = {}

    # setsamplers! is checked once the node lengths are known (init_matrix)
    def setsamplers(self, samplers):
        for s in samplers:
            if s.kind == abi.MMB_SAMPLER_GIBBS:
                raise ArgumentError("Gibbs (a user Sampler closure) cannot be lowered to the node IR")
            for p in s.params:
                if p not in self.nodes:
                    raise ArgumentError(f"{p} is not a Stochastic node of this model")
        if not 1 <= len(samplers) <= abi.MMB_MAX_BLOCKS:
            raise ArgumentError(f"need 1..{abi.MMB_MAX_BLOCKS} sampling blocks")
        self.samplers = list(samplers)
        self.compiled = False
        return self

    def setinputs(self, inputs):
        self.inputs = {k: np.atleast_1d(np.asarray(v, dtype=np.float64)).ravel(order="F") for k, v in inputs.items()}
        self.compiled = False
        return self

    def data_arrays(self):
        return []

    def block_dim(self, s):
        return sum(self.lens[p] for p in s.params)

    # ---- setinits!: node lengths, layout, lowering ----
    def init_matrix(self, inits, chains):
        if isinstance(inits, np.ndarray):
            if not self.compiled:
                raise ArgumentError("a node-IR model needs dict inits (node lengths) before a value matrix")
            return super().init_matrix(inits, chains)
        if len(inits) < chains:
            raise ArgumentError("fewer initial values than chains")
        self._compile(inits[0])
        for k in range(1, chains):  # fixed (observed) nodes are data: equal in every chain
            for n in self.fixed:
                if not np.array_equal(self._initval(inits[k], n), self.fixed_vals[n]):
                    raise ArgumentError(f"fixed node {n} differs between chains' inits")
        return super().init_matrix([{p: inits[k][p] for p in self.params} for k in range(chains)], chains)

    def _initval(self, d, n):
        if n not in d:
            raise ArgumentError(f"missing initial value for node : {n}")
        return np.atleast_1d(np.asarray(d[n], dtype=np.float64)).ravel(order="F")

    def _compile(self, init0):
        if not self.samplers:
            raise ArgumentError("no samplers set (setsamplers!)")
        inblock = {p for s in self.samplers for p in s.params}
        self.params = [n for n in self.stoch if n in inblock]
        self.fixed = [n for n in self.stoch if n not in inblock]
        self.lens = {}
        for n in self.stoch:
            v = self._initval(init0, n)
            if self.defs[n].dim == 0 and v.size != 1:
                raise ArgumentError(f"incompatible initial value for node : {n}")
            self.lens[n] = v.size
        self.fixed_vals = {n: self._initval(init0, n) for n in self.fixed}
        for n in self.params:
            if self.traced[n].fam not in _SAMPLEABLE:
                raise ArgumentError(f"node {n}: its distribution family cannot be sampled by these samplers")
        # state layout: sampled nodes in declaration order
        off = 0
        self.nodes = {}
        for i, n in enumerate(self.order):
            if n in self.params:
                self.nodes[n] = Node(n, i, off, self.lens[n], self.traced[n].fam in _POSITIVE)
                off += self.lens[n]
        self.nvalues = off
        if not 1 <= off <= abi.MMB_IR_MAX_VALUES:
            raise ArgumentError(f"node IR: 1..{abi.MMB_IR_MAX_VALUES} sampled values")
        for s in self.samplers:
            d = self.block_dim(s)
            if d > 32:
                raise ArgumentError(f"node IR: blocks of at most 32 elements (block {s.params} has {d})")
            s.validate(d)
        _Lowering(self).run()
        self.compiled = True

    def spec(self):
        if not self.compiled:
            raise ArgumentError("node-IR model: call init_matrix (setinits!) first")
        return super().spec()

    def ir(self):
        if not self.compiled:
            raise ArgumentError("node-IR model: call init_matrix (setinits!) first")
        return self._ir


class _Lowering:
    """Model -> mmb_ir_model (include/mamba_hip.h)."""

    def __init__(self, m):
        self.m = m
        self.code, self.consts, self.pool = [], [], []
        self.pool_of = {}
        self.depth = 1

    # -- pool / const helpers
    def const(self, v):
        self.consts.append(float(v))
        return len(self.consts) - 1

    @staticmethod
    def word(opc, arg):
        """One code word: opcode in the top byte, operand (pool / value / constant offset) in
        the low 24 bits; a larger operand would carry into the opcode, so it is refused."""
        if not 0 <= arg < 1 << 24:
            raise ArgumentError(f"node IR operand {arg} does not fit in 24 bits (pool or model too large)")
        return opc << 24 | arg

    def put(self, key, arr):
        if key in self.pool_of:
            return self.pool_of[key]
        off = len(self.pool)
        self.pool.extend(float(a) for a in np.asarray(arr, dtype=np.float64).ravel())
        self.pool_of[key] = off
        return off

    def kind(self, name):
        m = self.m
        if name in m.defs:
            if m.defs[name].kind == "logical":
                return "logical"
            return "param" if name in m.params else "fixed"
        if name in m.inputs:
            return "data"
        raise ArgumentError(f"{name} is neither a node nor an input")

    def length(self, e, seen=()):
        """Broadcast length of an expression (1 = scalar)."""
        if isinstance(e, Const) or isinstance(e, Elem):
            return 1
        if isinstance(e, Ref):
            k = self.kind(e.name)
            if k == "logical":
                if e.name in seen:
                    raise ArgumentError(f"cycle through logical {e.name}")
                return self.length(self.m.traced[e.name], seen + (e.name,))
            if k == "data":
                return self.m.inputs[e.name].size
            return self.m.lens[e.name]
        if isinstance(e, Gather):
            return self.m.inputs[e.idx].size if e.idx in self.m.inputs else self.length(Ref(e.idx))
        if isinstance(e, Bin):
            a, b = self.length(e.a, seen), self.length(e.b, seen)
            if a != 1 and b != 1 and a != b:
                raise ArgumentError("length mismatch in a node expression")
            return max(a, b)
        return self.length(e.a, seen)

    def host_value(self, e, n):
        """Numeric value of a data/constant-only expression (length n), else None."""
        if isinstance(e, Const):
            return np.full(n, e.v)
        if isinstance(e, Ref):
            k = self.kind(e.name)
            if k == "data":
                v = self.m.inputs[e.name]
                return np.full(n, v[0]) if v.size == 1 else v.copy()
            if k == "fixed":
                v = self.m.fixed_vals[e.name]
                return np.full(n, v[0]) if v.size == 1 else v.copy()
            if k == "logical":
                return self.host_value(self.m.traced[e.name], n)
            return None
        if isinstance(e, Bin):
            a, b = self.host_value(e.a, n), self.host_value(e.b, n)
            if a is None or b is None:
                return None
            return {"+": a + b, "-": a - b, "*": a * b, "/": a / b}[e.op]
        if isinstance(e, Un):
            a = self.host_value(e.a, n)
            if a is None:
                return None
            return {"neg": -a, "abs": np.abs(a), "exp": np.exp(a), "log": np.log(a), "sqrt": np.sqrt(a),
                    "invlogit": 1.0 / (np.exp(-a) + 1.0), "logit": np.log(a / (1.0 - a))}[e.op]
        return None

    # -- code emission for an expression evaluated at elements 0..n-1
    def emit(self, e, n, sp, refs):
        op = abi.IR_OP
        m = self.m

        def push(word):
            self.code.append(word)
            self.depth = max(self.depth, sp + 1)
            return sp + 1

        if isinstance(e, Const):
            return push(self.word(op["const"], self.const(e.v)))
        if isinstance(e, Elem):
            k = self.kind(e.name)
            ln = self.length(Ref(e.name))
            if not 1 <= e.k <= ln:
                raise ArgumentError(f"{e.name}[{e.k}] out of range")
            if k == "param":
                refs.add(e.name)
                return push(self.word(op["val"], (m.nodes[e.name].offset + e.k - 1)))
            if k in ("fixed", "data"):
                v = m.fixed_vals[e.name] if k == "fixed" else m.inputs[e.name]
                return push(self.word(op["datas"], self.put(("elem", e.name, e.k), v[e.k - 1:e.k])))
            raise ArgumentError("element of a logical: index its parents instead")
        if isinstance(e, Ref):
            k = self.kind(e.name)
            if k == "logical":
                ln = self.length(e)
                if ln not in (1, n):
                    raise ArgumentError(f"logical {e.name} has length {ln}, expected 1 or {n}")
                return self.emit(m.traced[e.name], n, sp, refs)
            ln = self.length(e)
            if ln not in (1, n):
                raise ArgumentError(f"{e.name} has length {ln}, expected 1 or {n}")
            if k == "param":
                refs.add(e.name)
                o = m.nodes[e.name].offset
                return push(self.word(op["val"] if ln == 1 else op["vali"], o))
            v = m.fixed_vals[e.name] if k == "fixed" else m.inputs[e.name]
            o = self.put(("v", e.name), v)
            return push(self.word(op["datas"] if ln == 1 else op["data"], o))
        if isinstance(e, Gather):
            if e.idx not in m.inputs:
                raise ArgumentError(f"gather index {e.idx} must be an input (data) vector")
            idx = m.inputs[e.idx]
            if idx.size != n:
                raise ArgumentError(f"gather index {e.idx} has length {idx.size}, expected {n}")
            k = self.kind(e.name)
            ln = self.length(Ref(e.name))
            if np.any(idx != np.round(idx)) or idx.min() < 1 or idx.max() > ln:
                raise ArgumentError(f"{e.name}[{e.idx}]: indices must be integers in 1..{ln}")
            if k == "param":
                refs.add(e.name)
                w = self.put(("idx", e.idx), idx - 1.0)
                sp2 = push(self.word(op["valg"], m.nodes[e.name].offset))
                self.code.append(w)
                return sp2
            if k in ("fixed", "data"):
                v = m.fixed_vals[e.name] if k == "fixed" else m.inputs[e.name]
                return push(self.word(op["data"], self.put(("g", e.name, e.idx), v[(idx - 1).astype(int)])))
            raise ArgumentError("gather from a logical: gather its parents instead")
        if isinstance(e, Bin):
            sp = self.emit(e.a, n, sp, refs)
            sp = self.emit(e.b, n, sp, refs)
            self.code.append(op[e.op] << 24)
            return sp - 1
        sp = self.emit(e.a, n, sp, refs)
        self.code.append(op[e.op] << 24)
        return sp

    def expr(self, e, n, refs):
        start = len(self.code)
        self.emit(e, n, 0, refs)
        self.code.append(0)  # END
        return start

    def run(self):
        m = self.m
        ids = {n: i for i, n in enumerate(m.order)}
        nodes = (abi.IrNode * len(m.order))()
        parents = {}
        for n in m.order:
            N = nodes[ids[n]]
            N.expr[0] = N.expr[1] = N.expr[2] = -1
            N.cterm = -1
            N.lo = N.hi = 0.0
            d = m.defs[n]
            refs = set()
            if d.kind == "logical":
                e = m.traced[n]
                N.family, N.fixed, N.off = abi.MMB_IR_LOGICAL, 0, 0
                N.len = self.length(e)
                N.expr[0] = self.expr(e, N.len, refs)
                continue
            dist = m.traced[n]
            ln = m.lens[n]
            N.family, N.len = dist.fam, ln
            if n in m.params:
                N.fixed, N.off = 0, m.nodes[n].offset
            else:
                N.fixed, N.off = 1, self.put(("v", n), m.fixed_vals[n])
            ps = dist.params
            if dist.fam == abi.MMB_IR_ISONORMAL:
                N.expr[0] = self.expr(ps[0], ln, refs)
                if self.length(ps[1]) != 1:
                    raise ArgumentError(f"MvNormal sigma of {n} must be a scalar")
                N.expr[1] = self.expr(ps[1], 1, refs)
            else:
                for k, p in enumerate(ps):
                    N.expr[k] = self.expr(p, ln, refs)
            if dist.fam == abi.MMB_IR_UNIFORM:
                lo, hi = self.host_value(ps[0], 1), self.host_value(ps[1], 1)
                if lo is None or hi is None:
                    raise ArgumentError(f"Uniform bounds of {n} must be constants or data")
                N.lo, N.hi = float(lo[0]), float(hi[0])
            if dist.fam in _DISCRETE:
                if n in m.params:
                    raise ArgumentError(f"discrete node {n} cannot be sampled")
                x = m.fixed_vals[n]
                if np.any(x != np.round(x)) or x.min() < 0:
                    raise ArgumentError(f"{n}: discrete observations must be non-negative integers")
                if dist.fam == abi.MMB_IR_BINOMIAL:
                    nn = self.host_value(ps[0], ln)
                    if nn is None:
                        raise ArgumentError(f"Binomial n of {n} must be data")
                    if np.any(x > nn):
                        raise ArgumentError(f"{n}: Binomial observations exceed n")
                    ct = [math.lgamma(a + 1) - math.lgamma(k + 1) - math.lgamma(a - k + 1) for a, k in zip(nn, x)]
                    N.cterm = self.put(("ct", n), ct)
                elif dist.fam == abi.MMB_IR_POISSON:
                    N.cterm = self.put(("ct", n), [-math.lgamma(k + 1) for k in x])
                elif np.any((x != 0) & (x != 1)):
                    raise ArgumentError(f"{n}: Bernoulli observations must be 0/1")
            parents[n] = refs
        # targets (stochastic children through logicals) and topological order
        children = {n: [c for c in m.stoch if n in parents[c]] for n in m.stoch}
        indeg = {n: sum(1 for p in parents[n] if p != n) for n in m.stoch}
        topo, ready = [], [n for n in m.stoch if indeg[n] == 0]
        while ready:
            ready.sort(key=lambda x: ids[x])
            n = ready.pop(0)
            topo.append(n)
            for c in children[n]:
                if c != n:
                    indeg[c] -= 1
                    if indeg[c] == 0:
                        ready.append(c)
        if len(topo) != len(m.stoch):
            raise ArgumentError("the model graph has a cycle")
        ir = abi.IrModel()
        for b, s in enumerate(m.samplers):
            targets = {c for p in s.params for c in children[p]}
            terms = [p for p in s.params if p not in targets] + [t for t in topo if t in targets]
            if len(terms) > abi.MMB_IR_MAX_TERMS:
                raise ArgumentError("too many nodes in one block's logpdf!")
            ir.blocks[b].nterms = len(terms)
            for t, nm in enumerate(terms):
                ir.blocks[b].term[t] = ids[nm]
                ir.blocks[b].trans[t] = int(nm in s.params)
            s.targets = [t for t in topo if t in targets]
        mon, names = [], []
        for n in m.order:
            d = m.defs[n]
            if not d.monitor:
                continue
            N = nodes[ids[n]]
            mon.append(ids[n])
            names += [n] if (d.dim == 0 and N.len == 1) else [f"{n}[{i + 1}]" for i in range(N.len)]
        if self.depth > abi.MMB_IR_MAX_STACK:
            raise ArgumentError("node expression too deep")
        m.monitor_names = names
        m.topo = topo
        keep = {"nodes": nodes, "code": np.asarray(self.code, dtype=np.int32),
                "consts": np.asarray(self.consts + [0.0], dtype=np.float64),
                "pool": np.asarray(self.pool + [0.0], dtype=np.float64),
                "mon": np.asarray(mon + [0], dtype=np.int32)}
        ir.nvalues = m.nvalues
        ir.nnodes = len(m.order)
        ir.nodes = nodes
        ir.ncode = len(self.code)
        ir.code = keep["code"].ctypes.data_as(C.POINTER(C.c_int32))
        ir.nconst = len(self.consts)
        ir.consts = keep["consts"].ctypes.data_as(C.POINTER(C.c_double))
        ir.npool = len(self.pool)
        ir.pool = keep["pool"].ctypes.data_as(C.POINTER(C.c_double))
        ir.nmon = len(mon)
        ir.mon = keep["mon"].ctypes.data_as(C.POINTER(C.c_int32))
        ir.stack = self.depth
        m._ir, m._ir_keep = ir, keep


# ------------------------------------------------------------------ reference examples

def line_model():
    """doc/tutorial/line.jl:5-25 written in the IR (mu = xmat * beta as beta[1] + beta[2] x)."""
    return Model(
        y=Stochastic(1, lambda mu, s2: MvNormal(mu, sqrt(s2)), False),
        mu=Logical(1, lambda x, beta: beta[1] + beta[2] * x, False),
        beta=Stochastic(1, lambda: MvNormal(2, math.sqrt(1000))),
        s2=Stochastic(lambda: InverseGamma(0.001, 0.001)))


def rats_model():
    """doc/examples/rats.jl:48-97 (y rat-major, 1-based `rat` index, Xm = x[week] - xbar)."""
    return Model(
        y=Stochastic(1, lambda alpha, beta, rat, Xm, s2_c: MvNormal(alpha[rat] + beta[rat] * Xm, sqrt(s2_c)),
                     False),
        alpha=Stochastic(1, lambda mu_alpha, s2_alpha: Normal(mu_alpha, sqrt(s2_alpha)), False),
        alpha0=Logical(lambda mu_alpha, xbar, mu_beta: mu_alpha - xbar * mu_beta),
        mu_alpha=Stochastic(lambda: Normal(0.0, 1000), False),
        s2_alpha=Stochastic(lambda: InverseGamma(0.001, 0.001), False),
        beta=Stochastic(1, lambda mu_beta, s2_beta: Normal(mu_beta, sqrt(s2_beta)), False),
        mu_beta=Stochastic(lambda: Normal(0.0, 1000)),
        s2_beta=Stochastic(lambda: InverseGamma(0.001, 0.001), False),
        s2_c=Stochastic(lambda: InverseGamma(0.001, 0.001)))


def rats_inputs():
    from .model import RATS_DATA
    x = np.asarray(RATS_DATA["x"])
    xbar = x.mean()
    i = np.arange(150)
    return {"y": RATS_DATA["y"], "rat": i // 5 + 1.0, "Xm": x[i % 5] - xbar, "xbar": xbar}


SEEDS = {  # doc/examples/seeds.jl:4-12
    "r": [10, 23, 23, 26, 17, 5, 53, 55, 32, 46, 10, 8, 10, 8, 23, 0, 3, 22, 15, 32, 3],
    "n": [39, 62, 81, 51, 39, 6, 74, 72, 51, 79, 13, 16, 30, 28, 45, 4, 12, 41, 30, 51, 7],
    "x1": [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1],
    "x2": [0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1]}


def seeds_model():
    """doc/examples/seeds.jl:16-56 (random-effect logistic regression, Binomial)."""
    return Model(
        r=Stochastic(1, lambda alpha0, alpha1, x1, alpha2, x2, alpha12, b, n:
                     Binomial(n, invlogit(alpha0 + alpha1 * x1 + alpha2 * x2 + alpha12 * x1 * x2 + b)), False),
        b=Stochastic(1, lambda s2: Normal(0, sqrt(s2)), False),
        alpha0=Stochastic(lambda: Normal(0, 1000)),
        alpha1=Stochastic(lambda: Normal(0, 1000)),
        alpha2=Stochastic(lambda: Normal(0, 1000)),
        alpha12=Stochastic(lambda: Normal(0, 1000)),
        s2=Stochastic(lambda: InverseGamma(0.001, 0.001)))


def seeds_inits():
    """doc/examples/seeds.jl:60-65"""
    r = SEEDS["r"]
    return [{"r": r, "alpha0": 0, "alpha1": 0, "alpha2": 0, "alpha12": 0, "s2": 0.01, "b": [0.0] * 21},
            {"r": r, "alpha0": 0, "alpha1": 0, "alpha2": 0, "alpha12": 0, "s2": 1, "b": [0.0] * 21}]


PUMPS = {"y": [5, 1, 5, 14, 3, 19, 1, 1, 4, 22],                       # doc/examples/pumps.jl:4-8
         "t": [94.3, 15.7, 62.9, 126, 5.24, 31.4, 1.05, 1.05, 2.1, 10.5]}


def pumps_model():
    """doc/examples/pumps.jl:12-39 (Gamma-Poisson hierarchical model)."""
    return Model(
        y=Stochastic(1, lambda theta, t: Poisson(theta * t), False),
        theta=Stochastic(1, lambda alpha, beta: Gamma(alpha, 1 / beta)),
        alpha=Stochastic(lambda: Exponential(1.0)),
        beta=Stochastic(lambda: Gamma(0.1, 1.0)))


SURGICAL = {"r": [0, 18, 8, 46, 8, 13, 9, 31, 14, 8, 29, 24],        # doc/examples/surgical.jl:4-8
            "n": [47, 148, 119, 810, 211, 196, 148, 215, 207, 97, 256, 360]}


def surgical_model():
    """doc/examples/surgical.jl:12-41 (random-effects logistic, Logical p and pop_mean)."""
    return Model(
        r=Stochastic(1, lambda n, p: Binomial(n, p), False),
        p=Logical(1, lambda b: invlogit(b)),
        b=Stochastic(1, lambda mu, s2: Normal(mu, sqrt(s2)), False),
        mu=Stochastic(lambda: Normal(0, 1000)),
        pop_mean=Logical(lambda mu: invlogit(mu)),
        s2=Stochastic(lambda: InverseGamma(0.001, 0.001)))


DYES_Y = [1545, 1440, 1440, 1520, 1580, 1540, 1555, 1490, 1560, 1495, 1595, 1550, 1605, 1510, 1560,
          1445, 1440, 1595, 1465, 1545, 1595, 1630, 1515, 1635, 1625, 1520, 1455, 1450, 1480, 1445]


def dyes_model():
    """doc/examples/dyes.jl:22-45 (variance components, MvNormal with a batch gather)."""
    return Model(
        y=Stochastic(1, lambda mu, batch, s2_within: MvNormal(mu[batch], sqrt(s2_within)), False),
        mu=Stochastic(1, lambda theta, s2_between: Normal(theta, sqrt(s2_between))),
        theta=Stochastic(lambda: Normal(0, 1000)),
        s2_within=Stochastic(lambda: InverseGamma(0.001, 0.001)),
        s2_between=Stochastic(lambda: InverseGamma(0.001, 0.001)))


def dyes_inputs():
    return {"y": DYES_Y, "batch": np.repeat(np.arange(1, 7), 5).astype(float)}


SALM = {"y": [15, 21, 29, 16, 18, 21, 16, 26, 33, 27, 41, 60, 33, 38, 41, 20, 27, 42],  # 3 x 6, column-major
        "x": [0.0, 10, 33, 100, 333, 1000],                                            # doc/examples/salm.jl:4-11
        "dose": np.repeat(np.arange(1, 7), 3).astype(float)}                          # column index of y[i, j]


def salm_model():
    """doc/examples/salm.jl:15-47 (Poisson log-linear dose response with plate effects; the
    node `lambda` is `lam` here, a Python keyword)."""
    return Model(
        y=Stochastic(2, lambda alpha, beta, gamma, x, dose, lam:
                     Poisson(exp(alpha + beta * log(x[dose] + 10) + gamma * x[dose] + lam)), False),
        alpha=Stochastic(lambda: Normal(0, 1000)),
        beta=Stochastic(lambda: Normal(0, 1000)),
        gamma=Stochastic(lambda: Normal(0, 1000)),
        lam=Stochastic(2, lambda s2: Normal(0, sqrt(s2)), False),
        s2=Stochastic(lambda: InverseGamma(0.001, 0.001)))


def salm_inits():
    """doc/examples/salm.jl:51-56"""
    y = SALM["y"]
    return [{"y": y, "alpha": 0, "beta": 0, "gamma": 0, "s2": 10, "lam": np.zeros(18)},
            {"y": y, "alpha": 1, "beta": 1, "gamma": 0.01, "s2": 1, "lam": np.zeros(18)}]


BLOCKER = {  # doc/examples/blocker.jl:4-17
    "rt": [3, 7, 5, 102, 28, 4, 98, 60, 25, 138, 64, 45, 9, 57, 25, 33, 28, 8, 6, 32, 27, 22],
    "nt": [38, 114, 69, 1533, 355, 59, 945, 632, 278, 1916, 873, 263, 291, 858, 154, 207, 251, 151, 174, 209,
           391, 680],
    "rc": [3, 14, 11, 127, 27, 6, 152, 48, 37, 188, 52, 47, 16, 45, 31, 38, 12, 6, 3, 40, 43, 39],
    "nc": [39, 116, 93, 1520, 365, 52, 939, 471, 282, 1921, 583, 266, 293, 883, 147, 213, 122, 154, 134, 218,
           364, 674]}


def blocker_model():
    """doc/examples/blocker.jl:21-64 (random-effects meta-analysis of 22 trials)."""
    return Model(
        rc=Stochastic(1, lambda mu, nc: Binomial(nc, invlogit(mu)), False),
        rt=Stochastic(1, lambda mu, delta, nt: Binomial(nt, invlogit(mu + delta)), False),
        mu=Stochastic(1, lambda: Normal(0, 1000), False),
        delta=Stochastic(1, lambda d, s2: Normal(d, sqrt(s2)), False),
        delta_new=Stochastic(lambda d, s2: Normal(d, sqrt(s2))),
        d=Stochastic(lambda: Normal(0, 1000)),
        s2=Stochastic(lambda: InverseGamma(0.001, 0.001)))


def blocker_inits():
    """doc/examples/blocker.jl:68-73"""
    b = BLOCKER
    return [{"rc": b["rc"], "rt": b["rt"], "d": 0, "delta_new": 0, "s2": 1, "mu": np.zeros(22), "delta": np.zeros(22)},
            {"rc": b["rc"], "rt": b["rt"], "d": 2, "delta_new": 2, "s2": 10, "mu": np.full(22, 2.0),
             "delta": np.full(22, 2.0)}]
