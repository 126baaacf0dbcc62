# MambaHIP.jl — the Julia side of the drop-in boundary (SURVEY §8b): ccall bindings of
# include/mamba_hip.h plus the lowering of a Mamba `Model` to an mmb_model_spec, the packing
# of the samplers' tune objects to the engine's canonical tune rows and back, and the branch
# that `mcmc_master!` (src/model/mcmc.jl:36-59) gains.
#
# Julia 0.5 syntax, like the reference.  No Julia toolchain exists in the build image, so this
# file is not executed here: it is the code a maintainer adds as src/hip/MambaHIP.jl and
# `include`s from src/Mamba.jl.  Its tested mirror is the Python host package:
#   lower        <-> mamba.jl_amd/model.py  Model.spec() / samplers.py
#   pack_tune    <-> the canonical tune layout of engine.cpp mmb_get_tune / mmb_set_tune
#   run_chains!  <-> mamba.jl_amd/mcmc.py  mcmc() / mcmc_restart()
#   gelmandiag   <-> mamba.jl_amd/gelman.py gelmandiag_rccl() (mmb_comm_* / mmb_gr_allreduce)
module MambaHIP

using Mamba
import Distributions
import Distributions: Univariate, Multivariate
import Mamba: Model, Sampler, ModelState, ModelChains, Chains, AMWGTune, AMMTune, NUTSTune,
              SliceTune, HMCTune, MALATune, SamplerTune, relist!, unlist, gettune

const libmambahip = "libmambahip"              # on LD_LIBRARY_PATH / DL_LOAD_PATH

# ---- constants of include/mamba_hip.h -----------------------------------------------------
const MMB_E_UNSUPPORTED = Int32(-2)
const MMB_MODEL_LINE, MMB_MODEL_RATS, MMB_MODEL_LOGISTIC = Int32(1), Int32(2), Int32(3)
const MMB_SAMPLER_AMWG, MMB_SAMPLER_AMM, MMB_SAMPLER_NUTS, MMB_SAMPLER_SLICE = Int32(1), Int32(2), Int32(3), Int32(4)
const MMB_SAMPLER_GIBBS, MMB_SAMPLER_HMC, MMB_SAMPLER_MALA = Int32(5), Int32(6), Int32(7)
const MMB_ADAPT = Dict(:all => Int32(0), :burnin => Int32(1), :none => Int32(2))
const MMB_GRAD_DEFAULT, MMB_GRAD_FORWARD, MMB_GRAD_ANALYTIC = Int32(0), Int32(1), Int32(2)  # mmb_gradient
# dtype of NUTS / HMC / MALA -> mmb_gradient.  :forward is the reference's default (Calculus,
# simulation.jl:47-51), passed as MMB_GRAD_FORWARD: the logistic kernel has no forward-difference
# gradient and mmb_create answers MMB_E_UNSUPPORTED, so that model keeps the Julia path instead of
# silently getting another gradient.  :analytic is MambaHIP's opt-in to the hand-derived gradient
# (line, logistic); the Julia-side Sampler is built with :forward (Calculus has no :analytic).
const MMB_GRAD = Dict(:forward => MMB_GRAD_FORWARD, :analytic => MMB_GRAD_ANALYTIC)
julia_dtype(dtype::Symbol) = dtype == :analytic ? :forward : dtype
const MMB_COMM_ID_BYTES = 128

# ---- structs (layout-checked against the header by tests/test_abi.py on the Python side) ----
immutable BlockSpec                      # mmb_block_spec
  sampler::Int32; nnodes::Int32; nodes::NTuple{4,Int32}
  adapt::Int32; form::Int32; transform::Int32; batchsize::Int32
  target::Float64; beta::Float64; scale::Float64
  dim::Int32; ntuning::Int32; tuning::Ptr{Float64}
  epsilon::Float64; nsteps::Int32; gradient::Int32
end
const NOBLOCK = BlockSpec(0, 0, (0, 0, 0, 0), 0, 0, 0, 0, 0.0, 0.0, 0.0, 0, 0, C_NULL, 0.0, 0, 0)

immutable ModelSpec                      # mmb_model_spec
  model::Int32; nblocks::Int32; blocks::NTuple{8,BlockSpec}
  nobs::Int32; ncoef::Int32; prior_sd::Float64; reserved::NTuple{8,Int32}
end

type RunArgs                             # mmb_run_args (passed by reference)
  iters::Int64; burnin::Int64; thin::Int64; model_burnin::Int64
  draws::Ptr{Float64}; keep_device::Int32; time_kernels::Int32
end

# ---- raw bindings --------------------------------------------------------------------------
last_error(e) = unsafe_string(ccall((:mmb_last_error, libmambahip), Cstring, (Ptr{Void},), e))
check(rc, e) = rc == 0 ? nothing :
  throw(rc == -1 ? ArgumentError(last_error(e)) : ErrorException("libmambahip error $rc: " * last_error(e)))

function create(spec::ModelSpec, device::Integer)
  h = Ref{Ptr{Void}}(C_NULL)
  rc = ccall((:mmb_create, libmambahip), Cint, (Ref{ModelSpec}, Cint, Ref{Ptr{Void}}), spec, device, h)
  rc == MMB_E_UNSUPPORTED && return nothing          # not lowered: the caller keeps the Julia path
  check(rc, C_NULL); h[]
end
destroy(e) = ccall((:mmb_destroy, libmambahip), Void, (Ptr{Void},), e)
set_data!(e, name::AbstractString, x::Vector{Float64}) =
  check(ccall((:mmb_set_data, libmambahip), Cint, (Ptr{Void}, Cstring, Ptr{Float64}, Int64),
              e, name, x, length(x)), e)
num_values(e)    = ccall((:mmb_num_values, libmambahip), Cint, (Ptr{Void},), e)
num_monitored(e) = ccall((:mmb_num_monitored, libmambahip), Cint, (Ptr{Void},), e)
init_chains!(e, init::Matrix{Float64}, offset::Integer, seed::UInt64) =   # P x K (column = chain)
  check(ccall((:mmb_init_chains, libmambahip), Cint, (Ptr{Void}, Ptr{Float64}, Int64, Int64, UInt64),
              e, init, size(init, 2), offset, seed), e)
run!(e, a::RunArgs) = check(ccall((:mmb_run, libmambahip), Cint, (Ptr{Void}, Ref{RunArgs}), e, a), e)
get_values!(e, v::Matrix{Float64}) =
  check(ccall((:mmb_get_values, libmambahip), Cint, (Ptr{Void}, Ptr{Float64}), e, v), e)
tune_len(e) = ccall((:mmb_tune_len, libmambahip), Int64, (Ptr{Void},), e)
get_tune!(e, t::Matrix{Float64}) = check(ccall((:mmb_get_tune, libmambahip), Cint, (Ptr{Void}, Ptr{Float64}), e, t), e)
set_tune!(e, t::Matrix{Float64}) = check(ccall((:mmb_set_tune, libmambahip), Cint, (Ptr{Void}, Ptr{Float64}), e, t), e)
set_iter!(e, it::Integer) = check(ccall((:mmb_set_iter, libmambahip), Cint, (Ptr{Void}, Int64), e, it), e)
gr_len(e) = ccall((:mmb_gr_len, libmambahip), Int64, (Ptr{Void},), e)
num_kept(e) = ccall((:mmb_num_kept, libmambahip), Int64, (Ptr{Void},), e)
reserve_draws(e, nkept::Integer) =
    check(ccall((:mmb_reserve_draws, libmambahip), Cint, (Ptr{Void}, Int64), e, nkept), e)

# the one collective (mmb_comm_*): RCCL over xGMI inside the library
function comm_id()
  id = zeros(UInt8, MMB_COMM_ID_BYTES)
  check(ccall((:mmb_comm_id, libmambahip), Cint, (Ptr{UInt8},), id), C_NULL); id
end
function comm_init(engines::Vector{Ptr{Void}}, nranks::Integer=length(engines), rank0::Integer=0,
                   id::Vector{UInt8}=UInt8[])
  c = Ref{Ptr{Void}}(C_NULL)
  check(ccall((:mmb_comm_init, libmambahip), Cint,
              (Ptr{Ptr{Void}}, Cint, Cint, Cint, Ptr{UInt8}, Ref{Ptr{Void}}),
              engines, length(engines), nranks, rank0, isempty(id) ? C_NULL : pointer(id), c), engines[1])
  c[]
end
comm_destroy(c) = ccall((:mmb_comm_destroy, libmambahip), Void, (Ptr{Void},), c)
# diagnostics: AMM factorization counters per sampling block (adaptive updates, rank(F) == n,
# rank sum, executed steps, redone passes; amm.jl:81-90) and which node-IR kernel an engine runs
const MMB_AMM_STATS = 5
function amm_stats(e)
  out = zeros(Int64, MMB_AMM_STATS, 8)
  check(ccall((:mmb_amm_stats, libmambahip), Cint, (Ptr{Void}, Ptr{Int64}), e, out), e); out
end
# AMWG block updates that ran the sequential coordinate loop (amwg_sub!, amwg.jl:97-115)
function amwg_stats(e)
  out = zeros(Int64, 1)
  check(ccall((:mmb_amwg_stats, libmambahip), Cint, (Ptr{Void}, Ptr{Int64}), e, out), e); out[1]
end
# the slot -> chain table of the last window (wavefront pairing; results do not depend on it)
function chain_order(e, K)
  out = zeros(Int32, K)
  check(ccall((:mmb_chain_order, libmambahip), Cint, (Ptr{Void}, Ptr{Int32}), e, out), e); out
end
function ir_jit_info(e)
  buf = zeros(UInt8, 4096)
  r = ccall((:mmb_ir_jit_info, libmambahip), Cint, (Ptr{Void}, Ptr{UInt8}, Int64), e, buf, length(buf))
  r < 0 && check(r, e)
  (r == 1, unsafe_string(pointer(buf)))
end
function range_allreduce(c, e, p::Integer)
  mm = Array{Float64}(2, p)
  check(ccall((:mmb_range_allreduce, libmambahip), Cint, (Ptr{Void}, Ptr{Float64}), c, mm), e); mm
end
function gr_allreduce(c, e, link::Vector{Int32}, shift::Vector{Float64})
  out = Array{Float64}(gr_len(e))
  check(ccall((:mmb_gr_allreduce, libmambahip), Cint, (Ptr{Void}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64}),
              c, link, shift, out), e); out
end

# ---- sampler registry ------------------------------------------------------------------------
# `Sampler(params, samplerfx, tune)` stores `modelfx(samplerfxargs, samplerfx)` in `s.eval`
# (src/samplers/sampler.jl:22-24): a new top-level function `eval`'d from an AST
# (src/utils.jl:3-12) whose body names the closure as a literal.  It has no fields, so a
# sampler's constructor arguments (sigma, Sigma, width, form, pargs, adapt, keyword args)
# cannot be read back from the Sampler.  The MambaHIP constructors below call Mamba's own and
# record those arguments here, keyed by the `s.eval` object: `mcmc` deep-copies the Model
# (src/model/mcmc.jl:27), which copies every Sampler but returns a field-less object itself
# (Base deepcopy_internal: `nfields(T) == 0 && return x`), so the key survives the copy.
# `lower` reads only this registry; an unregistered block keeps the Julia path.
immutable HIPSampler
  kind::Int32
  pargs::Tuple                     # positional constructor arguments after `params`
  kwargs::Dict{Symbol,Any}         # keyword arguments, incl. `adapt` with its default
end
const REGISTRY = ObjectIdDict()

function register(s::Sampler, kind::Int32, pargs::Tuple, kwargs)
  d = Dict{Symbol,Any}()
  for (k, v) in kwargs; d[k] = v; end
  REGISTRY[s.eval] = HIPSampler(kind, pargs, d)
  s
end
registered(s::Sampler) = get(REGISTRY, s.eval, nothing)
kwarg(r::HIPSampler, name::Symbol, default) = get(r.kwargs, name, default)

"A Gibbs block the engine runs natively: `Sampler(params, f, GibbsTune())` with f the
conjugate full conditional of INTEGRATION.md §3 (the Julia path still calls f)."
type GibbsTune <: SamplerTune end
Gibbs(params::Vector{Symbol}, f::Function) =
  register(Sampler(params, f, GibbsTune()), MMB_SAMPLER_GIBBS, (), ())

# Same signatures and defaults as the reference constructors; each returns Mamba's Sampler.
AMWG(params, sigma; adapt::Symbol=:all, args...) =                           # amwg.jl:47-61
  register(Mamba.AMWG(params, sigma; adapt=adapt, args...), MMB_SAMPLER_AMWG, (sigma,),
           Any[(:adapt, adapt), args...])
AMM(params, Sigma::Matrix; adapt::Symbol=:all, args...) =                    # amm.jl:45-59
  register(Mamba.AMM(params, Sigma; adapt=adapt, args...), MMB_SAMPLER_AMM, (Sigma,),
           Any[(:adapt, adapt), args...])
NUTS(params; dtype::Symbol=:forward, args...) =                              # nuts.jl:47-56
  register(Mamba.NUTS(params; dtype=julia_dtype(dtype), args...), MMB_SAMPLER_NUTS, (),
           Any[(:dtype, dtype), args...])
Slice(params, width, F::Type=Multivariate; transform::Bool=false) =          # slice.jl:47-58
  register(Mamba.Slice(params, width, F; transform=transform), MMB_SAMPLER_SLICE, (width, F),
           Any[(:transform, transform)])
HMC(params, epsilon::Real, L::Integer, pargs...; dtype::Symbol=:forward) =   # hmc.jl:47-65
  register(Mamba.HMC(params, epsilon, L, pargs...; dtype=julia_dtype(dtype)), MMB_SAMPLER_HMC,
           (epsilon, L, pargs...), Any[(:dtype, dtype)])
MALA(params, epsilon::Real, pargs...; dtype::Symbol=:forward) =              # mala.jl:43-58
  register(Mamba.MALA(params, epsilon, pargs...; dtype=julia_dtype(dtype)), MMB_SAMPLER_MALA,
           (epsilon, pargs...), Any[(:dtype, dtype)])

# tune type each constructor creates (amwg.jl:60, amm.jl:58, nuts.jl:55, slice.jl:57,
# hmc.jl:64, mala.jl:59): a registered block must still carry it
const TUNE_OF = Dict(MMB_SAMPLER_AMWG => AMWGTune, MMB_SAMPLER_AMM => AMMTune, MMB_SAMPLER_NUTS => NUTSTune,
                     MMB_SAMPLER_SLICE => SliceTune, MMB_SAMPLER_HMC => HMCTune, MMB_SAMPLER_MALA => MALATune,
                     MMB_SAMPLER_GIBBS => GibbsTune)

# ---- model lowering --------------------------------------------------------------------------
# Engine value layout per model kind (include/mamba_hip.h node ids; model.py offsets):
const LAYOUT = Dict(
  MMB_MODEL_LINE => [(:beta, 0, 2), (:s2, 1, 1)],                         # doc/tutorial/line.jl:5-25
  MMB_MODEL_RATS => [(:s2_c, 0, 1), (:alpha, 1, 30), (:mu_alpha, 2, 1), (:s2_alpha, 3, 1),
                     (:beta, 4, 30), (:mu_beta, 5, 1), (:s2_beta, 6, 1)],  # doc/examples/rats.jl:48-97
  MMB_MODEL_LOGISTIC => [(:beta, 0, 0)])                                   # SURVEY §8a, p from the node

function model_kind(m::Model)
  ks = Set(keys(m, :dependent))                     # Logical + Stochastic nodes (inputs excluded)
  ks == Set([:y, :beta, :s2, :mu]) && return MMB_MODEL_LINE
  ks == Set([:y, :alpha, :alpha0, :mu_alpha, :s2_alpha, :beta, :mu_beta, :s2_beta, :s2_c]) &&
    return MMB_MODEL_RATS
  ks == Set([:y, :p, :beta]) && return MMB_MODEL_LOGISTIC
  nothing                                           # any other DAG: lower_ir (node IR, below)
end

node_id(kind, key::Symbol) = (for (k, id, _) in LAYOUT[kind]; k == key && return id; end; nothing)
fillvec(x, n) = isa(x, Real) ? fill(Float64(x), n) : Float64[x...]

"Sampler b -> BlockSpec (+ buffers to keep alive), or nothing when the block is not registered.
Argument errors are the reference's own (amwg.jl:37-42, amm.jl:35-40, slice.jl:36-43, hmc.jl:38-44)."
function block_spec(s::Sampler, nodes::NTuple{4,Int32}, nnodes::Integer, dim::Integer, keep::Vector{Any})
  r = registered(s)
  r === nothing && return nothing                   # an arbitrary user closure: keep the Julia path
  isa(s.tune, TUNE_OF[r.kind]) || return nothing
  grad = get(MMB_GRAD, kwarg(r, :dtype, :forward), Int32(-1))
  blk(adapt_, form, transform, batchsize, target, beta, scale, tun, eps, L) =
    BlockSpec(r.kind, nnodes, nodes, adapt_, form, transform, batchsize, target, beta, scale, dim,
              length(tun), isempty(tun) ? C_NULL : pointer(tun), eps, L,
              r.kind in (MMB_SAMPLER_NUTS, MMB_SAMPLER_HMC, MMB_SAMPLER_MALA) ? grad : MMB_GRAD_DEFAULT)
  adapt = MMB_ADAPT[kwarg(r, :adapt, :none)]
  if r.kind == MMB_SAMPLER_GIBBS
    return blk(MMB_ADAPT[:none], 0, 0, 0, 0.0, 0.0, 0.0, Float64[], 0.0, 0)
  elseif r.kind == MMB_SAMPLER_AMWG                                            # amwg.jl:5-33
    sig = fillvec(r.pargs[1], dim); push!(keep, sig)
    length(sig) == dim || throw(ArgumentError("length(sigma) differs from variate length $dim"))
    return blk(adapt, 0, 1, kwarg(r, :batchsize, 50), kwarg(r, :target, 0.44), 0.0, 0.0, sig, 0.0, 0)
  elseif r.kind == MMB_SAMPLER_AMM                                             # amm.jl:5-30
    Sig = vec(Float64[r.pargs[1]...]); push!(keep, Sig)                         # column-major
    size(r.pargs[1], 1) == dim || throw(ArgumentError("Sigma dimension differs from variate length $dim"))
    return blk(adapt, 0, 1, 0, 0.0, kwarg(r, :beta, 0.05), kwarg(r, :scale, 2.38), Sig, 0.0, 0)
  elseif r.kind == MMB_SAMPLER_NUTS                                            # nuts.jl:5-39
    # :forward (Calculus forward differences, simulation.jl:47-51; refused by the logistic kernel:
    # MMB_E_UNSUPPORTED -> Julia path) or :analytic (MMB_GRAD); any other dtype keeps the Julia path
    grad < 0 && return nothing
    return blk(MMB_ADAPT[:burnin], 0, 1, 0, kwarg(r, :target, 0.6), 0.0, 0.0, Float64[], 0.0, 0)
  elseif r.kind == MMB_SAMPLER_SLICE                                           # slice.jl:7-26
    w = fillvec(r.pargs[1], dim); push!(keep, w)
    length(w) == dim || throw(ArgumentError("length(width) differs from variate length $dim"))
    form = r.pargs[2] == Univariate ? Int32(1) : Int32(0)
    return blk(MMB_ADAPT[:none], form, Int32(kwarg(r, :transform, false)), 0, 0.0, 0.0, 0.0, w, 0.0, 0)
  else                                                                         # hmc.jl:5-32, mala.jl:5-30
    grad < 0 && return nothing
    hmc = r.kind == MMB_SAMPLER_HMC
    nS = hmc ? 3 : 2                                  # (epsilon, L[, Sigma]) / (epsilon[, Sigma])
    S = length(r.pargs) >= nS ? vec(Float64[r.pargs[nS]...]) : Float64[]; push!(keep, S)
    isempty(S) || size(r.pargs[nS], 1) == dim ||
      throw(ArgumentError("Sigma dimension differs from variate length $dim"))
    return blk(MMB_ADAPT[:none], 0, 1, 0, 0.0, 0.0, 0.0, S, Float64(r.pargs[1]),
               hmc ? Int32(r.pargs[2]) : Int32(0))
  end
end

"Model -> (ModelSpec, buffers to keep alive) or nothing (Julia path).  Mirror: model.py Model.spec()."
function lower(m::Model)
  kind = model_kind(m)
  kind === nothing && return nothing
  length(m.samplers) > 8 && return nothing
  blocks = fill(NOBLOCK, 8)
  keep = Any[]
  for (b, s) in enumerate(m.samplers)
    length(s.params) > 4 && return nothing
    ids = Int32[]
    for p in s.params
      id = node_id(kind, p)
      id === nothing && return nothing
      push!(ids, id)
    end
    nodes = ntuple(i -> i <= length(ids) ? ids[i] : Int32(0), 4)
    dim = sum(p -> length(m[p].value), s.params)
    sp = block_spec(s, nodes, length(ids), dim, keep)
    sp === nothing && return nothing
    blocks[b] = sp
  end
  nobs = kind == MMB_MODEL_LOGISTIC ? length(m[:y].value) : 0
  ncoef = kind == MMB_MODEL_LOGISTIC ? length(m[:beta].value) : 0
  prior_sd = kind == MMB_MODEL_LOGISTIC ? sqrt(m[:beta].distr.Σ.value) : 0.0
  (ModelSpec(kind, length(m.samplers), tuple(blocks...), nobs, ncoef, prior_sd, ntuple(_ -> Int32(0), 8)), keep)
end

# ---- node IR lowering (any other Model: MMB_MODEL_IR, mmb_create_ir; INTEGRATION.md §2a) ------
# Mirror: mamba.jl_amd/ir.py.  Each node's own function (node.eval, src/model/dependent.jl:75-
# 152, src/utils.jl:3-43) is called once on a tracer Model whose sampled Stochastic nodes are
# arrays of scalar expression trees (element k of node s = TElem(s, k)), whose inputs and
# fixed (unsampled) Stochastic nodes are their actual values, and whose Logical nodes hold
# the trees their own functions return (so Logicals are inlined).  Node functions run
# unchanged: `alpha[rat] + beta[rat] .* Xm`, `xmat * beta`, `UnivariateDistribution[...
# for i in 1:N]` comprehensions all evaluate to per-element trees, because TExpr is a Number
# whose arithmetic records itself.  The per-element trees of a node parameter are then
# anti-unified into ONE elementwise expression of the IR (element i: CONST, VAL, VALI, VALG
# gathers, DATA vectors) -- the broadcast form mmb_ir_node expects.  Anything else (a closure
# that branches on a node value, a distribution outside the IR's families, a partial monitor,
# a user Gibbs closure) raises inside the trace or the unification and `lower_ir` returns
# `nothing`: the unchanged Julia path runs.
const MMB_MODEL_IR = Int32(4)
const MMB_IR_NORMAL, MMB_IR_ISONORMAL, MMB_IR_INVGAMMA, MMB_IR_GAMMA = Int32(1), Int32(2), Int32(3), Int32(4)
const MMB_IR_EXPONENTIAL, MMB_IR_UNIFORM, MMB_IR_BETA = Int32(5), Int32(6), Int32(7)
const MMB_IR_BINOMIAL, MMB_IR_POISSON, MMB_IR_BERNOULLI, MMB_IR_LOGICAL = Int32(8), Int32(9), Int32(10), Int32(11)
const IR_OP = Dict(:end => 0, :const => 1, :val => 2, :vali => 3, :valg => 4, :data => 5, :datas => 6,
                   :+ => 16, :- => 17, :* => 18, :/ => 19,
                   :neg => 32, :exp => 33, :log => 34, :sqrt => 35, :invlogit => 36, :logit => 37, :abs => 38)
const MMB_IR_MAX_STACK, MMB_IR_MAX_TERMS, MMB_IR_MAX_VALUES = 16, 16, 512
const IR_SAMPLEABLE = [MMB_IR_NORMAL, MMB_IR_ISONORMAL, MMB_IR_INVGAMMA, MMB_IR_GAMMA, MMB_IR_EXPONENTIAL,
                       MMB_IR_UNIFORM, MMB_IR_BETA]
const IR_DISCRETE = [MMB_IR_BINOMIAL, MMB_IR_POISSON, MMB_IR_BERNOULLI]

immutable IrNode                         # mmb_ir_node
  family::Int32; fixed::Int32; off::Int32; len::Int32
  expr::NTuple{3,Int32}; cterm::Int32; lo::Float64; hi::Float64
end
immutable IrBlock                        # mmb_ir_block
  nterms::Int32; term::NTuple{16,Int32}; trans::NTuple{16,Int32}
end
const NOIRBLOCK = IrBlock(0, ntuple(_ -> Int32(0), 16), ntuple(_ -> Int32(0), 16))
immutable IrModel                        # mmb_ir_model
  nvalues::Int32; nnodes::Int32; nodes::Ptr{IrNode}; ncode::Int32; code::Ptr{Int32}
  nconst::Int32; consts::Ptr{Float64}; npool::Int64; pool::Ptr{Float64}
  nmon::Int32; mon::Ptr{Int32}; stack::Int32; blocks::NTuple{8,IrBlock}
end

function create_ir(spec::ModelSpec, ir::IrModel, device::Integer)
  h = Ref{Ptr{Void}}(C_NULL)
  rc = ccall((:mmb_create_ir, libmambahip), Cint, (Ref{ModelSpec}, Ref{IrModel}, Cint, Ref{Ptr{Void}}),
             spec, ir, device, h)
  rc == MMB_E_UNSUPPORTED && return nothing
  check(rc, C_NULL); h[]
end

# -- tracer: scalar expression trees ---------------------------------------------------------
abstract TExpr <: Number
immutable TConst <: TExpr; v::Float64; end
immutable TElem <: TExpr; node::Symbol; k::Int; end       # element k (1-based) of a sampled node
immutable TBin <: TExpr; op::Symbol; a::TExpr; b::TExpr; end
immutable TUn <: TExpr; op::Symbol; a::TExpr; end

Base.convert(::Type{TExpr}, x::Real) = TConst(Float64(x))
Base.convert(::Type{TExpr}, x::TExpr) = x
Base.promote_rule{S<:TExpr, T<:Real}(::Type{S}, ::Type{T}) = TExpr
Base.promote_rule{S<:TExpr, T<:TExpr}(::Type{S}, ::Type{T}) = TExpr
Base.zero{T<:TExpr}(::Type{T}) = TConst(0.0)             # generic matmul / sum start
Base.zero(::TExpr) = TConst(0.0)
for op in (:+, :-, :*, :/)
  @eval Base.$op(a::TExpr, b::TExpr) = TBin($(QuoteNode(op)), a, b)
end
Base.:-(a::TExpr) = TUn(:neg, a)
Base.:+(a::TExpr) = a
Base.:^(a::TExpr, p::Integer) = p == 2 ? a * a : throw(ArgumentError("node IR: only x^2"))
for f in (:exp, :log, :sqrt, :abs)
  @eval Base.$f(a::TExpr) = TUn($(QuoteNode(f)), a)
end
Mamba.invlogit(a::TExpr) = TUn(:invlogit, a)              # src/utils.jl:64
Mamba.logit(a::TExpr) = TUn(:logit, a)                    # src/utils.jl:67

# -- tracer: distributions of traced parameters -----------------------------------------------
immutable TDist
  fam::Int32
  p::Vector{Any}                        # per parameter: a scalar (TExpr or Real) or a vector of them
end
typealias TR Union{TExpr, Real}
import Distributions: Normal, MvNormal, InverseGamma, Gamma, Exponential, Uniform, Beta, Binomial,
                      Poisson, Bernoulli, ScalMat
# (Real, Real) arguments keep Distributions' own, more specific methods
Normal(mu::TR, s::TR) = TDist(MMB_IR_NORMAL, Any[mu, s])
Normal(mu::TExpr) = TDist(MMB_IR_NORMAL, Any[mu, 1.0])
InverseGamma(a::TR, b::TR) = TDist(MMB_IR_INVGAMMA, Any[a, b])
Gamma(a::TR, b::TR) = TDist(MMB_IR_GAMMA, Any[a, b])
Exponential(b::TExpr) = TDist(MMB_IR_EXPONENTIAL, Any[b])
Uniform(a::TR, b::TR) = TDist(MMB_IR_UNIFORM, Any[a, b])
Beta(a::TR, b::TR) = TDist(MMB_IR_BETA, Any[a, b])
Binomial(n::Real, p::TExpr) = TDist(MMB_IR_BINOMIAL, Any[n, p])
Poisson(l::TExpr) = TDist(MMB_IR_POISSON, Any[l])
Bernoulli(p::TExpr) = TDist(MMB_IR_BERNOULLI, Any[p])
MvNormal{T<:TExpr}(mu::AbstractVector{T}, s::Real) = TDist(MMB_IR_ISONORMAL, Any[mu, s])
MvNormal(mu::AbstractVector, s::TExpr) = TDist(MMB_IR_ISONORMAL, Any[mu, s])
MvNormal(k::Integer, s::TExpr) = TDist(MMB_IR_ISONORMAL, Any[0.0, s])

"A distribution object of constant parameters (no tracer reached it) as a TDist."
function as_tdist(d)
  isa(d, TDist) && return d
  params = Distributions.params
  isa(d, Normal) && return TDist(MMB_IR_NORMAL, Any[params(d)...])
  isa(d, InverseGamma) && return TDist(MMB_IR_INVGAMMA, Any[params(d)...])
  isa(d, Gamma) && return TDist(MMB_IR_GAMMA, Any[params(d)...])
  isa(d, Exponential) && return TDist(MMB_IR_EXPONENTIAL, Any[params(d)...])
  isa(d, Uniform) && return TDist(MMB_IR_UNIFORM, Any[params(d)...])
  isa(d, Beta) && return TDist(MMB_IR_BETA, Any[params(d)...])
  isa(d, Binomial) && return TDist(MMB_IR_BINOMIAL, Any[params(d)...])
  isa(d, Poisson) && return TDist(MMB_IR_POISSON, Any[params(d)...])
  isa(d, Bernoulli) && return TDist(MMB_IR_BERNOULLI, Any[params(d)...])
  if isa(d, MvNormal) && isa(d.Σ, ScalMat)                 # IsoNormal (PDMats ScalMat)
    return TDist(MMB_IR_ISONORMAL, Any[Float64[mean(d)...], sqrt(d.Σ.value)])
  end
  throw(ArgumentError("node IR: distribution $(typeof(d)) is not lowered"))
end

# -- anti-unification of per-element trees into one elementwise IR expression ------------------
# IR expression: (:const, v) | (:val, slot) | (:vali, off) | (:valg, off, idx0) | (:data, vec) |
#                (op, a, b) | (op, a)
function vectorize(ts::Vector, L)                # L: the IR lowering state
  n = length(ts)
  t = map(x -> isa(x, Real) ? TConst(Float64(x)) : x, ts)
  isa(t[1], TExpr) || throw(ArgumentError("node IR: a parameter is not arithmetic"))
  if all(x -> isa(x, TConst), t)
    v = Float64[x.v for x in t]
    return all(x -> x == v[1], v) ? (:const, v[1]) : (:data, v)
  elseif all(x -> isa(x, TElem), t)
    s = t[1].node
    all(x -> x.node == s, t) || throw(ArgumentError("node IR: elements of different nodes in one position"))
    ks = Int[x.k for x in t]
    off = L.slot[s]
    all(k -> k == ks[1], ks) && return (:val, off + ks[1] - 1)
    ks == collect(1:n) && L.len[s] == n && return (:vali, off)
    return (:valg, off, Float64[k - 1 for k in ks])
  elseif all(x -> isa(x, TBin), t)
    op = t[1].op
    all(x -> x.op == op, t) || throw(ArgumentError("node IR: elements differ in an operation"))
    return (op, vectorize(Any[x.a for x in t], L), vectorize(Any[x.b for x in t], L))
  elseif all(x -> isa(x, TUn), t)
    op = t[1].op
    all(x -> x.op == op, t) || throw(ArgumentError("node IR: elements differ in an operation"))
    return (op, vectorize(Any[x.a for x in t], L))
  end
  throw(ArgumentError("node IR: elements of a parameter do not share one expression"))
end

"Elementwise trees of parameter `p` for an n-element node: a scalar is shared by every element."
per_element(p, n) = isa(p, AbstractArray) ? (length(p) == n ? Any[p...] :
                      throw(ArgumentError("node IR: parameter length $(length(p)) for $n elements"))) : Any[p]

type IrLowering
  slot::Dict{Symbol,Int}; len::Dict{Symbol,Int}
  code::Vector{Int32}; consts::Vector{Float64}; pool::Vector{Float64}; depth::Int
end

word(op::Symbol, arg::Integer) = (0 <= arg < 1 << 24 ||
  throw(ArgumentError("node IR operand $arg does not fit in 24 bits")); Int32(IR_OP[op] << 24 | arg))
function pool!(L::IrLowering, v::Vector{Float64})
  off = length(L.pool); append!(L.pool, v); off
end
function emit!(L::IrLowering, e, sp::Int)
  push(w) = (push!(L.code, w); L.depth = max(L.depth, sp + 1); sp + 1)
  k = e[1]
  if k == :const
    push!(L.consts, e[2]); return push(word(:const, length(L.consts) - 1))
  elseif k == :val
    return push(word(:val, e[2]))
  elseif k == :vali
    return push(word(:vali, e[2]))
  elseif k == :valg
    sp2 = push(word(:valg, e[2])); push!(L.code, Int32(pool!(L, e[3]))); return sp2
  elseif k == :data
    return push(word(:data, pool!(L, e[2])))
  elseif length(e) == 3
    sp = emit!(L, e[2], sp); sp = emit!(L, e[3], sp); push!(L.code, word(k, 0)); return sp - 1
  end
  sp = emit!(L, e[2], sp); push!(L.code, word(k, 0)); sp
end
function expr!(L::IrLowering, e)
  start = length(L.code)
  emit!(L, e, 0)
  push!(L.code, Int32(0))                 # END
  Int32(start)
end
host_const(e) = e[1] == :const ? e[2] : throw(ArgumentError("node IR: a bound must be a constant"))
host_data(e, n) = e[1] == :const ? fill(e[2], n) : e[1] == :data ? e[2] :
                  throw(ArgumentError("node IR: Binomial n must be data"))

"""
    lower_ir(m) -> (ModelSpec, IrModel, layout, keep) or nothing

Walks m.nodes (src/model/dependent.jl:75-152, model.jl:5-27) into an mmb_ir_model.  `layout`
lists (node, length) of the sampled nodes in the order of their state slots: the engine value
row of a chain.  Term lists per block are the reference's own: `keys(m, :block, b)` minus the
targets, then the Stochastic nodes of `keys(m, :target, b)` (simulation.jl:79-88).
"""
function lower_ir(m::Model)
  try
    return lower_ir_(m)
  catch err
    isa(err, ArgumentError) || isa(err, MethodError) || isa(err, BoundsError) || rethrow(err)
    return nothing                       # not lowerable: the Julia path
  end
end

function lower_ir_(m::Model)
  length(m.samplers) > 8 && return nothing
  deps = keys(m, :dependent)            # tsorted Logical + Stochastic keys
  inblock = Set(vcat([s.params for s in m.samplers]...))
  stoch = filter(k -> isa(m[k], Mamba.AbstractStochastic), deps)
  sampled = filter(k -> k in inblock, stoch)
  L = IrLowering(Dict{Symbol,Int}(), Dict{Symbol,Int}(), Int32[], Float64[], Float64[], 1)
  off = 0
  for k in sampled                       # state slots: sampled nodes in dependent order
    L.slot[k], L.len[k] = off, length(m[k].value); off += L.len[k]
  end
  1 <= off <= MMB_IR_MAX_VALUES || throw(ArgumentError("node IR: 1..$MMB_IR_MAX_VALUES sampled values"))
  # tracer model: sampled nodes -> element trees, inputs / fixed nodes -> their values
  tm = Model(Dict{Symbol,Any}(), Sampler[], ModelState[], 0, 0, false, false)
  for (k, v) in m.nodes
    if k in inblock
      tm.nodes[k] = isa(v.value, AbstractArray) ?
        reshape(TExpr[TElem(k, i) for i in 1:length(v.value)], size(v.value)) : TElem(k, 1)
    else
      tm.nodes[k] = isa(v, Mamba.AbstractDependent) ? v.value : v
    end
  end
  for k in deps                          # Logicals inlined, in topological order
    isa(m[k], Mamba.AbstractLogical) && (tm.nodes[k] = m[k].eval(tm))
  end
  ids = Dict(k => Int32(i - 1) for (i, k) in enumerate(deps))
  nodes = IrNode[]
  for k in deps
    node = m[k]
    n = length(node.value)
    ex = Int32[-1, -1, -1]
    if isa(node, Mamba.AbstractLogical)
      val = tm.nodes[k]
      ex[1] = expr!(L, vectorize(per_element(isa(val, AbstractArray) ? vec(val) : val, n), L))
      push!(nodes, IrNode(MMB_IR_LOGICAL, 0, 0, n, (ex...), -1, 0.0, 0.0)); continue
    end
    d = node.eval(tm)                    # TDist, a Distribution, or an array of them (per element)
    if isa(d, AbstractArray)
      ds = map(as_tdist, vec(d))
      length(ds) == n || throw(ArgumentError("node IR: $k has $(length(ds)) distributions for $n elements"))
      fam = ds[1].fam
      all(x -> x.fam == fam, ds) || throw(ArgumentError("node IR: $k mixes distribution families"))
      np = length(ds[1].p)
      par = [Any[x.p[j] for x in ds] for j in 1:np]          # parameter j, element i
    else
      dd = as_tdist(d)
      fam = dd.fam
      par = fam == MMB_IR_ISONORMAL ?
        Any[per_element(dd.p[1] == 0.0 ? 0.0 : dd.p[1], isa(dd.p[1], AbstractArray) ? n : 1), Any[dd.p[2]]] :
        [per_element(p, isa(p, AbstractArray) ? n : 1) for p in dd.p]
    end
    fixed = !(k in inblock)
    fixed || fam in IR_SAMPLEABLE || throw(ArgumentError("node IR: $k cannot be sampled by these samplers"))
    vecs = Any[vectorize(p, L) for p in par]
    for (j, e) in enumerate(vecs); ex[j] = expr!(L, e); end
    x = Float64[node.value...]
    lo = hi = 0.0
    cterm = Int32(-1)
    if fam == MMB_IR_UNIFORM
      lo, hi = host_const(vecs[1]), host_const(vecs[2])
    elseif fam in IR_DISCRETE
      fixed || throw(ArgumentError("node IR: discrete node $k cannot be sampled"))
      all(v -> v == round(v) && v >= 0, x) || throw(ArgumentError("node IR: $k: counts must be integers >= 0"))
      if fam == MMB_IR_BINOMIAL
        nn = host_data(vecs[1], n)
        cterm = Int32(pool!(L, Float64[lgamma(a + 1) - lgamma(b + 1) - lgamma(a - b + 1) for (a, b) in zip(nn, x)]))
      elseif fam == MMB_IR_POISSON
        cterm = Int32(pool!(L, Float64[-lgamma(b + 1) for b in x]))
      end
    end
    o = fixed ? pool!(L, x) : L.slot[k]
    push!(nodes, IrNode(fam, fixed ? 1 : 0, o, n, (ex...), cterm, lo, hi))
  end
  L.depth <= MMB_IR_MAX_STACK || throw(ArgumentError("node IR: expression too deep"))
  # blocks: BlockSpec from the sampler registry, term list of logpdf! (simulation.jl:79-88)
  blocks, irb, keep = fill(NOBLOCK, 8), fill(NOIRBLOCK, 8), Any[nodes, L]
  for (b, s) in enumerate(m.samplers)
    length(s.params) > 4 && return nothing
    pids = Int32[ids[p] for p in s.params]
    dim = sum(p -> L.len[p], s.params)
    dim <= 32 || throw(ArgumentError("node IR: blocks of at most 32 elements"))
    sp = block_spec(s, ntuple(i -> i <= length(pids) ? pids[i] : Int32(0), 4), length(pids), dim, keep)
    sp === nothing && return nothing
    blocks[b] = sp
    targets = filter(k -> isa(m[k], Mamba.AbstractStochastic), keys(m, :target, b))
    terms = vcat(setdiff(s.params, targets), targets)
    length(terms) <= MMB_IR_MAX_TERMS || throw(ArgumentError("node IR: too many nodes in one logpdf!"))
    irb[b] = IrBlock(length(terms), ntuple(i -> i <= length(terms) ? ids[terms[i]] : Int32(0), 16),
                     ntuple(i -> i <= length(terms) ? Int32(terms[i] in s.params) : Int32(0), 16))
  end
  # monitored nodes in names(m, true) order (model.jl:231-239): whole nodes only
  mon = Int32[]
  for k in deps
    mk = m[k].monitor
    isempty(mk) && continue
    mk == collect(1:length(m[k].value)) || throw(ArgumentError("node IR: partial monitor of $k"))
    push!(mon, ids[k])
  end
  code, consts, pool = L.code, vcat(L.consts, 0.0), vcat(L.pool, 0.0)
  append!(keep, Any[code, consts, pool, mon])
  ir = IrModel(off, length(nodes), pointer(nodes), length(code), pointer(code), length(L.consts),
               pointer(consts), length(L.pool), pointer(pool), length(mon), pointer(mon), L.depth, (irb...))
  spec = ModelSpec(MMB_MODEL_IR, length(m.samplers), (blocks...), 0, 0, 0.0, ntuple(_ -> Int32(0), 8))
  layout = [(k, L.len[k]) for k in sampled]
  (spec, ir, layout, keep)
end

"One chain's engine value row of a node-IR model (layout from lower_ir)."
ir_values(m::Model, layout) = vcat([Float64[m[k].value...] for (k, _) in layout]...)
function set_ir_values!(m::Model, layout, v::AbstractVector{Float64})
  o = 0
  for (k, n) in layout
    m[k].value = isa(m[k].value, AbstractArray) ? reshape(v[o + (1:n)], size(m[k].value)) : v[o + 1]
    o += n
  end
end

"setinputs! data the kernels read (names of include/mamba_hip.h mmb_set_data)."
function inputs(m::Model, kind)
  kind == MMB_MODEL_LINE && return [("x", Float64[m[:x].value...]), ("y", Float64[m[:y].value...])]
  kind == MMB_MODEL_RATS && return [("y", Float64[m[:y].value...]), ("x", Float64[m[:x].value...])]
  [("X", vec(full(m[:X].value)')), ("y", Float64[m[:y].value...])]                # X row-major
end

"One chain's values in the engine layout (P), after relist!(m, state.value) (mcmc.jl:68-70)."
function engine_values(m::Model, kind)
  vcat([Float64[m[k].value...] for (k, _, _) in LAYOUT[kind]]...)
end
function set_engine_values!(m::Model, kind, v::AbstractVector{Float64})
  o = 0
  for (k, _, _) in LAYOUT[kind]
    n = length(m[k].value)
    m[k].value = n == 1 && isa(m[k].value, Real) ? v[o + 1] : reshape(v[o + (1:n)], size(m[k].value))
    o += n
  end
end

# ---- tune <-> canonical engine tune row (engine.cpp mmb_get_tune / mmb_set_tune) -------------
tri(i) = div(i * (i + 1), 2)                        # 0-based packed-lower helpers (device.h)
slot(i, k) = i >= k ? tri(i) + k : tri(k) + i

"Canonical tune row of block b for one chain from its Julia tune object."
function pack_tune(t, s::Sampler, dim::Integer, iter::Integer)
  if isa(t, AMWGTune)                               # [adapt, m, sigma[d], accept[d]]
    return vcat(Float64(t.adapt), Float64(t.m), t.sigma, Float64[t.accept...])
  elseif isa(t, AMMTune)                            # [adapt, m, valid, alias, Mv, Mvv, Ls, piv]
    T = tri(dim)
    Mv = isempty(t.Mv) ? zeros(dim) : Float64[t.Mv...]
    Mvv, Ls, piv = zeros(T), zeros(T), zeros(dim)
    if !isempty(t.Mvv)
      for i in 0:dim-1, k in 0:i; Mvv[tri(i) + k + 1] = t.Mvv[k + 1, i + 1]; end     # upper semantics
    end
    valid = !isempty(t.SigmaLm) && any(x -> x != 0.0, t.SigmaLm)
    if valid                                        # SigmaLm = P*L: row e's last nonzero = pos(e)
      pos = [findlast(x -> x != 0.0, t.SigmaLm[e + 1, :]) - 1 for e in 0:dim-1]
      for e in 0:dim-1; piv[pos[e + 1] + 1] = e; end
      for e in 0:dim-1
        for k in 0:pos[e + 1]-1; Ls[slot(e, Int(piv[k + 1])) + 1] = t.SigmaLm[e + 1, k + 1]; end
        Ls[slot(e, e) + 1] = t.SigmaLm[e + 1, pos[e + 1] + 1]
      end
    end
    return vcat(Float64(t.adapt), Float64(t.m), Float64(valid), 0.0, Mv, Mvv, Ls, piv)
  elseif isa(t, NUTSTune)                           # [adapt, m, eps, epsbar, Hbar, mu, alpha, nalpha, init]
    return Float64[t.adapt, t.m, t.epsilon, t.epsbar, t.Hbar, t.mu, t.alpha, t.nalpha, iter >= 1]
  elseif isa(t, HMCTune)
    return Float64[t.epsilon, t.L]
  elseif isa(t, MALATune)
    return Float64[t.epsilon]
  end
  Float64[]                                         # Slice, Gibbs: nothing is adapted
end

"Inverse of pack_tune: write one chain's canonical row back into its Julia tune object."
function unpack_tune!(t, row::AbstractVector{Float64}, dim::Integer)
  if isa(t, AMWGTune)
    t.adapt = row[1] != 0; t.m = Int(row[2])
    t.sigma = row[3:2+dim]; t.accept = Int[row[3+dim:2+2dim]...]
  elseif isa(t, AMMTune)
    T = tri(dim)
    t.adapt = row[1] != 0; t.m = Int(row[2])
    t.Mv = row[5:4+dim]
    Mvv = zeros(dim, dim)
    for i in 0:dim-1, k in 0:i; Mvv[k + 1, i + 1] = Mvv[i + 1, k + 1] = row[5 + dim + tri(i) + k]; end
    t.Mvv = Mvv
    if row[3] != 0
      Ls = row[5+dim+T:4+dim+2T]; piv = Int[row[5+dim+2T:4+2dim+2T]...]
      pos = zeros(Int, dim); for k in 0:dim-1; pos[piv[k + 1] + 1] = k; end
      S = zeros(dim, dim)
      for e in 0:dim-1
        for k in 0:pos[e + 1]-1; S[e + 1, k + 1] = Ls[slot(e, piv[k + 1]) + 1]; end
        S[e + 1, pos[e + 1] + 1] = Ls[slot(e, e) + 1]
      end
      t.SigmaLm = S
    else
      t.SigmaLm = zeros(dim, dim)
    end
  elseif isa(t, NUTSTune)
    t.adapt = row[1] != 0; t.m = Int(row[2]); t.epsilon, t.epsbar, t.Hbar, t.mu, t.alpha = row[3:7]
    t.nalpha = Int(row[8])
  elseif isa(t, HMCTune)
    t.epsilon, t.L = row[1], Int(row[2])
  elseif isa(t, MALATune)
    t.epsilon = row[1]
  end
  t
end

"K x TL canonical tune (column = chain) from the per-chain ModelStates."
function pack_tunes(m::Model, states::Vector{ModelState}, iter::Integer)
  cols = Vector{Float64}[]
  for st in states
    row = Float64[]
    for (b, s) in enumerate(m.samplers)
      dim = sum(p -> length(m[p].value), s.params)
      append!(row, pack_tune(st.tune[b], s, dim, iter))
    end
    push!(cols, row)
  end
  hcat(cols...)
end

"m.states[k] = ModelState(values, tune) from the engine after a window (mcmc.jl:54-56, 82)."
function store_states!(m::Model, e, setvals!::Function, states::Vector{ModelState})
  K = length(states)
  vals = Array{Float64}(num_values(e), K); get_values!(e, vals)
  TL = tune_len(e)
  tunes = Array{Float64}(TL, K)
  TL > 0 && get_tune!(e, tunes)
  for k in 1:K
    setvals!(vals[:, k])
    tune = deepcopy(states[k].tune)
    o = 0
    for (b, s) in enumerate(m.samplers)
      dim = sum(p -> length(m[p].value), s.params)
      n = length(pack_tune(tune[b], s, dim, 1))
      unpack_tune!(tune[b], tunes[o + 1:o + n, k], dim)
      o += n
    end
    states[k] = ModelState(unlist(m), tune)
  end
  m.states = states
end

# ---- the mcmc_master! branch (src/model/mcmc.jl:36-59) ----------------------------------------
"""
    run_chains!(m, window, burnin, thin, chains; device=0, seed=...) -> ModelChains or nothing

The GPU path of `mcmc_master!`: `nothing` when neither `lower(m)` (the hand-lowered line /
rats / logistic kinds) nor `lower_ir(m)` (any other DAG, the node IR) takes the model and its
blocks (the caller then runs `pmap2(mcmc_worker!, lsts)` unchanged).  Global chain id of
chains[k] is chains[k] - 1, so a chain's Philox streams (and its draws) do not depend on
how chains are split over calls or GPUs.
"""
function run_chains!(m::Model, window::UnitRange{Int}, burnin::Integer, thin::Integer,
                     chains::AbstractArray{Int}; device::Integer=0, seed::UInt64=UInt64(20261015))
  low = lower(m)
  if low !== nothing
    spec, keep = low
    kind = spec.model
    getvals = () -> engine_values(m, kind)
    setvals! = v -> set_engine_values!(m, kind, v)
    e = create(spec, device)
  else
    irl = lower_ir(m)                                  # the node IR (mmb_create_ir)
    irl === nothing && return nothing
    spec, ir, layout, keep = irl
    kind = MMB_MODEL_IR
    getvals = () -> ir_values(m, layout)
    setvals! = v -> set_ir_values!(m, layout, v)
    e = create_ir(spec, ir, device)
  end
  e === nothing && return nothing
  try
    if kind != MMB_MODEL_IR                            # (the node IR carries its data in the pool)
      for (name, x) in inputs(m, kind); set_data!(e, name, x); end
    end
    states = m.states
    length(states) == length(chains) || throw(ArgumentError("one ModelState per chain expected"))
    init = hcat([(relist!(m, st.value); getvals()) for st in states]...)   # P x K
    offset = first(chains) - 1
    chains == offset + (1:length(chains)) || throw(ArgumentError("chains must be a contiguous range"))
    init_chains!(e, init, offset, seed)
    first(window) > 1 && set_tune!(e, pack_tunes(m, states, first(window) - 1))        # restart
    set_iter!(e, first(window) - 1)
    K = length(chains)
    # draws are sized exactly as mcmc_worker! sizes them (src/model/mcmc.jl:70-71):
    # Chains(last(window), p, start=burnin+thin, thin=thin) has length(burnin+thin:thin:last(window))
    # rows (src/output/chains.jl:5-11), and the keep rule of mcmc.jl:76 fills row
    # (i - burnin) / thin for every kept i of the window.  mmb_run writes n_kept rows.
    nkept = count(i -> i > burnin && (i - burnin) % thin == 0, window)
    pnames = Mamba.names(m, true)
    sim = Chains(last(window), length(pnames), start=burnin + thin, thin=thin, chains=K, names=pnames)
    size(sim.value, 1) == nkept ||
      throw(ArgumentError("window $window, burnin $burnin, thin $thin: $(size(sim.value, 1)) Chains rows " *
                          "but $nkept kept iterations"))
    size(sim.value, 2) == num_monitored(e) || return nothing   # monitor flags the engine does not lower
    a = RunArgs(length(window), burnin, thin, m.burnin, nkept == 0 ? Ptr{Float64}(C_NULL) : pointer(sim.value), 0, 0)
    run!(e, a)                                         # writes n x p x K in Chains order
    store_states!(m, e, setvals!, states)
    m.iter = last(window)
    return ModelChains(sim, m)
  finally
    destroy(e)
    keep = nothing
  end
end

# In src/model/mcmc.jl, first lines of mcmc_master!:
#   if haskey(ENV, "MAMBA_HIP")
#     mc = MambaHIP.run_chains!(m, window, burnin, thin, chains; device=gpu_device())
#     mc === nothing || return mc
#   end

"""
    gelmandiag(engines, p; nranks, rank, id) -> psrf sums (mmb_gr_len doubles)

Cross-GPU sufficient statistics of gelmandiag (gelmandiag.jl:11-25) through the library's own
RCCL communicator; the PSRF follows as in Mamba's gelmandiag (mirror: gelman.py psrf_from_sums).
"""
function gelmandiag_sums(engines::Vector{Ptr{Void}}, p::Integer; nranks::Integer=length(engines),
                         rank0::Integer=0, id::Vector{UInt8}=UInt8[])
  c = comm_init(engines, nranks, rank0, id)
  try
    mm = range_allreduce(c, engines[1], p)
    shift = vec(0.5 * (mm[1, :] + mm[2, :]))
    return gr_allreduce(c, engines[1], zeros(Int32, p), shift)
  finally
    comm_destroy(c)
  end
end

end # module
