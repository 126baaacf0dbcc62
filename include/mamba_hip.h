/*
 * mamba_hip.h — C ABI of the MI355X many-chain MCMC engine (libmambahip.so).
 *
 * Drop-in boundary: this library replaces, for the supported
 * lowered models, everything Mamba.jl runs under `pmap2(mcmc_worker!, lsts)`
 * in `mcmc_master!`:
 *   /root/reference/src/model/mcmc.jl:36-59   mcmc_master!  (chain fan-out)
 *   /root/reference/src/model/mcmc.jl:62-83   mcmc_worker!  (per-chain loop, keep rule)
 *   /root/reference/src/model/simulation.jl:93-107  sample!(m)  (block sweep)
 *   /root/reference/src/samplers/{amwg,amm,nuts,slice}.jl  (block updates)
 *   /root/reference/src/model/simulation.jl:47-90   logpdf! / gradlogpdf!
 * A Julia `ccall` shim binds these symbols from a specialised
 * mcmc_master!; unsupported models/schemes return MMB_E_UNSUPPORTED so the
 * shim can fall back to the Julia path.
 *
 * Conventions: every function returns 0 on success or a negative MMB_E* code
 * (message via mmb_last_error); nothing throws across the ABI.  All real
 * arrays are FP64 (Mamba is Float64-only, src/Mamba.jl:57-58).  Host buffers
 * are caller-owned; device memory is owned by the engine.  An engine is used by
 * one host thread at a time (one engine per GPU; multi-GPU = one process per
 * GPU, each with its own shard of global chain ids).
 */
#ifndef MAMBA_HIP_H
#define MAMBA_HIP_H

#if !defined(__HIPCC_RTC__)
#include <stddef.h>
#include <stdint.h>
#else  /* hipRTC (node-IR specialisation): fixed-width types from its runtime header */
typedef __hip_internal::int8_t int8_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::int16_t int16_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __UINTPTR_TYPE__ uintptr_t;
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define MMB_ABI_VERSION 9
#define MMB_MAX_BLOCKS 8
#define MMB_MAX_NODES_PER_BLOCK 4

/* ---- error codes ---- */
#define MMB_OK 0
#define MMB_E_ARG (-1)         /* invalid argument (ArgumentError in mcmc.jl:22-25, amwg.jl:37-42) */
#define MMB_E_UNSUPPORTED (-2) /* model/scheme not lowered to a kernel: fall back to Julia */
#define MMB_E_HIP (-3)         /* HIP runtime error */
#define MMB_E_STATE (-4)       /* call out of order (e.g. run before init) */
#define MMB_E_NOMEM (-5)
#define MMB_E_COMM (-6)        /* RCCL error in a cross-GPU collective (mmb_comm_*, mmb_gr_allreduce) */
/* Slice shrinkage bound: the reference shrinks until it accepts (slice.jl:78-88,103-113); a
 * kernel must end, so an update still rejecting after this many candidates stops and mmb_run
 * returns MMB_E_STATE (only a degenerate target, e.g. an infinite width, gets there). */
#define MMB_SLICE_MAX_SHRINK 100000

/* ---- lowered model kinds ---- */
typedef enum {
  MMB_MODEL_LINE = 1,    /* doc/tutorial/line.jl:5-25   y ~ IsoNormal(xmat*beta, sqrt(s2)) */
  MMB_MODEL_RATS = 2,    /* doc/examples/rats.jl:48-97  hierarchical growth model */
  MMB_MODEL_LOGISTIC = 3, /* build-defined:  y ~ Bernoulli(invlogit(X*beta)) */
  MMB_MODEL_IR = 4        /* generic node IR: created by mmb_create_ir */
} mmb_model_kind;

/* node ids (Stochastic nodes that can appear in a sampling block) */
enum { MMB_LINE_BETA = 0, MMB_LINE_S2 = 1 };
enum {
  MMB_RATS_S2_C = 0, MMB_RATS_ALPHA = 1, MMB_RATS_MU_ALPHA = 2, MMB_RATS_S2_ALPHA = 3,
  MMB_RATS_BETA = 4, MMB_RATS_MU_BETA = 5, MMB_RATS_S2_BETA = 6
};
enum { MMB_LOGISTIC_BETA = 0 };

/* ---- sampler kinds (src/samplers/{amwg,amm,nuts,slice,hmc,mala}.jl) ---- */
typedef enum {
  MMB_SAMPLER_AMWG = 1,  /* src/samplers/amwg.jl:47-61 */
  MMB_SAMPLER_AMM = 2,   /* src/samplers/amm.jl:45-59    */
  MMB_SAMPLER_NUTS = 3,  /* src/samplers/nuts.jl:47-56 */
  MMB_SAMPLER_SLICE = 4, /* src/samplers/slice.jl:47-58 */
  MMB_SAMPLER_GIBBS = 5, /* user Sampler(params, f): conjugate full conditional of the block's node,
                            e.g. doc/tutorial/line.jl:27-45 */
  MMB_SAMPLER_HMC = 6,   /* src/samplers/hmc.jl:47-65 */
  MMB_SAMPLER_MALA = 7   /* src/samplers/mala.jl:43-58 */
} mmb_sampler_kind;

typedef enum { MMB_ADAPT_ALL = 0, MMB_ADAPT_BURNIN = 1, MMB_ADAPT_NONE = 2 } mmb_adapt;
typedef enum { MMB_SLICE_MULTIVARIATE = 0, MMB_SLICE_UNIVARIATE = 1 } mmb_slice_form;

/* One sampling block = one Sampler in Model.samplers (src/Mamba.jl:119-124). */
/* Gradient of a NUTS / HMC / MALA block.  The reference differentiates logpdf! with Calculus
 * (gradlogpdf!(m, x, block, transform; dtype = :forward), simulation.jl:47-51): forward
 * differences with epsilon = sqrt(eps()) * max(1, |x_i|), non-finite entries -> 0.
 *   MMB_GRAD_DEFAULT  the model's default: forward differences on line and the node IR (the
 *                     reference's), the analytic gradient kernel on logistic (configs[3]) --
 *                     C callers only; the Python mirror and the Julia shim pass FORWARD or
 *                     ANALYTIC explicitly, so the substitution is never implicit
 *   MMB_GRAD_FORWARD  forward differences (line, node IR, logistic: p + 1 log-density columns
 *                     per gradient through the batched MFMA kernel, ABI 9)
 *   MMB_GRAD_ANALYTIC the hand-derived gradient (line, logistic; node IR: MMB_E_ARG) */
typedef enum { MMB_GRAD_DEFAULT = 0, MMB_GRAD_FORWARD = 1, MMB_GRAD_ANALYTIC = 2 } mmb_gradient;

typedef struct {
  int32_t sampler;                         /* mmb_sampler_kind */
  int32_t nnodes;                          /* number of nodes in `params` */
  int32_t nodes[MMB_MAX_NODES_PER_BLOCK];  /* node ids in block (params) order */
  int32_t adapt;                           /* AMWG/AMM: mmb_adapt (default :all) */
  int32_t form;                            /* Slice: mmb_slice_form (default Multivariate) */
  int32_t transform;                       /* Slice: transform flag (default false); AMWG/AMM/NUTS use true */
  int32_t batchsize;                       /* AMWG batchsize (default 50) */
  double target;                           /* AMWG target (0.44) / NUTS target (0.6) */
  double beta;                             /* AMM beta (0.05) */
  double scale;                            /* AMM scale (2.38) */
  int32_t dim;                             /* unlisted block length (checked by mmb_create) */
  int32_t ntuning;                         /* length of `tuning` */
  const double* tuning;                    /* AMWG sigma[dim] | Slice width[dim] | AMM Sigma[dim*dim] col-major
                                              | HMC/MALA Sigma[dim*dim] col-major, or none (SigmaL = I) */
  double epsilon;                          /* HMC/MALA step size (hmc.jl:13, mala.jl:12) */
  int32_t nsteps;                          /* HMC leapfrog steps L (hmc.jl:13) */
  int32_t gradient;                        /* NUTS/HMC/MALA logpdfgrad! (sampler.jl:97-111): mmb_gradient */
} mmb_block_spec;

typedef struct {
  int32_t model;                           /* mmb_model_kind */
  int32_t nblocks;
  mmb_block_spec blocks[MMB_MAX_BLOCKS];   /* Model.samplers, in sweep order */
  int32_t nobs;                            /* logistic: N (rows of X) */
  int32_t ncoef;                           /* logistic: p (columns of X) */
  double prior_sd;                         /* logistic: beta ~ MvNormal(p, prior_sd) */
  int32_t reserved[8];
} mmb_model_spec;

/* ---- generic node IR (ABI version 3) ----------------------------------
 * A Mamba Model DAG (src/model/model.jl:5-27, src/model/dependent.jl:75-152) lowered by the
 * host (mamba.jl_amd/ir.py; a Julia shim would walk m.nodes the same way):
 *   - Logical nodes are inlined into the expressions of their Stochastic children;
 *   - Stochastic nodes that no sampling block updates are fixed: values in the data pool;
 *   - the sampled ones own slots [off, off+len) of the chain state (P = nvalues);
 *   - each node's distribution parameters are stack-code expressions evaluated per element i
 *     of the node (elementwise broadcast, src/distributions/distributionstruct.jl:142-158).
 * Block ids in mmb_block_spec.nodes index `nodes`. */
typedef enum {
  MMB_IR_NORMAL = 1,      /* Normal(mu, sigma)                          RealDistribution      */
  MMB_IR_ISONORMAL = 2,   /* MvNormal(mu[], sigma) (PDMats ScalMat)     node-level density    */
  MMB_IR_INVGAMMA = 3,    /* InverseGamma(shape, scale)                 PositiveDistribution  */
  MMB_IR_GAMMA = 4,       /* Gamma(shape, scale)                        PositiveDistribution  */
  MMB_IR_EXPONENTIAL = 5, /* Exponential(scale)                         PositiveDistribution  */
  MMB_IR_UNIFORM = 6,     /* Uniform(a, b), constant bounds lo/hi       bounded (affine logit) */
  MMB_IR_BETA = 7,        /* Beta(a, b)                                 UnitDistribution      */
  MMB_IR_BINOMIAL = 8,    /* Binomial(n, p)     fixed (observed) nodes only */
  MMB_IR_POISSON = 9,     /* Poisson(lambda)    fixed (observed) nodes only */
  MMB_IR_BERNOULLI = 10,  /* Bernoulli(p)       fixed (observed) nodes only */
  MMB_IR_LOGICAL = 11     /* Logical: expr[0] is the value (monitored logicals) */
} mmb_ir_family;

/* expression code: one int32 word per op, op << 24 | arg; a push spills the previous top */
enum {
  MMB_IR_OP_END = 0,
  MMB_IR_OP_CONST = 1,  /* push consts[arg] */
  MMB_IR_OP_VAL = 2,    /* push state[arg] */
  MMB_IR_OP_VALI = 3,   /* push state[arg + i] */
  MMB_IR_OP_VALG = 4,   /* push state[arg + (int)pool[w + i]], w = the next code word */
  MMB_IR_OP_DATA = 5,   /* push pool[arg + i] */
  MMB_IR_OP_DATAS = 6,  /* push pool[arg] */
  MMB_IR_OP_ADD = 16, MMB_IR_OP_SUB = 17, MMB_IR_OP_MUL = 18, MMB_IR_OP_DIV = 19,
  MMB_IR_OP_NEG = 32, MMB_IR_OP_EXP = 33, MMB_IR_OP_LOG = 34, MMB_IR_OP_SQRT = 35,
  MMB_IR_OP_INVLOGIT = 36, MMB_IR_OP_LOGIT = 37, MMB_IR_OP_ABS = 38
};
#define MMB_IR_MAX_STACK 16
#define MMB_IR_MAX_TERMS 16
#define MMB_IR_MAX_VALUES 512

typedef struct {
  int32_t family;    /* mmb_ir_family */
  int32_t fixed;     /* 1: values in the pool at `off` (not sampled) */
  int32_t off, len;  /* state slots (or pool offset) */
  int32_t expr[3];   /* code offsets of the distribution parameters (Distributions order), -1 none */
  int32_t cterm;     /* pool offset of a per-element constant (log binomial coefficient,
                        -lgamma(k+1)) or -1 */
  double lo, hi;     /* Uniform bounds */
} mmb_ir_node;

/* logpdf!(m, x, block, transform) terms (simulation.jl:77-90): params \ targets in block
 * order, then targets in topological order; trans = node is a block param (evaluated with
 * the block's transform) */
typedef struct {
  int32_t nterms;
  int32_t term[MMB_IR_MAX_TERMS];
  int32_t trans[MMB_IR_MAX_TERMS];
} mmb_ir_block;

typedef struct {
  int32_t nvalues;              /* P */
  int32_t nnodes;
  const mmb_ir_node* nodes;
  int32_t ncode;
  const int32_t* code;
  int32_t nconst;
  const double* consts;
  int64_t npool;
  const double* pool;           /* data, fixed node values, gather indices (0-based), cterms */
  int32_t nmon;
  const int32_t* mon;           /* monitored node ids in Chains order, each contributing len values */
  int32_t stack;                /* max expression stack depth (<= MMB_IR_MAX_STACK) */
  mmb_ir_block blocks[MMB_MAX_BLOCKS];  /* one per sampling block of the spec */
} mmb_ir_model;

/* Arguments of one mcmc window (mcmc.jl:36-83). */
typedef struct {
  int64_t iters;        /* window = iter+1 : iter+iters  (mcmc_master! `window`) */
  int64_t burnin;       /* keep iteration i iff i > burnin && (i-burnin) % thin == 0 (mcmc.jl:76) */
  int64_t thin;
  int64_t model_burnin; /* Model.burnin: gate for adapt=:burnin (amwg.jl:55) and NUTS (nuts.jl:52) */
  double* draws;        /* host out, Mamba Chains order n_kept x p_mon x K (iteration fastest) or NULL */
  int32_t keep_device;  /* nonzero: keep this window's draws on the device (mmb_get_draws / GR) */
  int32_t time_kernels; /* nonzero: bracket each kernel launch with HIP events (mmb_kernel_time) */
} mmb_run_args;

typedef struct mmb_engine mmb_engine;

/* Engine lifetime ---------------------------------------------------------------- */
int mmb_abi_version(void);
int mmb_create(const mmb_model_spec* spec, int device, mmb_engine** out);
/* Node-IR model (spec->model == MMB_MODEL_IR): the IR is copied and validated (every code
 * word, slot and pool range against the node lengths) before anything touches the device.
 * Replaces the same fan-out as mmb_create for any Model lowered to the IR. */
int mmb_create_ir(const mmb_model_spec* spec, const mmb_ir_model* ir, int device, mmb_engine** out);
void mmb_destroy(mmb_engine* e);
const char* mmb_last_error(const mmb_engine* e); /* e may be NULL: last global error */

/* setinputs! (initialization.jl:30-40): named data arrays.
 * line: "x"(5), "y"(5); rats: "y"(150, rat-major), "x"(5); logistic: "X"(N*p row-major), "y"(N) */
int mmb_set_data(mmb_engine* e, const char* name, const double* x, int64_t n);

/* setinits! (initialization.jl:20-28): K chains, `init` is K x P row-major (chain-major),
 * P = mmb_num_values(); global chain ids are chain_offset .. chain_offset+K-1 (they key the
 * Philox streams, so a chain's trajectory does not depend on how chains are sharded). */
int mmb_num_values(const mmb_engine* e);
int mmb_num_monitored(const mmb_engine* e);
int mmb_init_chains(mmb_engine* e, const double* init, int64_t K, int64_t chain_offset, uint64_t seed);

/* mcmc_worker! loop for all chains of this engine (mcmc.jl:62-83). */
int mmb_run(mmb_engine* e, const mmb_run_args* args);
int64_t mmb_iter(const mmb_engine* e);              /* Model.iter after the last window */
/* Restore Model.iter when resuming from a checkpoint (read(name, ModelChains) followed by
 * mcmc(mc, iters), fileio.jl:3-11 + mcmc.jl:3-16).  Philox streams are keyed by
 * (seed, global chain id, iteration), so values + tune + iter + seed reproduce the
 * uninterrupted trajectory exactly.  Call after mmb_init_chains; iter >= 0. */
int mmb_set_iter(mmb_engine* e, int64_t iter);

/* ModelState / gettune / settune! (mcmc.jl:56,82; simulation.jl:3-28):
 * values: K x P row-major.  tune: K x mmb_tune_len() doubles in the canonical layout
 * (DESIGN.md §tune layout; ints stored exactly as doubles). */
int mmb_get_values(mmb_engine* e, double* values);
int mmb_set_values(mmb_engine* e, const double* values);
int64_t mmb_tune_len(const mmb_engine* e);
int mmb_get_tune(mmb_engine* e, double* tune);
int mmb_set_tune(mmb_engine* e, const double* tune);

/* Draws of the last window kept on device (keep_device=1), host copy in Mamba order. */
int64_t mmb_num_kept(const mmb_engine* e);
int mmb_get_draws(mmb_engine* e, double* draws);
/* Allocate the device draw buffer for windows keeping up to nkept iterations now, so a
 * later mmb_run does not allocate inside a timed or latency-sensitive window (mmb_run grows
 * the buffer itself when a window needs more).  nkept >= 0. */
int mmb_reserve_draws(mmb_engine* e, int64_t nkept);

/* Gelman-Rubin sufficient statistics of the device-kept draws (gelmandiag.jl:3-60).
 * mmb_gr_range: per monitored param [min, max] over local chains/draws (for link()).
 * mmb_gr_partials: per-chain mean/covariance reduced over local chains, after optional
 * log/logit link (link_kind per param: 0 none, 1 log, 2 logit) and shift `shift[p]`;
 * out has mmb_gr_len() doubles: these are summed across GPUs (RCCL all-reduce). */
int mmb_gr_range(mmb_engine* e, double* minmax /* 2*p */);
int64_t mmb_gr_len(const mmb_engine* e);
int mmb_gr_partials(mmb_engine* e, const int32_t* link_kind, const double* shift, double* out);

/* The one cross-GPU exchange (gelmandiag.jl:11-25), over RCCL/xGMI, inside the
 * library so a ccall caller reaches it (SURVEY §8b mmb_gr_allreduce).  Chains never interact
 * while sampling (mcmc.jl:48-52), so this is the only collective.
 * A communicator spans the engines (one per GPU) of every participating process:
 *   one process driving all GPUs (Julia threads / async streams):
 *       mmb_comm_init(engines, ngpu, ngpu, 0, NULL, &c)          -> ncclCommInitAll
 *   one process per GPU (torchrun-style, or Julia workers):
 *       rank 0: mmb_comm_id(id); the caller broadcasts the MMB_COMM_ID_BYTES bytes;
 *       every process: mmb_comm_init(&e, 1, nranks, rank, id, &c) -> ncclCommInitRank
 *   (nlocal engines of one process take ranks rank0 .. rank0+nlocal-1 of nranks).
 * mmb_range_allreduce: global [min, max] per monitored param (one MAX all-reduce of
 *   (-min, max)), for link() (chains.jl:237-246) and the shift.
 * mmb_gr_allreduce: mmb_gr_partials of every local engine (same link/shift on every rank),
 *   summed over all ranks by one SUM all-reduce of mmb_gr_len doubles; out = global sums,
 *   from which the host evaluates the PSRF as gelmandiag.jl:26-60 (mamba.jl_amd/gelman.py
 *   psrf_from_sums).  Every rank must call each collective (RCCL semantics).
 * Errors are reported through mmb_last_error(engines[0]). */
#define MMB_COMM_ID_BYTES 128
typedef struct mmb_comm mmb_comm;
int mmb_comm_id(uint8_t* id /* MMB_COMM_ID_BYTES */);
int mmb_comm_init(mmb_engine** engines, int nlocal, int nranks, int rank0, const uint8_t* id, mmb_comm** out);
int mmb_range_allreduce(mmb_comm* c, double* minmax /* 2*p: [min, max] per param */);
int mmb_gr_allreduce(mmb_comm* c, const int32_t* link_kind, const double* shift, double* out);
void mmb_comm_destroy(mmb_comm* c);

/* Posterior summaries of the device-kept draws, pooled over chains.
 * mmb_chain_summary replaces the per-element work of summarystats(c; etype=:bm)
 * (/root/reference/src/output/stats.jl:85-94) and mcse_bm (src/output/mcse.jl:10-19):
 * per local chain k and monitored param j, out[(k*p + j)*MMB_SUMMARY_FIELDS + f] =
 *   [sum x', sum x'^2, sum d_b, sum d_b^2, #full batches, head sum, head count,
 *    tail sum, tail count, 0]    with x' = x - shift[j],
 * where batches are runs of `batch_size` consecutive elements of vec(x) (chains
 * concatenated; local chain k sits at position chain_base + k: the global chain id for a
 * pooled multi-GPU summary, k for this engine alone), d_b = batch mean - shift[j] for the batches lying
 * wholly in the chain, and head/tail are the chain's pieces of batches shared with the
 * previous/next chain (joined by the host, across GPUs too).
 * mmb_order_hist: one radix-select pass for quantile(c) (stats.jl:73-80): for each of
 * `ntargets` key prefixes (order-preserving uint64 key of the double, bits above digit
 * 56-8*pass), counts[t*256 + d] = #draws of `param` whose key matches prefix t and whose
 * digit is d. */
#define MMB_SUMMARY_FIELDS 10
#define MMB_ORDER_MAX_TARGETS 16
int mmb_chain_summary(mmb_engine* e, const double* shift /* p */, int64_t batch_size, int64_t chain_base,
                      double* out /* K x p x MMB_SUMMARY_FIELDS */);
int mmb_order_hist(mmb_engine* e, int param, int ntargets, const uint64_t* prefix, int pass,
                   uint64_t* counts /* ntargets x 256 */);

/* Timing / sync (bench.py roofline) */
int mmb_sync(mmb_engine* e);
int mmb_kernel_time(const mmb_engine* e, double* total_ms, int64_t* launches, int64_t* units);
int mmb_state_bytes(const mmb_engine* e, double* bytes_per_chain_update);
/* Gradient evaluations (logpdf!+gradlogpdf! calls, sampler.jl:97-119) in the last mmb_run,
 * summed over chains; counted on device by the batched-gradient (logistic) engine, 0 else. */
int mmb_grad_evals(mmb_engine* e, int64_t* n);
/* NUTS tree statistics since mmb_init_chains, all NUTS blocks and chains: out[0] = completed
 * updates, out[1] = updates stopped by the depth cap MMB_NUTS_MAX_DEPTH (30: 2^30 leapfrogs
 * in one update, beyond any run that finishes) while the
 * reference's unbounded doubling loop (nuts.jl:106-125) would have continued, out[2] = sum of
 * final tree depths j.  out[1] == 0 means the cap never changed a draw. */
int mmb_nuts_stats(mmb_engine* e, int64_t out[3]);
/* Node-IR kernel specialisation.  mmb_create_ir writes the lowered model as
 * HIP source -- node log densities (dependent.jl:207-213 -> distributionstruct.jl:136-168) and
 * block logpdf! term lists (simulation.jl:77-90) as straight-line code -- and compiles it with
 * hipRTC (code objects cached by source hash: MMB_JIT_CACHE, else <library dir>/jit), replacing
 * the per-op interpreter; the same operations in the same order, so results are bit-identical.
 * On any failure, or with MMB_IR_JIT=0, the interpreter kernel runs.
 * mmb_ir_jit_info: 1 if the engine runs the specialised kernel, 0 if the interpreter; `buf`
 * receives the reason / cache status.  mmb_ir_jit_prebuild: validate and compile into the cache
 * without a device (build step).  mmb_ir_jit_source_text: the generated source (returns its
 * length; copies up to n - 1 bytes). */
int mmb_ir_jit_info(const mmb_engine* e, char* buf, int64_t n);
int mmb_ir_jit_prebuild(const mmb_model_spec* spec, const mmb_ir_model* ir, char* info, int64_t n);
int mmb_ir_jit_source_text(const mmb_model_spec* spec, const mmb_ir_model* ir, char* buf, int64_t n);
/* AMM factorization statistics since mmb_init_chains, per sampling block b (zero rows for
 * non-AMM blocks), summed over the engine's chains: out[b*MMB_AMM_STATS + i] =
 *   i = 0  adaptive updates, i.e. cholfact(Hermitian(Sigma), Val{true}) calls (amm.jl:81-87)
 *   i = 1  of them with rank(F) == n, i.e. SigmaLm replaced (amm.jl:88-90)
 *   i = 2  sum of rank(F) (dpstf2's pivots taken before its ajj <= 0 stop)
 *   i = 3  sum of factorization steps the device executed for the update's chain group:
 *          min(rank + 1, n) per chain, the max over the two chains of a wavefront on the
 *          32-lane kernels (both chains step together), the chain's own count elsewhere
 *   i = 4  updates whose optimistic factorization pass was redone by the checked pass
 * Diagnostics only (the bench reports the full-rank fraction and mean steps of its timed
 * window); no draw depends on them. */
#define MMB_AMM_STATS 5
int mmb_amm_stats(mmb_engine* e, int64_t* out /* MMB_MAX_BLOCKS x MMB_AMM_STATS */);

/* AMWG path counter since init_chains: out[0] = block updates that ran amwg_sub! one coordinate
 * at a time (samplers.h amwg) instead of the lane-parallel decision of every coordinate, which
 * is taken when each coordinate's accept test is certain under the logpdf's rounding bound
 * (rats alpha / beta; the environment variable MMB_AMWG_EXACT=1 forces the sequential loop,
 * MMB_SLICE_EXACT=1 the one-candidate-at-a-time Slice shrink loop of the rats scalar blocks).
 * Both paths give the same draws; diagnostics only. */
int mmb_amwg_stats(mmb_engine* e, int64_t* out /* 1 */);

/* The lane-group slot -> chain table the next window will run with (K entries; the identity
 * when no ordering applies).  The 32-lane sweep kernels (rats, node IR) pair chains whose
 * pivoted Cholesky stops alike in one wavefront; the table sorts the chains by their AMM blocks'
 * factor-valid flags (slow classes first; MMB_ORDER_MODE 0 ascending, 2 balanced workgroups),
 * computed on the device right after each window (and before one that follows a host write of
 * the tune state).  Results do not depend on it (every chain keeps its own state, draws column
 * and Philox id); diagnostics. */
int mmb_chain_order(mmb_engine* e, int32_t* slot_to_chain);

/* Diagnostics: the device's 32-lane pivoted Cholesky of the AMM update (cholfact(Hermitian(S),
 * :U, Val{true}) = LAPACK dpstf2 for n < 64, amm.jl:87) on n caller-supplied d x d matrices,
 * 1 <= d <= 30, packed lower triangle S[c][tri(i) + k] (i >= k, 480 doubles per matrix).  Out per
 * matrix: info[c] = {rank, redone} (redone: the optimistic pass was redone by the checked
 * one), pos[c][32] each element's pivot position (-1 past d) and, on full rank, L[c][480] the
 * factor in position form: element e's row at tri(pos[e]) + k, k = 0..pos[e].  Runs on `device`
 * outside any engine. */
int mmb_debug_pchol(int device, int64_t n, int d, const double* S, double* L, int32_t* pos, int32_t* info);

#ifdef __cplusplus
}
#endif
#endif /* MAMBA_HIP_H */
