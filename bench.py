"""bench.py — chain-updates/sec of the rats hierarchical model (BASELINE.json metric).

Workload (BASELINE.json configs[2], the metric's config): rats growth model
(doc/examples/rats.jl data), mixed Gibbs+AMM sweep (model.rats_scheme_gibbs_amm:
Gibbs s2_c, AMM(alpha, I), Gibbs mu_alpha, Gibbs s2_alpha, AMM(beta, 0.01 I), Gibbs
mu_beta, Gibbs s2_beta; AMM adapt=:all so every update runs the 30x30 pivoted
Cholesky), 16384 chains per GPU (weak scaling; N GPUs = N*16384 chains, configs[4] at
N=8).  A step = one sample!(m) sweep of every chain (one mcmc_worker! iteration) incl.
the keep rule and the Chains write (thin 2, draws kept in HBM).  Steps run as one
mmb_run window (kernels of up to 20 iterations, equal launches); state and data are resident in HBM.

Steady state: before --warmup, an untimed adaptation pre-run (--adapt-prerun, default
128 >= 2d+2 = 62 for the 30-d AMM blocks) takes every chain past AMM's switch to the
mixture proposal (tune.m > 2n, amm.jl:73-75), so every timed update runs the mixture
proposal and a pivoted Cholesky of the moment matrix (amm.jl:72-90).  That factorization does
NOT reach full rank in every chain: setadapt!'s `tune.Mv = v` alias (amm.jl:102) makes the
first adaptive update's Mvv - Mv Mv' = (v0 v0' - v1 v1') / 2, indefinite whenever that first
proposal was accepted (about half the alpha chains, a third of the beta chains), and the running
averages shrink it only like 2/(m+1); dpstf2 stops after a few pivots in those chains every
update and their SigmaLm stays zero (amm.jl:88-90, 104; pinned by tests/test_oracle.py::
test_rats_amm_alias_leaves_first_accepted_chains_without_factor).  The line therefore reports,
per AMM block over the timed window, the full-rank fraction, the mean rank and the mean
factorization steps the device executed (config.amm, from mmb_amm_stats).
The timed window's own kernel time (HIP events on the engine stream) is checked against
its wall time: the run fails if kernel ms per step exceeds ms_per_step by > 5 %.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)

Other BASELINE configs (reported in DESIGN.md, not the metric line):
  --workload line_amm   configs[1]: line regression, AMM, 4096 chains per GPU
  --workload logistic   configs[3]: logistic N=10000 p=50, NUTS, 4096 chains per GPU
                        (roofline bound "mfma": algorithmic 4*N*p flops per gradient)
  --workload seeds_ir   node IR: doc/examples/seeds.jl lowered generically,
                        its own scheme AMM(4) + AMWG(b, 21) + AMWG(s2), 16384 chains per GPU
  --workload rats_ir    node IR: the rats model + the reference Slice/AMWG scheme lowered
                        generically (compare: --workload rats --scheme reference, hand-fused)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CHAINS_PER_GPU = 16384
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
F64_MFMA_PEAK_TFS = 78.6  # MI355X FP64 matrix peak (spec, dense)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r5_rats_gibbs_amm_hbm_traffic.json")
F64_VALU_PEAK_TFS = 78.6  # MI355X FP64 vector peak (spec)
# FP64 VALU lane-flops per chain-update of the reference Slice+AMWG scheme (its binding roofline,
# SURVEY §8(d) row 3'), from the committed rocprofv3 SQ_INSTS_VALU_*_F64 pass
VALU_FILE = os.path.join(ROOT, "profiles", "r5_rats_reference_valu_flops.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--adapt-prerun", type=int, default=None,
                   help="untimed iterations before --warmup (default 128; logistic 0)")
    p.add_argument("--chains", type=int, default=None, help="chains per GPU")
    p.add_argument("--workload", default="rats", choices=["rats", "line_amm", "logistic", "seeds_ir", "rats_ir"])
    p.add_argument("--thin", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=20.0)
    p.add_argument("--nuts-burnin", type=int, default=None,
                   help="logistic: Model.burnin of the timed run (default steps // 2: 1000 of 2000)")
    p.add_argument("--scheme", default="gibbs_amm",
                   help="gibbs_amm (metric config) | reference | ablations: amm_noadapt, gibbs_only")
    p.add_argument("--gradient", default="analytic", choices=["analytic", "forward"],
                   help="logistic: the analytic gradient kernel, or the reference's default dtype=:forward "
                        "(Calculus forward differences: p + 1 log-density columns per gradient)")
    p.add_argument("--amm-fullrank", action="store_true",
                   help="ablation (rats gibbs_amm): AMM moments seeded positive definite, so every "
                        "factorization reaches full rank (no amm.jl:102 alias chains)")
    a = p.parse_args()
    # logistic (configs[3]): the timed steps are the config's whole run, 2000
    # iterations with NUTS adapting for the first 1000 (--nuts-burnin), on re-initialised chains
    dflt = {"rats": (CHAINS_PER_GPU, 400, 200), "line_amm": (4096, 2000, 500), "logistic": (4096, 2000, 20),
            "seeds_ir": (CHAINS_PER_GPU, 160, 80), "rats_ir": (CHAINS_PER_GPU, 64, 32)}
    k, st, wu = dflt[a.workload]
    a.chains = a.chains or k
    a.steps = a.steps if a.steps is not None else st
    a.warmup = a.warmup if a.warmup is not None else wu
    if a.adapt_prerun is None:
        a.adapt_prerun = 0 if a.workload == "logistic" else 128
    return a


def host_cores():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota (on the
    GPU box os.cpu_count() is the whole machine while the job's share is a quota)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, {"nproc": nproc, "affinity": aff, "cgroup_quota": quota}


def _timed_runs(orc, model, st, iters, threads, runs, model_burnin):
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        orc.run(model, st, iters, burnin=0, thin=2, seed=7, nthreads=threads, draws=True,
                model_burnin=model_burnin)
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2], ts


def _oracle_rate(orc, model, init, threads, per_thread, warm, run_s, runs, model_burnin):
    """Median-of-`runs` chain-updates/s of the oracle on `threads` OpenMP threads, timed
    after `warm` untimed iterations (AMM past its m > 2d switch, amm.jl:73-75)."""
    K = min(per_thread * threads, init.shape[0])
    st = orc.new_state(model, init[:K])
    orc.run(model, st, warm, seed=7, nthreads=threads, draws=False, model_burnin=model_burnin)
    iters = 4
    t, _ = _timed_runs(orc, model, st, iters, threads, 1, model_burnin)     # calibration
    iters = int(min(8192, max(4, iters * run_s / max(t, 1e-6))))
    med, ts = _timed_runs(orc, model, st, iters, threads, runs, model_burnin)
    return K * iters / med, K, iters, [round(x, 3) for x in ts]


def cpu_baseline(model, init, seconds, what="rats Gibbs+AMM sweep", per_thread=64, warm=128,
                 model_burnin=None, extra=None):
    """The CPU oracle (same algorithm, same Philox streams; the Julia reference cannot run
    here) on the host cores, SURVEY §8(d): all usable cores and 1 thread, median of 5 runs
    each, bounded to about `seconds` of wall time.  `extra`: (label, model, init) timed
    beside it on all cores (rats: the reference Slice+AMWG scheme)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    orc = oracle_lib.Oracle()
    threads, host = host_cores()
    share = seconds / (10.0 + (3.0 if extra else 0.0))  # 5 all-core + 5 one-thread (+3 extra) runs
    v, K, iters, ts = _oracle_rate(orc, model, init, threads, per_thread, warm, share, 5, model_burnin)
    v1, K1, it1, ts1 = _oracle_rate(orc, model, init, 1, per_thread, warm, share, 5, model_burnin)
    out = {"value": v, "unit": "chain-updates/s", "cores": threads, "kind": "port",
           "sample": f"oracle/oracle.c (CPU restatement; the Julia reference cannot run here): {K} chains x "
                     f"{iters} iterations of the same {what} after {warm} untimed warm-up iterations, "
                     f"OpenMP {threads} threads, median of 5 runs",
           "runs_s": ts, "single_thread": {"value": v1, "chains": K1, "iters": it1, "runs_s": ts1},
           "host": host}
    if extra:
        label, m2, init2 = extra
        v2, K2, it2, ts2 = _oracle_rate(orc, m2, init2, threads, per_thread, warm, share, 3, model_burnin)
        out[label] = {"value": v2, "cores": threads, "chains": K2, "iters": it2, "runs_s": ts2}
    return out


def scheme_for(mb, name):
    """Named rats schemes; "gibbs_amm:beta=0.5,adapt=burnin" overrides AMM keywords."""
    import numpy as np
    G = mb.Gibbs
    if name.startswith("gibbs_amm:"):
        kw = dict(x.split("=") for x in name.split(":", 1)[1].split(","))
        beta = float(kw.get("beta", 0.05))
        adapt = kw.get("adapt", "all")
        sa, sb = float(kw.get("sa", 1.0)), float(kw.get("sb", 0.01))
        return [G("s2_c"), mb.AMM("alpha", sa * np.eye(30), adapt=adapt, beta=beta), G("mu_alpha"),
                G("s2_alpha"), mb.AMM("beta", sb * np.eye(30), adapt=adapt, beta=beta), G("mu_beta"),
                G("s2_beta")]
    if name == "gibbs_amm":
        return mb.model.rats_scheme_gibbs_amm()
    if name == "reference":
        return mb.model.rats_scheme_reference()
    if name == "amm_noadapt":
        return [G("s2_c"), mb.AMM("alpha", np.eye(30), adapt="none"), G("mu_alpha"), G("s2_alpha"),
                mb.AMM("beta", 0.01 * np.eye(30), adapt="none"), G("mu_beta"), G("s2_beta")]
    if name == "gibbs_only":
        return [G("s2_c"), G("mu_alpha"), G("s2_alpha"), G("mu_beta"), G("s2_beta")]
    raise SystemExit(f"unknown scheme {name}")


def rats_model(mb, scheme):
    model = mb.rats()
    model.setinputs(mb.model.RATS_DATA)
    model.setsamplers(scheme)
    return model


def setup_workload(mb, args, rank):
    """Model, scheme, per-chain inits and the run keywords of one BASELINE config."""
    import numpy as np
    K = args.chains
    if args.workload == "rats":
        model = rats_model(mb, scheme_for(mb, args.scheme))
        init = mb.model.rats_init_ls(K, seed=1000 + rank)
        desc = ("rats mixed Gibbs+AMM sweep (BASELINE configs[2]; configs[4] at N=8)"
                if args.scheme == "gibbs_amm" else f"rats scheme {args.scheme}")
        return model, init, desc, {"thin": args.thin}, "f64"
    if args.workload == "line_amm":
        model = mb.line()
        model.setinputs(mb.model.LINE_DATA)
        model.setsamplers([mb.AMM(["beta", "s2"], np.eye(3))])
        init = mb.model.line_init_matrix(K, seed=1000 + rank)
        return model, init, "line AMM (BASELINE configs[1])", {"thin": 1}, "f64"
    if args.workload == "seeds_ir":
        ir = mb.ir
        model = ir.seeds_model().setinputs(ir.SEEDS)
        model.setsamplers([mb.AMM(["alpha0", "alpha1", "alpha2", "alpha12"], 0.01 * np.eye(4)), mb.AMWG("b", 0.01),
                           mb.AMWG("s2", 0.1)])
        rng = np.random.default_rng(1000 + rank)
        inits = [{**ir.seeds_inits()[k % 2], "b": rng.normal(0.0, 0.1, 21)} for k in range(K)]
        return (model, model.init_matrix(inits, K), "seeds (doc/examples/seeds.jl) via the node IR: AMM(4) + "
                "AMWG(b) + AMWG(s2)", {"thin": args.thin}, "f64")
    if args.workload == "rats_ir":
        ir = mb.ir
        model = ir.rats_model().setinputs(ir.rats_inputs()).setsamplers(mb.model.rats_scheme_reference())
        inits = [{**mb.model.RATS_INITS[k % 2], "y": mb.model.RATS_Y} for k in range(K)]
        return (model, model.init_matrix(inits, K), "rats via the node IR, reference Slice+AMWG scheme "
                "(rats.jl:112-116)", {"thin": args.thin}, "f64")
    data, _ = mb.model.logistic_data(10000, 50)
    model = mb.logistic(10000, 50, 10.0)
    model.setinputs(data)
    # gradient: the analytic kernel (dtype=:analytic, asked for explicitly), or the reference's
    # default dtype=:forward -- Calculus forward differences, 51 log-density columns per gradient
    model.setsamplers([mb.NUTS("beta", dtype=args.gradient)])
    init = np.random.default_rng(1000 + rank).normal(0.0, 0.1, (K, 50))
    what = ("analytic gradient (dtype=:analytic)" if args.gradient == "analytic" else
            "the reference's default gradient dtype=:forward (Calculus forward differences, 51 logpdf! "
            "columns per gradient on the MFMA kernel)")
    return (model, init, f"logistic N=10000 p=50 NUTS (BASELINE configs[3]), {what}", {"thin": 1}, "f64")


def amm_window(model, before, after):
    """Per AMM block, the timed window's factorization statistics (mmb_amm_stats differences):
    the fraction of updates whose pivoted Cholesky reached rank n (SigmaLm replaced, amm.jl:88-90),
    the mean rank, the mean factorization steps the device executed per update (the two chains
    of a wavefront step together, so a chain that stops early still costs its partner's steps)
    and the fraction of optimistic passes redone by the checked pass."""
    out = {}
    for b, a in after.items():
        o = before.get(b, {})
        dv = {k: a[k] - o.get(k, 0) for k in a}
        n = dv["updates"]
        if n <= 0:
            continue
        s = model.samplers[b]
        name = ",".join(s.params) if isinstance(s.params, (list, tuple)) else str(s.params)
        d = model.block_dim(s)
        out[name] = {"updates": n, "d": d, "full_rank_frac": dv["full_rank"] / n, "rank_mean": dv["rank_sum"] / n,
                     "pchol_steps_mean": dv["steps_sum"] / n, "pchol_steps_frac": dv["steps_sum"] / (n * d),
                     "redo_frac": dv["redo"] / n}
    return out


def seed_fullrank_moments(mb, model, eng):
    """Ablation: every AMM block's moments start as if from m = 1000 draws with covariance D
    (alpha 6.0, beta 0.05: about the posterior variances), Mv = the current block value, no
    alias (amm.jl:102) and no factor yet.  Sigma = Mvv - Mv Mv' = D stays positive definite under
    the running averages, so every timed factorization runs all n pivots: the intrinsic cost of
    the update, which the headline's alias-stopped chains (about half) do not pay."""
    import numpy as np
    t, v = eng.tune(), eng.values()
    off, T = 0, lambda i: i * (i + 1) // 2  # noqa: E731
    vo = {"alpha": 1, "beta": 33}
    var = {"alpha": 6.0, "beta": 0.05}
    for s in model.samplers:
        d = model.block_dim(s)
        if s.kind == mb.abi.MMB_SAMPLER_AMM:
            name = s.params if isinstance(s.params, str) else s.params[0]
            x = v[:, vo[name]:vo[name] + d]
            r = t[:, off:off + 4 + 2 * d + 2 * T(d)]
            r[:, 0], r[:, 1], r[:, 2], r[:, 3] = 1.0, 1000.0, 0.0, 0.0
            r[:, 4:4 + d] = x
            for i in range(d):
                r[:, 4 + d + T(i):4 + d + T(i) + i + 1] = x[:, i:i + 1] * x[:, :i + 1]
                r[:, 4 + d + T(i) + i] += var[name]
            off += 4 + 2 * d + d * (d + 1)
        elif s.kind == mb.abi.MMB_SAMPLER_AMWG:
            off += 2 + 2 * d
    eng.set_tune(t)


def pmc_traffic(args, W):
    """HBM bytes per sweep launch from the committed rocprofv3 PMC pass of this exact kernel
    build and configuration (profiles/, gathered by tools/profiles_run.sh and corrected by
    tools/profiles_pmc_summary.py as MI355X_MICROARCH.md prescribes; the library's sha256 must
    match); None when no such pass matches."""
    if args.workload != "rats" or not os.path.exists(TRAFFIC_FILE):
        return None, None
    try:
        t = json.load(open(TRAFFIC_FILE))
    except (OSError, ValueError):
        return None, None
    if (t.get("scheme"), t.get("chains"), t.get("iters_per_launch")) != (args.scheme, args.chains, W):
        return None, None
    import hashlib
    import _mamba_path
    lib = _mamba_path.load().abi.LIB_PATH
    if t.get("lib_sha256") != hashlib.sha256(open(lib, "rb").read()).hexdigest():
        return None, None  # counters of another build of the kernel: not this run's traffic
    return t.get("bytes_per_launch"), os.path.relpath(TRAFFIC_FILE, ROOT)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch  # noqa: F401  (pins the HIP runtime; RCCL via torch.distributed)
    import torch.distributed as dist
    # backend "nccl" is RCCL over xGMI; MMB_DIST_BACKEND=gloo rehearses the multi-rank path
    # on a single GPU (ranks share the device, the all-reduces run on host tensors)
    backend = os.environ.get("MMB_DIST_BACKEND", "nccl")
    local = local % max(torch.cuda.device_count(), 1)
    coll_dev = "cuda" if backend == "nccl" else "cpu"
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)
    import _mamba_path
    mb = _mamba_path.load()
    import numpy as np

    K = args.chains
    model, init_all, desc, kw, dtype = setup_workload(mb, args, rank)
    thin = kw["thin"]
    nuts = args.workload == "logistic"
    eng = mb.Engine(model, device=local)
    eng.init_chains(init_all, chain_offset=rank * K, seed=20261015)
    if args.amm_fullrank:
        if args.workload != "rats" or args.scheme != "gibbs_amm":
            raise SystemExit("--amm-fullrank applies to --workload rats --scheme gibbs_amm")
        seed_fullrank_moments(mb, model, eng)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        eng.sync()

    # untimed adaptation pre-run, then warmup: AMM's m > 2d switch has happened in every chain
    # before the timed window; NUTS dual averaging runs while iter <= model_burnin (the warmup),
    # then the step size is fixed (nuts.jl:52)
    pre = args.adapt_prerun
    mburn = pre + args.warmup if nuts else 0
    if pre > 0:
        eng.run(pre, burnin=0, thin=thin, model_burnin=mburn, draws=False, keep_device=False)
    early = os.environ.get("MMB_BENCH_STATS_EARLY") == "1"  # (experiment: no host reads after the warm-up)
    if early and not nuts:
        eng.reserve_draws(args.steps // thin + 1)
        amm_before = eng.amm_stats()
        amwg_before = eng.amwg_stats()["sequential_updates"]
    # warm-up with event timing on (the engine's event pools exist before the timed window),
    # then the device draw buffer for the timed window's kept rows: no allocation in the window
    eng.run(args.warmup, burnin=0, thin=thin, model_burnin=mburn, draws=False, keep_device=False,
            time_kernels=True)
    tburn = pre + args.warmup
    if nuts:
        # the config's own run: fresh chains, NUTS adapting while iter <= nuts_burnin (nuts.jl:52),
        # kept draws after it (mcmc(m, ..., 2000, burnin=1000)); the warm-up above only warmed
        # the kernels and the engine's buffers
        eng.init_chains(init_all, chain_offset=rank * K, seed=20261015)
        mburn = tburn = args.nuts_burnin if args.nuts_burnin is not None else args.steps // 2
    nuts_before = eng.nuts_stats() if nuts else None
    if not (early and not nuts):
        eng.reserve_draws(args.steps // thin + 1)
        amm_before = eng.amm_stats()
        amwg_before = eng.amwg_stats()["sequential_updates"]
    barrier()
    t0 = time.perf_counter()
    eng.run(args.steps, burnin=tburn, thin=thin, model_burnin=mburn, draws=False, keep_device=True,
            time_kernels=True)
    barrier()
    dt = time.perf_counter() - t0
    t_kms, t_launches, t_units = eng.kernel_time()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    total_units = K * world * args.steps
    value = total_units / dt
    ms_per_step = dt / args.steps * 1e3
    kernel_ms_per_step = t_kms / args.steps
    # logistic: the window's chains run as independent parts on their own streams (engine.cpp
    # run_logistic), so the summed gradient-kernel time may exceed the wall time up to that factor
    lg_parts = 1
    if nuts:
        lg_parts = max(1, min(4, int(os.environ.get("MMB_LG_SPLIT", "3"))))
        lg_parts = 1 if K < 32 * lg_parts else lg_parts
    if kernel_ms_per_step > 1.05 * ms_per_step * lg_parts:
        raise SystemExit(f"bench: kernel time per step {kernel_ms_per_step:.4f} ms exceeds the timed "
                         f"window's {ms_per_step:.4f} ms by more than 5 % — timing is inconsistent")
    grads_timed = eng.grad_evals() if nuts else 0  # (the counter restarts with every mmb_run)
    amm_timed = amm_window(model, amm_before, eng.amm_stats())
    # AMWG block updates of the window that fell back to amwg_sub!'s sequential loop (the
    # lane-parallel decision was not certain for some coordinate; samplers.h amwg_lanes)
    amwg_seq = eng.amwg_stats()["sequential_updates"] - amwg_before
    n_amwg = sum(1 for s in model.samplers if getattr(s, "kind", None) == mb.abi.MMB_SAMPLER_AMWG)
    nuts_timed = None
    if nuts:
        after = eng.nuts_stats()
        nuts_timed = {k: after[k] - nuts_before[k] for k in after}

    # Gelman-Rubin over all chains of all GPUs: device partials + the library's own RCCL
    # communicator (mmb_comm_init / mmb_range_allreduce / mmb_gr_allreduce, the C-ABI collective
    # a Julia caller uses); rank 0's unique id travels over the launcher's process group.
    # MMB_DIST_BACKEND=gloo (several ranks sharing one GPU, which RCCL refuses) reduces the same
    # device partials through torch.distributed on the host instead.
    psrf, coll_note = None, None
    if backend == "nccl":
        # RCCL prints a version banner on stdout at communicator init: keep stdout for the one
        # JSON line (the banner goes to stderr)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            uid = [mb.Comm.unique_id() if rank == 0 else None]
            if world > 1:
                dist.broadcast_object_list(uid, src=0)
            comm = mb.Comm([eng], nranks=world, rank0=rank, uid=uid[0])
            psrf, _ = mb.gelmandiag_rccl(comm)
            comm.close()
        except Exception as ex:  # noqa: BLE001 -- the timed throughput above stands either way
            # a failing library communicator (init is collective: every rank sees it) falls back
            # to the same device partials reduced through torch.distributed, and says so
            coll_note = f"library RCCL communicator failed ({type(ex).__name__}: {ex}); partials " \
                        "reduced through torch.distributed instead"
            print(f"bench: {coll_note}", file=sys.stderr)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if backend == "nccl" and world > 1:
        # the fallback decision is collective too: one rank's local failure after the library's
        # agreement step sends every rank to the torch.distributed reduction (no rank left waiting)
        flag = torch.tensor([1.0 if psrf is None else 0.0], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if float(flag.item()) != 0.0 and psrf is not None:
            psrf = None
            coll_note = "library RCCL communicator failed on another rank; partials reduced through " \
                        "torch.distributed instead"
    if psrf is None:
        def ar_sum(x):
            t = torch.tensor(x, dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t)
            return t.cpu().numpy()

        def ar_minmax(lo, hi):
            a = torch.tensor(np.concatenate([-lo, hi]), dtype=torch.float64, device=coll_dev)
            dist.all_reduce(a, op=dist.ReduceOp.MAX)
            a = a.cpu().numpy()
            return -a[:len(lo)], a[len(lo):]

        psrf, _ = mb.gelmandiag_sharded(eng, allreduce_sum=ar_sum if world > 1 else None,
                                        allreduce_minmax=ar_minmax if world > 1 else None)

    # roofline of the dominant kernel; per-launch device time from HIP events on the engine's
    # stream, over full launches in the same steady state as the timed window
    if nuts:  # lg_grad_kernel: 4*N*p algorithmic flops per gradient (X*beta and X'*res)
        # measured over the timed window itself (the config's whole 2000-iteration run): its
        # gradient count and the HIP-event time of its gradient launches
        kms, launches = t_kms, t_launches
        # forward differences: 51 columns of X * beta' (2 N p flops each), no X' res
        per_grad = 4.0 * 10000 * 50 if args.gradient == "analytic" else 2.0 * 10000 * 50 * 51
        flops = per_grad * grads_timed
        achieved = flops / (kms * 1e-3) / 1e12
        # the same flops over the window's wall time (one stream: the gradient launches were 77 %
        # of it, the control kernel 22 %, launch gaps 0.5 %, profiles/r4_logistic_walltime_split.json;
        # with the chains split over streams the parts' kernels overlap, and the per-launch
        # durations include that sharing)
        wall_tfs = flops / dt / 1e12
        roof = {"bound": "mfma", "achieved": achieved, "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": achieved / F64_MFMA_PEAK_TFS, "traffic": None,
                "achieved_wall": wall_tfs, "frac_wall": wall_tfs / F64_MFMA_PEAK_TFS,
                "kernel": "lg_grad_kernel", "algorithmic_flops_per_gradient": per_grad, "streams": lg_parts,
                "avg_launch_ms": kms / launches, "gradients_per_launch": grads_timed / launches,
                "gradients_per_chain_update_timed": grads_timed / (K * args.steps),
                "window": f"timed run: {args.steps} iterations, burnin {tburn}"}
    else:
        W = int(os.environ.get("MMB_ITERS_PER_LAUNCH", "20" if args.workload == "rats" else
                               "16" if args.workload.endswith("_ir") else "256"))
        # the timed window's own launches, HIP events on the engine stream (measured before the
        # collective: a separate window after it started on a GPU clocked down during the RCCL
        # init's idle seconds and read ~10 % slow)
        kms, launches, units = t_kms, t_launches, t_units
        per_update = eng.state_bytes() + 8.0 * eng.pmon / thin  # 2*S_state + S_draw/thin
        bytes_per_launch = per_update * units / launches
        avg_ms = kms / launches
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(args, W)
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "sweep_kernel",
                "algorithmic_bytes_per_chain_update": per_update, "algorithmic_bytes_per_launch": bytes_per_launch,
                "avg_launch_ms": avg_ms, "launches": launches, "chain_updates_per_launch": units / launches}
        if tsrc:
            roof["traffic_source"] = tsrc
        if args.workload == "line_amm" and not os.environ.get("MMB_LINE_GENERIC"):
            # one AMM block: the engine runs the four-lanes-per-chain kernel (csrc/line_amm.hip);
            # latency-bound (256 waves on 1,024 SIMDs), so the HBM fraction is a floor, not a target
            roof["kernel"] = "line_amm_kernel"
        if args.workload == "rats" and args.scheme == "reference" and os.path.exists(VALU_FILE):
            # f1 row: bound by FP64 vector issue, not HBM (SURVEY §8(d) row 3'); HBM kept alongside
            v = json.load(open(VALU_FILE))
            flops = v["f64_lane_flops_per_chain_update"] * units / launches
            tfs = flops / (avg_ms * 1e-3) / 1e12
            hbm = {k: roof[k] for k in ("achieved", "peak", "unit", "frac")}
            roof.update({"bound": "valu", "achieved": tfs, "peak": F64_VALU_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": tfs / F64_VALU_PEAK_TFS, "hbm": hbm,
                         "f64_lane_flops_per_chain_update": v["f64_lane_flops_per_chain_update"],
                         "flops_source": os.path.relpath(VALU_FILE, ROOT)})
    roof["timed_window_kernel_ms_per_step"] = kernel_ms_per_step
    roof["timed_window_launches"] = t_launches

    out = {
        "metric": "chain-updates/sec (iters×chains) on rats model at 1/2/4/8 MI355X",
        "value": value,
        "unit": "chain-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "adapt_prerun": pre,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": ("rats.jl data (real, 30 rats x 5 weeks); synthetic per-chain inits (per-rat LS + jitter)"
                 if args.workload == "rats" else
                 "line.jl data; synthetic inits" if args.workload == "line_amm" else
                 f"{args.workload[:-3]}.jl data and inits (+ N(0, 0.1^2) jitter on seeds b)" if args.workload.endswith("_ir")
                 else
                 "synthetic X ~ N(0,1), y ~ Bernoulli(invlogit(X beta_true)) (SURVEY §8d seeds); inits N(0, 0.1^2)"),
        "config": {"workload": desc, "chains_per_gpu": K, "global_chains": K * world, "thin": thin,
                   "parallelism": f"chain-shard x{world}",
                   "collective": ("rccl (mmb_gr_allreduce)" if backend == "nccl" and coll_note is None else
                                  f"{backend} (torch.distributed)")},
        "roofline": roof,
    }
    if args.workload != "rats":
        out["metric"] = f"chain-updates/sec on {args.workload} (not the headline metric)"
    if nuts:
        out["config"]["gradient"] = args.gradient
    if args.workload == "rats":
        out["config"].update({"iters_per_launch": int(os.environ.get("MMB_ITERS_PER_LAUNCH", "20")),
                              "scheme": args.scheme})
        if args.scheme == "gibbs_amm":
            out["config"]["amm_adapt"] = "all"
        if args.amm_fullrank:
            out["metric"] = "chain-updates/sec, rats Gibbs+AMM full-rank ablation (not the headline)"
            out["config"]["amm_moments"] = "seeded positive definite (--amm-fullrank): every factorization full rank"
    if amm_timed:
        out["config"]["amm"] = amm_timed
    if n_amwg:
        out["config"]["amwg"] = {"block_updates": n_amwg * K * args.steps, "sequential_fallbacks": int(amwg_seq)}
    if args.workload.endswith("_ir"):
        # node IR: the specialised kernel (mmb_create_ir -> hipRTC, csrc/ir_jit.cpp) or the interpreter
        jit, info = eng.ir_jit()
        out["config"]["ir_kernel"] = {"specialised": jit, "info": info}
    if nuts_timed is not None:
        out["nuts"] = nuts_timed
    if psrf is not None:
        out["gelman_rubin_psrf"] = [float(x) for x in psrf[:, 0]]
    if coll_note is not None:
        out["config"]["collective_note"] = coll_note
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.workload == "rats":
            ref = rats_model(mb, scheme_for(mb, "reference"))
            out["cpu_baseline"] = cpu_baseline(model, init_all, args.cpu_seconds,
                                               what=f"rats {args.scheme} sweep",
                                               extra=("reference_scheme", ref, init_all))
        elif args.workload == "line_amm":
            out["cpu_baseline"] = cpu_baseline(model, init_all, args.cpu_seconds, "line AMM update",
                                               per_thread=256)
        elif args.workload.endswith("_ir"):
            out["cpu_baseline"] = cpu_baseline(model, init_all, args.cpu_seconds,
                                               f"{args.workload} node-IR sweep", per_thread=16, warm=16)
        else:
            out["cpu_baseline"] = cpu_baseline(model, init_all, args.cpu_seconds, "logistic NUTS update",
                                               per_thread=4, warm=20, model_burnin=20)
    if rank == 0:
        print(json.dumps(out))
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
