"""bench.py — chain-updates/sec of the rats hierarchical model (BASELINE.json metric).

Workload (BASELINE.json configs[2], the metric's config): rats growth model
(doc/examples/rats.jl data), mixed Gibbs+AMM sweep (model.rats_scheme_gibbs_amm:
Gibbs s2_c, AMM(alpha, I), Gibbs mu_alpha, Gibbs s2_alpha, AMM(beta, 0.01 I), Gibbs
mu_beta, Gibbs s2_beta; AMM adapt=:all so every update runs the 30x30 pivoted
Cholesky), 16384 chains per GPU (weak scaling; N GPUs = N*16384 chains, configs[4] at
N=8).  A step = one sample!(m) sweep of every chain (one mcmc_worker! iteration) incl.
the keep rule and the Chains write (thin 2, draws kept in HBM).  Steps run as one
mmb_run window (kernels of 8 iterations); state and data are resident in HBM.

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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--chains", type=int, default=None, help="chains per GPU")
    p.add_argument("--workload", default="rats", choices=["rats", "line_amm", "logistic", "seeds_ir", "rats_ir"])
    p.add_argument("--thin", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--scheme", default="gibbs_amm",
                   help="gibbs_amm (metric config) | reference | ablations: amm_noadapt, gibbs_only")
    a = p.parse_args()
    dflt = {"rats": (CHAINS_PER_GPU, 400, 200), "line_amm": (4096, 2000, 500), "logistic": (4096, 100, 100),
            "seeds_ir": (CHAINS_PER_GPU, 160, 80), "rats_ir": (CHAINS_PER_GPU, 64, 32)}
    k, st, wu = dflt[a.workload]
    a.chains = a.chains or k
    a.steps = a.steps if a.steps is not None else st
    a.warmup = a.warmup if a.warmup is not None else wu
    return a


def cpu_baseline(mb, model, init, seconds, what="rats Gibbs+AMM sweep", per_thread=64, warm=64,
                 model_burnin=None):
    """The CPU oracle (same algorithm, same Philox streams) on the host cores: bounded
    sample (a few thousand chain-updates per thread), OpenMP over chains."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    orc = oracle_lib.Oracle()
    threads = min(os.cpu_count() or 1, 16)
    K = min(per_thread * threads, init.shape[0])
    st = orc.new_state(model, init[:K])
    orc.run(model, st, warm, seed=7, nthreads=threads, draws=False, model_burnin=model_burnin)  # warm-up
    iters, t = 16, 0.0
    while True:
        t0 = time.perf_counter()
        orc.run(model, st, iters, burnin=0, thin=2, seed=7, nthreads=threads, draws=True,
                model_burnin=model_burnin)
        t = time.perf_counter() - t0
        if t > seconds / 2 or iters >= 8192:
            break
        iters *= 2
    return {"value": K * iters / t, "unit": "chain-updates/s", "cores": threads, "kind": "port",
            "sample": f"oracle/oracle.c, {K} chains x {iters} iterations (after {warm} warm-up) of the same "
                      f"{what}, OpenMP {threads} threads, {t:.1f} s"}


def scheme_for(mb, name):
    import numpy as np
    G = mb.Gibbs
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


def setup_workload(mb, args, rank):
    """Model, scheme, per-chain inits and the run keywords of one BASELINE config."""
    import numpy as np
    K = args.chains
    if args.workload == "rats":
        model = mb.rats()
        model.setinputs(mb.model.RATS_DATA)
        model.setsamplers(scheme_for(mb, args.scheme))
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
    model.setsamplers([mb.NUTS("beta")])
    init = np.random.default_rng(1000 + rank).normal(0.0, 0.1, (K, 50))
    return model, init, "logistic N=10000 p=50 NUTS (BASELINE configs[3])", {"thin": 1}, "f64"


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

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        eng.sync()

    # warmup: adaptation reaches steady state (AMM m > 2d uses the adaptive factor; NUTS
    # dual averaging runs while iter <= model_burnin = warmup, then the step size is fixed)
    mburn = args.warmup if nuts else 0
    eng.run(args.warmup, burnin=0, thin=thin, model_burnin=mburn, draws=False, keep_device=False)
    barrier()
    t0 = time.perf_counter()
    eng.run(args.steps, burnin=args.warmup, thin=thin, model_burnin=mburn, draws=False, keep_device=True)
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    total_units = K * world * args.steps
    value = total_units / dt
    grads_timed = eng.grad_evals() if nuts else 0

    psrf = None
    # Gelman-Rubin over all chains of all GPUs: device partials + one RCCL all-reduce
    def ar_sum(x):
        if world == 1:
            return x
        t = torch.tensor(x, dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t)
        return t.cpu().numpy()

    def ar_minmax(lo, hi):
        if world == 1:
            return lo, hi
        a = torch.tensor(np.concatenate([-lo, hi]), dtype=torch.float64, device=coll_dev)
        dist.all_reduce(a, op=dist.ReduceOp.MAX)
        a = a.cpu().numpy()
        return -a[:len(lo)], a[len(lo):]

    psrf, _ = mb.gelmandiag_sharded(eng, allreduce_sum=ar_sum, allreduce_minmax=ar_minmax)

    # roofline of the dominant kernel; per-launch device time from HIP events on the engine's stream
    if nuts:  # lg_grad_kernel: 4*N*p algorithmic flops per gradient (X*beta and X'*res)
        nroof = 16
        eng.run(nroof, burnin=0, thin=1, model_burnin=mburn, draws=False, time_kernels=True)
        kms, launches, units = eng.kernel_time()
        flops = 4.0 * 10000 * 50 * eng.grad_evals()
        achieved = flops / (kms * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": achieved, "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": achieved / F64_MFMA_PEAK_TFS, "traffic": None,
                "kernel": "lg_grad_kernel", "algorithmic_flops_per_gradient": 4.0 * 10000 * 50,
                "avg_launch_ms": kms / launches, "gradients_per_launch": eng.grad_evals() / launches,
                "gradients_per_chain_update_timed": grads_timed / (K * args.steps)}
    else:
        W = int(os.environ.get("MMB_ITERS_PER_LAUNCH",
                               "8" if args.workload == "rats" else "16" if args.workload.endswith("_ir") else "64"))
        nroof = max(W * 8, 64)
        eng.run(nroof, burnin=0, thin=thin, model_burnin=0, draws=False, keep_device=False, time_kernels=True)
        kms, launches, units = eng.kernel_time()
        per_update = eng.state_bytes() + 8.0 * eng.pmon / thin  # 2*S_state + S_draw/thin
        bytes_per_launch = per_update * units / launches
        avg_ms = kms / launches
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        traffic = None
        tfile = os.path.join(ROOT, "profiles", "hbm_traffic.json")
        if args.workload == "rats" and args.scheme == "gibbs_amm" and os.path.exists(tfile):
            try:
                traffic = json.load(open(tfile)).get("bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "sweep_kernel",
                "algorithmic_bytes_per_chain_update": per_update,
                "avg_launch_ms": avg_ms, "chain_updates_per_launch": units / launches}

    out = {
        "metric": "chain-updates/sec (iters×chains) on rats model at 1/2/4/8 MI355X",
        "value": value,
        "unit": "chain-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
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
                   "parallelism": f"chain-shard x{world}", "collective": "rccl" if backend == "nccl" else backend},
        "roofline": roof,
    }
    if args.workload != "rats":
        out["metric"] = f"chain-updates/sec on {args.workload} (not the headline metric)"
    if args.workload == "rats":
        out["config"].update({"iters_per_launch": int(os.environ.get("MMB_ITERS_PER_LAUNCH", "8")),
                              "amm_adapt": "all"})
    if psrf is not None:
        out["gelman_rubin_psrf"] = [float(x) for x in psrf[:, 0]]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.workload == "rats":
            out["cpu_baseline"] = cpu_baseline(mb, model, init_all, args.cpu_seconds)
        elif args.workload == "line_amm":
            out["cpu_baseline"] = cpu_baseline(mb, model, init_all, args.cpu_seconds, "line AMM update",
                                               per_thread=256, warm=64)
        elif args.workload.endswith("_ir"):
            out["cpu_baseline"] = cpu_baseline(mb, model, init_all, args.cpu_seconds,
                                               f"{args.workload} node-IR sweep", per_thread=16, warm=16)
        else:
            out["cpu_baseline"] = cpu_baseline(mb, model, init_all, args.cpu_seconds, "logistic NUTS update",
                                               per_thread=4, warm=20, model_burnin=20)
    if rank == 0:
        print(json.dumps(out))
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
