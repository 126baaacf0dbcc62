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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=400)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--chains", type=int, default=CHAINS_PER_GPU, help="chains per GPU")
    p.add_argument("--thin", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--scheme", default="gibbs_amm",
                   help="gibbs_amm (metric config) | reference | ablations: amm_noadapt, gibbs_only")
    return p.parse_args()


def cpu_baseline(mb, model, init, seconds):
    """The CPU oracle (same algorithm, same Philox streams) on the host cores: bounded
    sample (a few thousand chain-updates per thread), OpenMP over chains."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    orc = oracle_lib.Oracle()
    threads = min(os.cpu_count() or 1, 16)
    K = 64 * threads
    st = orc.new_state(model, init[:K])
    orc.run(model, st, 64, seed=7, nthreads=threads, draws=False)  # warm (adaptation, rank)
    iters, t = 16, 0.0
    while True:
        t0 = time.perf_counter()
        orc.run(model, st, iters, burnin=0, thin=2, seed=7, nthreads=threads, draws=True)
        t = time.perf_counter() - t0
        if t > seconds / 2 or iters >= 8192:
            break
        iters *= 2
    return {"value": K * iters / t, "unit": "chain-updates/s", "cores": threads, "kind": "port",
            "sample": f"oracle/oracle.c, {K} chains x {iters} iterations (after 64 warm-up) of the same "
                      f"rats Gibbs+AMM sweep, OpenMP {threads} threads, {t:.1f} s"}


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


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch  # noqa: F401  (pins the HIP runtime; RCCL via torch.distributed)
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    import _mamba_path
    mb = _mamba_path.load()

    K = args.chains
    model = mb.rats()
    model.setinputs(mb.model.RATS_DATA)
    model.setsamplers(scheme_for(mb, args.scheme))
    import numpy as np
    init_all = mb.model.rats_init_ls(K, seed=1000 + rank)
    eng = mb.Engine(model, device=local)
    eng.init_chains(init_all, chain_offset=rank * K, seed=20261015)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        eng.sync()

    # warmup: adaptation reaches steady state (AMM m > 2d uses the adaptive factor)
    eng.run(args.warmup, burnin=0, thin=args.thin, model_burnin=0, draws=False, keep_device=False)
    barrier()
    t0 = time.perf_counter()
    eng.run(args.steps, burnin=args.warmup, thin=args.thin, model_burnin=0, draws=False, keep_device=True)
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    total_units = K * world * args.steps
    value = total_units / dt

    # Gelman-Rubin over all chains of all GPUs: device partials + one RCCL all-reduce
    def ar_sum(x):
        if world == 1:
            return x
        t = torch.tensor(x, dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        return t.cpu().numpy()

    def ar_minmax(lo, hi):
        if world == 1:
            return lo, hi
        a = torch.tensor(np.concatenate([-lo, hi]), dtype=torch.float64, device="cuda")
        dist.all_reduce(a, op=dist.ReduceOp.MAX)
        a = a.cpu().numpy()
        return -a[:len(lo)], a[len(lo):]

    psrf, _ = mb.gelmandiag_sharded(eng, allreduce_sum=ar_sum, allreduce_minmax=ar_minmax)

    # roofline: dominant kernel = the fused sweep; per-launch device time from HIP events
    W = int(os.environ.get("MMB_ITERS_PER_LAUNCH", "8"))
    nroof = max(W * 8, 64)
    eng.run(nroof, burnin=0, thin=args.thin, model_burnin=0, draws=False, keep_device=False,
            time_kernels=True)
    kms, launches, units = eng.kernel_time()
    per_update = eng.state_bytes() + 8.0 * 3 / args.thin  # 2*S_state + S_draw/thin
    bytes_per_launch = per_update * units / launches
    avg_ms = kms / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    if os.path.exists(tfile):
        try:
            traffic = json.load(open(tfile)).get("bytes_per_launch")
        except Exception:
            traffic = None

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
        "dtype": "f64",
        "data": "rats.jl data (real, 30 rats x 5 weeks); synthetic per-chain inits (per-rat LS + jitter)",
        "config": {"workload": "rats mixed Gibbs+AMM sweep (BASELINE configs[2]; configs[4] at N=8)"
                   if args.scheme == "gibbs_amm" else f"rats scheme {args.scheme}",
                   "chains_per_gpu": K, "global_chains": K * world, "thin": args.thin,
                   "iters_per_launch": W, "amm_adapt": "all", "parallelism": f"chain-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_chain_update": per_update,
                     "avg_launch_ms": avg_ms, "chain_updates_per_launch": units / launches},
        "gelman_rubin_psrf": [float(x) for x in psrf[:, 0]],
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(mb, model, init_all, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out))
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
