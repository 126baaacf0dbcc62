"""Where the logistic config's wall time goes.

  python tools/lg_walltime.py [--iters 2000] [--out gpurun_out/lg_walltime.json]
  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/lg_walltime.py --trace-only

Runs BASELINE configs[3]'s window (logistic N=10000 p=50, NUTS(:beta, dtype=:analytic),
4096 chains, 2000 iterations with NUTS adapting for the first 1000) twice on fresh chains with
the same seed -- identical work -- once with per-launch HIP events (mmb_run time_kernels) and
once without, and reports the host wall time of each, the gradient count, the HIP-event time of
the gradient launches and the MFMA fraction on kernel time and on wall time.  With a rocprofv3
kernel trace of the same process (--trace-only: one untimed window), tools/lg_trace_split.py
splits the window's span into gradient kernels, control kernels and gaps.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

F64_MFMA_PEAK_TFS = 78.6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--chains", type=int, default=4096)
    ap.add_argument("--out", default=None)
    ap.add_argument("--trace-only", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401
    import _mamba_path
    mb = _mamba_path.load()
    data, _ = mb.model.logistic_data(10000, 50)
    model = mb.logistic(10000, 50, 10.0)
    model.setinputs(data)
    model.setsamplers([mb.NUTS("beta", dtype="analytic")])
    init = np.random.default_rng(1000).normal(0.0, 0.1, (a.chains, 50))
    eng = mb.Engine(model, device=0)
    burn = a.iters // 2
    res = {}
    modes = [False] if a.trace_only else [False, True, False, True]
    for k, timed in enumerate(modes):
        eng.init_chains(init, chain_offset=0, seed=20261015)
        eng.sync()
        t0 = time.perf_counter()
        eng.run(a.iters, burnin=burn, thin=1, model_burnin=burn, draws=False, keep_device=True,
                time_kernels=timed)
        eng.sync()
        wall = time.perf_counter() - t0
        grads = eng.grad_evals()
        kms, launches, _ = eng.kernel_time()
        flops = 4.0 * 10000 * 50 * grads
        r = {"wall_s": wall, "gradients": grads, "grad_steps": launches,
             "frac_wall": flops / wall / 1e12 / F64_MFMA_PEAK_TFS}
        if timed:
            r.update({"grad_kernel_s": kms / 1e3, "frac_kernel": flops / (kms * 1e-3) / 1e12 / F64_MFMA_PEAK_TFS})
        res[f"run{k}_{'events' if timed else 'noevents'}"] = r
    res["config"] = {"chains": a.chains, "iters": a.iters, "burnin": burn, "N": 10000, "p": 50}
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        open(a.out, "w").write(s)


if __name__ == "__main__":
    main()
