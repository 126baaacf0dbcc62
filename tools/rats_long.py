"""Long rats runs on the GPU at the rats.rst length (10000 iterations, burnin 2500, thin 2;
doc/examples/rats.rst:37-40) to settle the config-3 s2_c question.

  python tools/rats_long.py [--chains K] [--iters N] [--schemes "gibbs_amm;amm_noadapt;reference"]

Per scheme prints pooled means, the median over chains of the chain means, and the
fraction of chains sitting in the near-zero-variance spike of the IG(0.001, 0.001) priors
(final s2_alpha < 1 or s2_beta < 1e-3), which even an exact conjugate Gibbs sampler enters.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--burnin", type=int, default=2500)
    ap.add_argument("--thin", type=int, default=2)
    ap.add_argument("--schemes", default="gibbs_amm;amm_noadapt;reference")
    ap.add_argument("--out", default=None)
    ap.add_argument("--chunks", type=int, default=0,
                    help="then run this many further windows of --iters, all kept: convergence series")
    a = ap.parse_args()
    import torch  # noqa: F401
    import _mamba_path
    mb = _mamba_path.load()
    import bench
    res = {}
    for sch in a.schemes.split(";"):
        m = mb.rats()
        m.setinputs(mb.model.RATS_DATA)
        m.setsamplers(bench.scheme_for(mb, sch))
        init = (mb.model.rats_init_matrix(a.chains) if sch == "reference_const"
                else mb.model.rats_init_ls(a.chains, seed=1))
        eng = mb.Engine(m, device=0)
        eng.init_chains(init, seed=20261016)
        t0 = time.perf_counter()
        eng.run(a.iters, burnin=a.burnin, thin=a.thin, draws=False, keep_device=True)
        eng.sync()
        dt = time.perf_counter() - t0
        d = eng.draws()                                   # n x 3 x K
        v = eng.values()
        cm = d.mean(axis=0)                               # 3 x K chain means
        spike = (v[:, 32] < 1.0) | (v[:, 64] < 1e-3)
        r = {"seconds": dt, "pooled_mean": d.mean(axis=(0, 2)).tolist(),
             "pooled_sd": d.std(axis=(0, 2)).tolist(),
             "median_chain_mean": np.median(cm, axis=1).tolist(),
             "mean_chain_mean_nonspike": cm[:, ~spike].mean(axis=1).tolist(),
             "se_nonspike": (cm[:, ~spike].std(axis=1) / np.sqrt((~spike).sum())).tolist(),
             "spike_frac": float(spike.mean())}
        series = []
        for _ in range(a.chunks):  # later windows of the same chains (mcmc restart, all kept)
            it0 = eng.iter
            eng.run(a.iters, burnin=it0, thin=a.thin, draws=False, keep_device=True)
            d = eng.draws()
            series.append({"window": [it0 + 1, eng.iter], "pooled_mean": d.mean(axis=(0, 2)).tolist(),
                           "se": (d.mean(axis=0).std(axis=1) / np.sqrt(d.shape[2])).tolist()})
            print(sch, json.dumps(series[-1]), flush=True)
        r["series"] = series
        res[sch] = r
        print(sch, json.dumps(r), flush=True)
        eng.close()
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
