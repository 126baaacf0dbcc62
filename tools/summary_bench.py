"""Timing of the on-device posterior summaries at the bench size (rats, 16384 chains).

  python tools/summary_bench.py [--iters 2000]

Prints one JSON line: draws bytes streamed per summary pass, wall time of
summarystats (2 streaming passes + host pooling) and of quantile (8 radix passes per
param).  Run under `rocprofv3 --kernel-trace --stats` for per-kernel durations.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=2000)
ap.add_argument("--chains", type=int, default=16384)
a = ap.parse_args()

import torch  # noqa: F401,E402
import _mamba_path  # noqa: E402

mb = _mamba_path.load()
m = mb.rats()
m.setinputs(mb.model.RATS_DATA)
m.setsamplers(mb.model.rats_scheme_gibbs_amm())
eng = mb.Engine(m)
eng.init_chains(mb.model.rats_init_ls(a.chains, seed=1), seed=2)
eng.run(a.iters, burnin=0, thin=1, draws=False, keep_device=True)
eng.sync()
n = eng.num_kept()
nbytes = n * eng.pmon * a.chains * 8
ss = mb.summarystats_sharded(eng)          # warm
t0 = time.perf_counter()
for _ in range(5):
    ss = mb.summarystats_sharded(eng)
t_ss = (time.perf_counter() - t0) / 5
t0 = time.perf_counter()
qs = mb.quantile_sharded(eng)
t_q = time.perf_counter() - t0
print(json.dumps({"draws_bytes": nbytes, "kept": n, "chains": a.chains,
                  "summarystats_s": t_ss, "quantile_s": t_q,
                  "summarystats": ss.tolist(), "quantile": qs.tolist()}))
