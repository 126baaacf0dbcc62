"""Concurrency experiment: S engines (each its own HIP stream) in one process, K chains
each, launched back to back; whole-process throughput of the rats Gibbs+AMM sweep."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import _mamba_path
mb = _mamba_path.load()
S, K, steps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
m = mb.rats(); m.setinputs(mb.model.RATS_DATA); m.setsamplers(mb.model.rats_scheme_gibbs_amm())
engs = []
for s in range(S):
    e = mb.Engine(m)
    e.init_chains(mb.model.rats_init_ls(K, seed=100 + s), chain_offset=s * K, seed=7)
    engs.append(e)
for e in engs:
    e.run(80, burnin=0, thin=2, model_burnin=0, draws=False)
for e in engs:
    e.sync()
t0 = time.perf_counter()
for e in engs:
    e.run(steps, burnin=80, thin=2, model_burnin=0, draws=False, keep_device=True)
for e in engs:
    e.sync()
dt = time.perf_counter() - t0
print(f"streams {S} chains/stream {K}: {S * K * steps / dt:.3e} chain-updates/s, {dt / steps * 1e3:.4f} ms/step")
