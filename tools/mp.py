"""Concurrency experiment: run as several simultaneous processes on one GPU; each warms up,
waits for the common wall-clock start time argv[3], then times argv[2] sweeps of argv[1]
chains (rats Gibbs+AMM) and prints its own throughput."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import _mamba_path
mb = _mamba_path.load()
K, steps, start_at = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
m = mb.rats(); m.setinputs(mb.model.RATS_DATA); m.setsamplers(mb.model.rats_scheme_gibbs_amm())
e = mb.Engine(m)
e.init_chains(mb.model.rats_init_ls(K, seed=os.getpid() % 1000), seed=7)
e.run(80, burnin=0, thin=2, model_burnin=0, draws=False)
e.sync()
while time.time() < start_at:
    time.sleep(0.001)
t0 = time.perf_counter()
e.run(steps, burnin=80, thin=2, model_burnin=0, draws=False, keep_device=True)
e.sync()
dt = time.perf_counter() - t0
print(f"pid {os.getpid()} chains {K}: {K * steps / dt:.3e} chain-updates/s, dt {dt:.3f}s", flush=True)
