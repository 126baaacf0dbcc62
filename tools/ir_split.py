"""Where the node IR's rats reference scheme spends its time: the sweep with every block, with
only the Slice blocks and with only the AMWG blocks (rats.jl:112-116), 16384 chains, specialised
kernel, HIP-event kernel time per iteration.

  python tools/ir_split.py [--iters 64]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--chains", type=int, default=16384)
    a = ap.parse_args()
    import torch  # noqa: F401
    import _mamba_path
    mb = _mamba_path.load()
    full = mb.model.rats_scheme_reference()
    kinds = {"all": full,
             "slice_only": [s for s in full if s.kind == mb.abi.MMB_SAMPLER_SLICE],
             "amwg_only": [s for s in full if s.kind == mb.abi.MMB_SAMPLER_AMWG]}
    out = {}
    for name, sch in kinds.items():
        m = mb.ir.rats_model().setinputs(mb.ir.rats_inputs()).setsamplers(sch)
        V = m.init_matrix([{**mb.model.RATS_INITS[0], "y": mb.model.RATS_Y}] * a.chains, a.chains)  # one init: unsampled nodes are data
        eng = mb.Engine(m)
        eng.init_chains(V, seed=3)
        eng.run(32, burnin=0, thin=2, draws=False)
        eng.run(a.iters, burnin=0, thin=2, draws=False, time_kernels=True)
        ms, launches, units = eng.kernel_time()
        out[name] = {"blocks": len(sch), "ms_per_iter": ms / a.iters, "chain_updates_per_s": units / (ms * 1e-3),
                     "jit": eng.ir_jit()[1]}
        eng.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
