"""How stable is the pivot order of AMM's pivoted Cholesky from one update to the next?

  python tools/pivot_stability.py [--chains 512] [--iters 600] [--prerun 128]

Runs the CPU oracle (test infrastructure) on the bench's rats Gibbs+AMM workload, one
iteration at a time, and after every iteration rebuilds each AMM block's Sigma from the oracle's
tune state (amm.jl:84-87: (scale^2/n/p) (Mvv - Mv Mv')), factorizes it with the oracle's dpstf2
restatement and compares the pivot sequence with the one of the previous update of the same
chain.  Reports per block:
* full_rank_frac: updates whose factorization reached rank d (rank(F) == n, amm.jl:88);
* rank_mean: mean rank reached (steps that took a pivot);
* pred_hit: updates whose pivots (all `rank` of them) are exactly the previous update's order
  (the previous order as a permutation: its pivots in step order, the elements it did not
  reach after them in their previous relative order) -- the fraction of factorizations a
  kernel that predicts the pivot order from the last update would not have to redo.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=512)
    ap.add_argument("--iters", type=int, default=600)
    ap.add_argument("--prerun", type=int, default=128)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    import _mamba_path
    import oracle_lib
    mb = _mamba_path.load()
    orc = oracle_lib.Oracle()
    model = mb.rats()
    model.setinputs(mb.model.RATS_DATA)
    model.setsamplers(mb.model.rats_scheme_gibbs_amm())
    init = mb.model.rats_init_ls(16384, seed=1000)[:a.chains]
    st = orc.new_state(model, init)
    d = 30
    T = d * (d + 1) // 2
    tl = 4 + 2 * d + 2 * T
    offs = {"alpha": 0, "beta": tl}
    tri = np.array([i * (i + 1) // 2 for i in range(d)])
    ii, kk = np.tril_indices(d)
    scale = 2.38
    orc.run(model, st, a.prerun, seed=7, nthreads=a.threads, draws=False)
    prev = {b: [None] * a.chains for b in offs}
    stats = {b: {"n": 0, "full": 0, "rank": 0, "hit": 0, "hit_full": 0, "n_full": 0, "hit_def": 0, "n_def": 0}
             for b in offs}
    for it in range(a.iters):
        orc.run(model, st, 1, seed=7, nthreads=a.threads, draws=False)
        for b, o in offs.items():
            t = st["tune"][:, o:o + tl]
            for c in range(a.chains):
                m = t[c, 1]
                p = m / (m + 1.0)
                Mv = t[c, 4:4 + d]
                Mvv = t[c, 4 + d:4 + d + T]
                cc = (scale * scale / d) / p
                S = np.zeros((d, d))
                # the oracle's Sigma: cc * (Mvv[tri(i)+k] - Mv[k] * Mv[i]), symmetric
                vals = cc * (Mvv[tri[ii] + kk] - Mv[kk] * Mv[ii])
                S[ii, kk] = vals
                S[kk, ii] = vals
                r, _, piv = orc.pchol(S)
                piv = list(piv[:r])
                s = stats[b]
                s["n"] += 1
                s["rank"] += r
                full = r == d
                s["full"] += full
                order = prev[b][c]
                if order is not None:
                    hit = order[:r] == piv
                    s["hit"] += hit
                    if full:
                        s["n_full"] += 1
                        s["hit_full"] += hit
                    else:
                        s["n_def"] += 1
                        s["hit_def"] += hit
                    if not hit:
                        fm = next(j for j in range(r) if order[j] != piv[j])
                        s.setdefault("first_miss", []).append(fm)
                    if hit:
                        continue  # a kernel that predicted right keeps its order
                rest = [e for e in (order or range(d)) if e not in piv]
                prev[b][c] = piv + rest
    out = {}
    for b, s in stats.items():
        n = s["n"]
        out[b] = {"updates": n, "full_rank_frac": s["full"] / n, "rank_mean": s["rank"] / n,
                  "pred_hit": s["hit"] / max(1, s["n_full"] + s["n_def"]),
                  "pred_hit_full_rank": s["hit_full"] / max(1, s["n_full"]),
                  "pred_hit_rank_deficient": s["hit_def"] / max(1, s["n_def"]),
                  "first_miss_step_hist": np.bincount(s.get("first_miss", [0]), minlength=d).tolist(),
                  "pred_steps_frac": (s["rank"] - sum(r_ for r_ in [0])) and None}
    out["config"] = {"chains": a.chains, "prerun": a.prerun, "iters": a.iters,
                     "inits": "rats_init_ls(16384, seed=1000)[:chains]", "seed": 7}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
