"""Per-kernel duration statistics from a rocprofv3 rocpd database (default output format).

  python tools/rocpd_kernels.py gpurun_out/prof_lg [--match lg_] [--tail-frac 0.5]

Prints, for each kernel name containing --match, the launch count, mean / median / 95th
percentile duration (us) and total (ms) over the last --tail-frac of the matching launches
(the timed region of a bench run comes last), plus the median gap between launches.
"""
import argparse
import glob
import os
import sqlite3

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--tail-frac", type=float, default=0.5)
    a = ap.parse_args()
    dbs = glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)
    if not dbs:
        raise SystemExit(f"no rocpd database under {a.dir}")
    rows = sqlite3.connect(dbs[0]).execute("select name, start, end from kernels order by start").fetchall()
    rows = [r for r in rows if a.match in r[0]]
    rows = rows[int(len(rows) * (1 - a.tail_frac)):]
    for nm in sorted({r[0] for r in rows}):
        d = np.array([(r[2] - r[1]) / 1e3 for r in rows if r[0] == nm])
        print(f"{nm[:60]:60s} n={len(d):6d} mean={d.mean():9.2f} med={np.median(d):9.2f} "
              f"p95={np.percentile(d, 95):9.2f} us  total={d.sum() / 1e3:9.3f} ms")
    st = np.array([r[1] for r in rows])
    en = np.array([r[2] for r in rows])
    if len(rows) > 1:
        print(f"median gap between launches {np.median((st[1:] - en[:-1]) / 1e3):.2f} us")


if __name__ == "__main__":
    main()
