"""Split a logistic window's span (rocprofv3 --kernel-trace csv of tools/lg_walltime.py
--trace-only) into gradient kernels, control kernels and the gaps between launches.

  python tools/lg_trace_split.py DIR [--out profiles/r4_logistic_walltime_split.json]
"""
import argparse
import csv
import glob
import json
import os

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {a.dir}")
    rows = []
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            nm = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            if "lg_" in nm:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm))
    rows.sort()
    st = np.array([r[0] for r in rows], dtype=np.float64)
    en = np.array([r[1] for r in rows], dtype=np.float64)
    grad = np.array(["lg_grad" in r[2] for r in rows])
    dur = (en - st) / 1e9
    span = (en.max() - st.min()) / 1e9
    busy = dur.sum()
    gaps = (st[1:] - en[:-1]) / 1e9
    out = {"trace": os.path.relpath(files[0]), "launches": len(rows), "span_s": span,
           "grad_kernel_s": float(dur[grad].sum()), "ctl_kernel_s": float(dur[~grad].sum()),
           "gaps_s": float(np.clip(gaps, 0, None).sum()), "busy_s": float(busy),
           "median_gap_us": float(np.median(gaps) * 1e6), "grad_launches": int(grad.sum()),
           "ctl_launches": int((~grad).sum()),
           "median_grad_us": float(np.median(dur[grad]) * 1e6), "median_ctl_us": float(np.median(dur[~grad]) * 1e6)}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s)


if __name__ == "__main__":
    main()
