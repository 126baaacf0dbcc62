"""Per-launch averages of the rats sweep kernel's counters from tools/pmc_quick.sh (last 16
launches = bench.py's steady-state roofline window), plus derived issue fractions."""
import csv
import glob
import json
import os
import sys

src = sys.argv[1]
out = {}
for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
    acc = {}
    for r in csv.DictReader(open(f)):
        if "sweep_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in acc.items():
        v = v[-16:]
        out[k] = sum(v) / len(v)
if "GRBM_GUI_ACTIVE" in out:
    cyc = out["GRBM_GUI_ACTIVE"] / 8.0                        # per XCD
    simd_cycles = cyc * 1024
    out["derived_cycles_per_xcd"] = cyc
    if "SQ_ACTIVE_INST_VALU" in out:
        out["derived_valu_issue_frac"] = 4.0 * out["SQ_ACTIVE_INST_VALU"] / simd_cycles
    if "SQ_INSTS_VALU" in out:
        out["derived_valu_inst_frac"] = 4.0 * out["SQ_INSTS_VALU"] / simd_cycles
json.dump(out, open(os.path.join(src, "summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
