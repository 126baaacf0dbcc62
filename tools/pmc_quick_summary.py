"""Per-launch averages of the sweep kernel's counters from tools/pmc_quick.sh, plus derived issue
fractions.

  python tools/pmc_quick_summary.py DIR [KERNEL_SUBSTRING] [LAST]

KERNEL_SUBSTRING: "sweep_kernel" (default) or "mmb_ir_jit_kernel" (the node-IR specialised
kernel); LAST: launches averaged, the bench's timed window (default 16)."""
import csv
import glob
import json
import os
import sys

src = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "sweep_kernel"
last = int(sys.argv[3]) if len(sys.argv) > 3 else 16
out = {"kernel": kname, "launches_averaged": last}
for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
    acc = {}
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in acc.items():
        v = v[-last:]
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
