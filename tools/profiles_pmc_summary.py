"""Summarise a profiles_run.sh output dir into profiles/.

  python profiles_pmc_summary.py gpurun_out/prof_r1c profiles/r1 [--last 8]

Writes <prefix>_sweep_summary.json (per-launch averages of the fused sweep kernel's PMC
counters, the rocprofv3 --stats average and the average of the last `--last` launches,
which are the event-timed roofline launches of bench.py), copies the kernel stats CSV
and bench line, and writes <prefix>_hbm_traffic.json (HBM bytes per launch, corrected as
MI355X_MICROARCH.md prescribes: FETCH_SIZE is KiB and reports half of wide coalesced
reads on gfx950, so bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE).
"""
import argparse
import csv
import glob
import json
import os
import hashlib
import shutil

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("prefix")
ap.add_argument("--last", type=int, default=16)
ap.add_argument("--scheme", default="gibbs_amm")
a = ap.parse_args()
# the engine build the counters were taken from (bench.py uses the traffic only for this build)
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba.jl_amd", "lib", "libmambahip.so")

out = {}
for f in sorted(glob.glob(os.path.join(a.src, "pmc_*", "run_counter_collection.csv"))):
    acc = {}
    for r in csv.DictReader(open(f)):
        if "sweep_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in acc.items():  # the last `--last` launches: bench.py's steady-state roofline window
        v = v[-a.last:]
        out[k] = sum(v) / len(v)
        out[k + "_launches"] = len(v)
st = os.path.join(a.src, "trace", "run_kernel_stats.csv")
if os.path.exists(st):
    for r in csv.DictReader(open(st)):
        if "sweep_kernel" in r["Name"]:
            out["kernel"] = r["Name"]
            out["stats_avg_ns"] = float(r["AverageNs"])
            out["stats_calls"] = int(r["Calls"])
tr = os.path.join(a.src, "trace", "run_kernel_trace.csv")
if os.path.exists(tr):
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for r in csv.DictReader(open(tr)) if "sweep_kernel" in r["Kernel_Name"]]
    last = durs[-a.last:]
    out[f"trace_avg_ns_last{len(last)}"] = sum(last) / len(last)
bench = os.path.join(a.src, "bench.json")
if os.path.exists(bench):
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    out["bench_event_avg_ns"] = b["roofline"]["avg_launch_ms"] * 1e6
    out["algorithmic_bytes_per_launch"] = (b["roofline"]["algorithmic_bytes_per_chain_update"]
                                           * b["roofline"]["chain_updates_per_launch"])
    shutil.copy(bench, a.prefix + "_bench.json")
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    hbm = 2 * 1024 * out["FETCH_SIZE"] + 1024 * out["WRITE_SIZE"]
    out["hbm_bytes_per_launch"] = hbm
    rd = os.path.dirname(os.path.abspath(a.prefix))
    cfg = b["config"] if os.path.exists(bench) else {}
    json.dump({"bytes_per_launch": hbm, "source": os.path.basename(a.prefix) + "_sweep_summary.json",
               "formula": "2*1024*FETCH_SIZE + 1024*WRITE_SIZE (KiB counters; gfx950 wide-read x2), "
                          "averaged over the last %d launches (the bench's steady-state roofline window)" % a.last,
               "algorithmic_bytes_per_launch": out.get("algorithmic_bytes_per_launch"),
               "scheme": a.scheme, "chains": cfg.get("chains_per_gpu"), "iters_per_launch": cfg.get("iters_per_launch"),
               "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest()},
              open(a.prefix + "_hbm_traffic.json", "w"), indent=1)
# FP64 VALU lane-flops (the reference Slice+AMWG scheme is bound by them, SURVEY §8(d) row 3'):
# the SQ_INSTS_VALU_*_F64 counters count wave instructions; x 64 lanes, an FMA = 2 flops
f64 = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"]
if all(k in out for k in f64) and os.path.exists(bench):
    fl = 64.0 * (out[f64[0]] + out[f64[1]] + 2.0 * out[f64[2]] + out[f64[3]])
    upd = b["roofline"]["chain_updates_per_launch"]
    out["f64_lane_flops_per_launch"] = fl
    out["f64_lane_flops_per_chain_update"] = fl / upd
    cfg = b["config"]
    json.dump({"f64_lane_flops_per_chain_update": fl / upd, "f64_lane_flops_per_launch": fl,
               "source": os.path.basename(a.prefix) + "_sweep_summary.json",
               "formula": "64 * (ADD_F64 + MUL_F64 + 2 * FMA_F64 + TRANS_F64) wave instructions per launch "
                          "(SQ_INSTS_VALU_*_F64), / chain-updates per launch; last %d launches" % a.last,
               "scheme": a.scheme, "chains": cfg.get("chains_per_gpu"), "iters_per_launch": cfg.get("iters_per_launch"),
               "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest()},
              open(a.prefix + "_valu_flops.json", "w"), indent=1)
if os.path.exists(st):
    shutil.copy(st, a.prefix + "_kernel_stats.csv")
json.dump(out, open(a.prefix + "_sweep_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
