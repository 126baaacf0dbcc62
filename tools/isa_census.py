"""ISA census of the rats sweep kernel's pivoted-Cholesky step (pchol32, samplers.h).

  python tools/isa_census.py [--out profiles/r3_pchol32_isa_census.json]

Disassembles `sweep_kernel<2, 36>` (rats Gibbs + AMM) from the in-tree build object (no GPU
needed), finds the optimistic pass of the 30-step factorization — each step issues one
`v_permlane16_swap` (the pivot search's 32-lane max) and step j issues j `v_fmac_f64_dpp`
(the row update's dot product over the j published pivot rows) — and counts the static
instructions of every step by class.  The per-step classes show what a step costs beyond its
dot product: the search (DPP max + swap + ballot), the pivot lane's sqrt/reciprocal and
row publish, the row update's address math, and the scalar bookkeeping of the redo test.
"""
import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "mamba.jl_amd", "lib", "obj", "sweep.hip.o")
LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "_Z12sweep_kernelILi2ELj36EEv9SweepArgs"

CLASSES = [
    ("dot_fmac_dpp", lambda m: m == "v_fmac_f64_dpp"),
    ("f64_arith", lambda m: re.match(r"v_(fma|fmac|mul|add|rsq|rcp|sqrt|min|max)_f64", m) is not None),
    ("dpp_int_max", lambda m: m.startswith("v_max_i32_dpp") or m.startswith("v_max_u32_dpp")),
    ("permlane", lambda m: m.startswith("v_permlane")),
    ("v_move_select", lambda m: m.startswith(("v_mov", "v_cndmask", "v_readlane", "v_readfirstlane", "v_writelane"))),
    ("v_compare", lambda m: m.startswith("v_cmp")),
    ("v_int_bitop", lambda m: m.startswith("v_")),
    ("lds", lambda m: m.startswith("ds_")),
    ("vmem", lambda m: m.startswith(("global_", "buffer_", "flat_"))),
    ("s_nop", lambda m: m == "s_nop"),
    ("s_waitcnt", lambda m: m.startswith("s_waitcnt")),
    ("branch", lambda m: m.startswith(("s_branch", "s_cbranch"))),
    ("salu", lambda m: m.startswith("s_")),
]


def classify(mn):
    for name, f in CLASSES:
        if f(mn):
            return name
    return "other"


def disassemble():
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    with tempfile.TemporaryDirectory() as tmp:
        fat, co = os.path.join(tmp, "fatbin.bin"), os.path.join(tmp, "sweep.co")
        subprocess.run([tools[0], f"--dump-section=.hip_fatbin={fat}", OBJ, os.path.join(tmp, "host.o")], check=True)
        subprocess.run([tools[1], "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fat}", f"--output={co}"], check=True)
        out = subprocess.run([tools[2], "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True)
    return out.stdout.splitlines()


def kernel_instructions(lines, symbol=KERNEL):
    ins, inside = [], False
    for ln in lines:
        if re.match(r"^[0-9a-f]+ <.*>:", ln):
            inside = f"<{symbol}>" in ln
            continue
        if inside:
            m = re.match(r"\s+([a-z_0-9]+)(?:\s+(.*?))?\s*// ([0-9A-F]+):", ln)
            if m:
                ins.append((m.group(1), m.group(2) or ""))
    return ins


def factorization_steps(ins):
    """Segments [swap_k, swap_k+1) of the first run where segment j holds j DPP fmacs."""
    sw = [i for i, (mn, _) in enumerate(ins) if mn.startswith("v_permlane16_swap")]
    segs = list(zip(sw, sw[1:] + [len(ins)]))
    ndpp = [sum(1 for mn, _ in ins[a:b] if mn == "v_fmac_f64_dpp") for a, b in segs]
    for s in range(len(segs)):
        run = 0
        while s + run < len(segs) and ndpp[s + run] == run:
            run += 1
        if run >= 29:
            return segs[s:s + run]
    raise RuntimeError("factorization step run not found")


def census(ins):
    return dict(collections.Counter(classify(mn) for mn, _ in ins))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r4_pchol32_isa_census.json"))
    a = ap.parse_args()
    ins = kernel_instructions(disassemble())
    steps = factorization_steps(ins)
    per_step = [census(ins[lo:hi]) for lo, hi in steps]
    names = [n for n, _ in CLASSES] + ["other"]
    # the last step of the run also holds the pass's exit code (rank, redo test, epilogue start)
    body = per_step[:-1]
    mean = {n: sum(s.get(n, 0) for s in body) / len(body) for n in names}
    non_dot_valu = {j: sum(v for k, v in s.items() if k in ("f64_arith", "dpp_int_max", "permlane", "v_move_select",
                                                           "v_compare", "v_int_bitop")) for j, s in enumerate(body)}
    out = {
        "kernel": "sweep_kernel<2, 36> (rats Gibbs + AMM)",
        "source": "mamba.jl_amd/lib/obj/sweep.hip.o (gfx950 code object), static instruction counts",
        "steps_found": len(steps),
        "per_step": per_step,
        "mean_over_steps_0_to_%d" % (len(body) - 1): mean,
        "non_dot_valu_per_step": non_dot_valu,
        "kernel_total": census(ins),
        "note": "step j = one v_permlane16_swap to the next; j v_fmac_f64_dpp = the dot product over the j "
                "published pivot rows; the remaining VALU is search, pivot sqrt/reciprocal (pivot lanes only, "
                "exec-masked but issued for the whole wave), address math and selects",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(steps)} steps; mean static instructions per step (steps 0-{len(body) - 1}):")
    for n in names:
        if mean[n]:
            print(f"  {n:14s} {mean[n]:6.1f}")
    print("non-dot VALU per step:", " ".join(str(non_dot_valu[j]) for j in sorted(non_dot_valu)))


if __name__ == "__main__":
    main()
