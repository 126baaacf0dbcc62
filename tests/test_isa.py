"""ISA checks of the built sweep kernels (no GPU needed: the gfx950 code object is taken
from the in-tree build's fat binary and disassembled with the ROCm LLVM tools).

device.h fmac_rowbc issues `v_fmac_f64_dpp ... row_newbcast` from inline asm, which the
compiler's hazard recognizer does not look into, and adds the wait states a DPP read of a
VGPR needs after a VALU write of it (two) by hand on the first use of each source value.
test_dpp_sources_have_wait_states checks every such instruction of the built code: where the
last VALU write of its DPP source lies in the same straight-line stretch of code, at least two
wait states (an s_nop N counts N + 1, any other instruction 1) separate the two.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "mamba.jl_amd", "lib", "obj", "sweep.hip.o")
LLVM = "/opt/rocm/lib/llvm/bin"


def _disassemble(tmp):
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    if not os.path.exists(OBJ) or not all(os.path.exists(t) for t in tools):
        pytest.skip("no in-tree build object or ROCm LLVM tools")
    fat, co = os.path.join(tmp, "fatbin.bin"), os.path.join(tmp, "sweep.co")
    subprocess.run([tools[0], f"--dump-section=.hip_fatbin={fat}", OBJ, os.path.join(tmp, "host.o")], check=True)
    subprocess.run([tools[1], "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--input={fat}", f"--output={co}"], check=True)
    out = subprocess.run([tools[2], "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True)
    return out.stdout.splitlines()


def _regs(op):
    """VGPR indices named by one operand: v7 -> {7}, v[8:9] -> {8, 9}."""
    m = re.fullmatch(r"v(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def test_dpp_sources_have_wait_states(tmp_path):
    lines = _disassemble(str(tmp_path))
    ins, targets = [], set()
    for ln in lines:
        m = re.match(r"\s+([a-z_0-9]+)(?:\s+(.*?))?\s*// ([0-9A-F]+):", ln)
        if m:
            mn, ops, addr = m.group(1), m.group(2) or "", int(m.group(3), 16)
            ins.append((mn, ops, addr))
            if mn.startswith(("s_branch", "s_cbranch")):   # target = pc + 4 + 4 * simm16
                off = int(ops.split()[0])
                targets.add(addr + 4 + 4 * (off - (1 << 16) if off >= 1 << 15 else off))
        elif re.match(r"^[0-9a-f]+ <.*>:", ln):
            ins.append(("<label>", "", -1))
    checked = 0
    last_write = {}      # vgpr -> index of the last VALU write in this straight-line stretch
    ws_at = [0]          # cumulative wait states before instruction i
    for i, (mn, ops, addr) in enumerate(ins):
        if addr in targets:  # another path may enter here: its writes are not in view
            last_write.clear()
        cost = (int(ops.split()[0], 0) + 1) if mn == "s_nop" and ops else 1
        if mn == "v_fmac_f64_dpp":
            src = ops.split(",")[1].strip()
            for r in _regs(src):
                if r in last_write:
                    j = last_write[r]
                    gap = ws_at[i] - ws_at[j + 1]   # wait states strictly between write j and read i
                    assert gap >= 2, f"DPP read of v{r} {gap} wait states after its VALU write (instr {j} -> {i})"
                    checked += 1
        # straight-line stretch ends at labels and branches: forget the writes
        if mn == "<label>" or mn.startswith("s_branch") or mn.startswith("s_cbranch") or mn.startswith("s_setpc"):
            last_write.clear()
        elif mn.startswith("v_") and not mn.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
            dst = ops.split(",")[0].strip() if ops else ""
            for r in _regs(dst):
                last_write[r] = i
            if mn.startswith("v_permlane") and "," in ops:  # permlane swaps write both operands
                for r in _regs(ops.split(",")[1].strip()):
                    last_write[r] = i
        ws_at.append(ws_at[-1] + cost)
    assert checked > 100, checked   # the rats / node-IR factorization steps are covered


def test_isa_census_finds_the_factorization_steps():
    """tools/isa_census.py locates the steps of the rats factorization (step j: j DPP fmacs).  The
    rats kernel's copy with d = 30 a compile-time constant has no dot product at its last step
    (no rows left), so the run it finds ends at step 28 (29 steps); a runtime-d copy shows 30."""
    if not os.path.exists(OBJ) or not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("no in-tree build object or ROCm LLVM tools")
    import importlib.util
    spec = importlib.util.spec_from_file_location("isa_census", os.path.join(ROOT, "tools", "isa_census.py"))
    ic = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ic)
    ins = ic.kernel_instructions(ic.disassemble())
    steps = ic.factorization_steps(ins)
    assert len(steps) in (29, 30)
    for j, (lo, hi) in enumerate(steps):
        assert sum(1 for mn, _ in ins[lo:hi] if mn == "v_fmac_f64_dpp") == j
