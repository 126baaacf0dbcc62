"""Every `file.jl:a-b` citation in the oracle, the kernels, the C ABI header and the host
mirror points at lines that exist in the reference (an oracle must cite what
it restates).  Bare file names are resolved against the reference tree by suffix; skipped
when /root/reference is absent (the GPU box)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
SCAN = ["oracle", "mamba.jl_amd", "include", "tests", "DESIGN.md", "INTEGRATION.md", "bench.py", "julia"]
CITE = re.compile(r"((?:[\w.-]+/)*[\w.-]+\.(?:jl|rst)):(\d+)(?:-(\d+))?")


def _sources():
    for entry in SCAN:
        p = os.path.join(ROOT, entry)
        if os.path.isfile(p):
            yield p
        for dp, _, fs in os.walk(p):
            for f in fs:
                if f.endswith((".c", ".h", ".hip", ".cpp", ".py", ".md", ".jl")):
                    yield os.path.join(dp, f)


def _ref_files():
    out = {}
    for dp, _, fs in os.walk(REF):
        for f in fs:
            if f.endswith((".jl", ".rst")):
                full = os.path.join(dp, f)
                out[os.path.relpath(full, REF)] = full
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_reference_citations_exist():
    ref = _ref_files()
    lines = {}
    bad, n = [], 0
    for src in _sources():
        for ln, text in enumerate(open(src, errors="replace"), 1):
            for m in CITE.finditer(text):
                name, a, b = m.group(1), int(m.group(2)), int(m.group(3) or m.group(2))
                cands = [k for k in ref if k == name or k.endswith("/" + name)]
                if not cands:
                    continue  # not a reference path (e.g. the repo's own julia/MambaHIP.jl)
                n += 1
                ok = False
                for k in cands:
                    if k not in lines:
                        lines[k] = sum(1 for _ in open(ref[k], errors="replace"))
                    ok |= 1 <= a <= b <= lines[k]
                if not ok:
                    bad.append(f"{os.path.relpath(src, ROOT)}:{ln}: {m.group(0)} ({cands[0]} has {lines[cands[0]]} lines)")
    assert n > 50
    assert not bad, "\n".join(bad)
