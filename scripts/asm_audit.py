#!/usr/bin/env python3
"""Audit the gfx950 assembly of a HIP source: per kernel, MFMA count, vmcnt(0) waits, branches,
scratch use, and the VGPR/SGPR/LDS numbers from the metadata (cdna_hip_programming.md §7)."""
import re
import subprocess
import sys
import tempfile
import os

src = os.path.abspath(sys.argv[1])
inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "include")
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{inc}", "-munsafe-fp-atomics",
                    "-c", src, "-o", os.path.join(d, "x.o"), "-save-temps"], cwd=d, check=True,
                   capture_output=True)
    s = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
    text = open(os.path.join(d, s)).read()
for m in re.finditer(r"^(_Z\S+):[^\n]*\n", text, re.M):
    name = m.group(1)
    end = text.find("s_endpgm", m.end())
    body = text[m.end():end]
    md = text.find(".name:           " + name)
    vg = re.search(r"\.vgpr_count:\s+(\d+)", text[md:]) if md >= 0 else None
    sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", text[md:]) if md >= 0 else None
    print(f"vgpr={vg.group(1) if vg else '?':>4} spill={sp.group(1) if sp else '?':>3} ", end="")
    print(f"{name[:70]:70s} mfma={body.count('v_mfma'):4d} vmcnt0={body.count('vmcnt(0)'):3d} "
          f"br={body.count('s_cbranch'):3d} scratch={body.count('scratch_'):3d} bufld={body.count('buffer_load'):3d}")
