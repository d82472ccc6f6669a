#!/usr/bin/env python3
"""Instruction mix of a fill kernel's steady-state 4-step groups (the basic
blocks holding the compact-plane byte inserts), from a device-only assembly
build of gx_kernels.hip:

    python tools/isa_mix.py [kernel-name-regex]   (default: the bench's W=15 compact-plane kernel)
    python tools/isa_mix.py twin|twin7            (the twin fill, gx_fill_pk.hip, W=8, twin plane codes, score tables, no code words, no skeleton: PLANES 30)

Compiles to /tmp/gx_isa/ (about 2 minutes) unless GX_ISA_S names an existing .s.
A twin group holds 16 cells per lane (4 steps x 2 rows x 2 pairs)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pat = sys.argv[1] if len(sys.argv) > 1 else r"_ZN2gx11fill_kernelILi15ELb0ELi2ELb1ELb0ELb0ELb1ELi0E"
src, cells = "gx_kernels", 8
if pat in ("twin", "twin7"):   # twin7: the 7-wave bands the headline batch takes (two workgroups per CU)
    pat, src, cells = r"_ZN2gx14fill_pk_kernelILi%sELi30E" % ("7" if pat == "twin7" else "8"), "gx_fill_pk", 16
s_path = os.environ.get("GX_ISA_S")
if not s_path:
    os.makedirs("/tmp/gx_isa", exist_ok=True)
    s_path = f"/tmp/gx_isa/{src}.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    "-o", s_path, os.path.join(ROOT, "genomics-rs_amd", "csrc", src + ".hip")], check=True)
s = open(s_path).read()
m = re.search(r"\n(" + pat + r"[A-Za-z0-9_]*):", s)
i = m.start()
j = s.index(".Lfunc_end", i)
blocks = collections.OrderedDict()
cur = "entry"
blocks[cur] = []
for line in s[i:j].split("\n"):
    mm = re.match(r"^(\.LBB\d+_\d+):", line)
    if mm:
        cur = mm.group(1)
        blocks[cur] = []
        continue
    t = line.strip()
    if t and not t.startswith(";") and not t.startswith("."):
        blocks[cur].append(t.split()[0])
print(m.group(1))
steady = [(k, v) for k, v in blocks.items() if sum(1 for op in v if "sdwa" in op) >= 24]
if not steady:   # the twin fill inserts its plane bytes by inline asm (counted as text, not by mnemonic)
    steady = [(k, v) for k, v in blocks.items() if sum(1 for op in v if op.startswith("v_pk_max")) >= 24]
for k, v in steady:
    c = collections.Counter(v)
    valu = sum(n for op, n in c.items() if op.startswith("v_"))
    print(f"{k}: {len(v)} insts, VALU {valu} ({valu / cells:.2f} per cell), SALU {sum(n for op, n in c.items() if op.startswith('s_'))}")
if steady:
    c = collections.Counter(steady[-1][1])
    for op, n in c.most_common(30):
        print(f"   {op:26s}{n}")
    if os.environ.get("GX_ISA_JSON"):
        import json
        valu = {op: n for op, n in c.items() if op.startswith("v_")}
        with open(os.environ["GX_ISA_JSON"], "w") as f:
            json.dump({"kernel": m.group(1), "block": steady[-1][0], "cells_per_lane": cells, "valu": valu,
                       "valu_total": sum(valu.values()),
                       "dual_rate": sum(n for op, n in valu.items() if op in ("v_add_u32_e32", "v_sub_u32_e32", "v_subrev_u32_e32")),
                       "source": f"tools/isa_mix.py (steady-state 4-step group: {cells} cells per lane)"}, f, indent=1)
