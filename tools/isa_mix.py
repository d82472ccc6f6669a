#!/usr/bin/env python3
"""Instruction mix of a fill kernel's steady-state 4-step groups (the basic
blocks holding the compact-plane byte inserts), from a device-only assembly
build of gx_kernels.hip:

    python tools/isa_mix.py [kernel-name-regex]   (default: the bench's W=15 compact-plane kernel)

Compiles to /tmp/gx_isa/ (about 2 minutes) unless GX_ISA_S names an existing .s."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pat = sys.argv[1] if len(sys.argv) > 1 else r"_ZN2gx11fill_kernelILi15ELb0ELi2ELb1ELb0ELb0ELb1ELi0E"
s_path = os.environ.get("GX_ISA_S")
if not s_path:
    os.makedirs("/tmp/gx_isa", exist_ok=True)
    s_path = "/tmp/gx_isa/gx_kernels.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    "-o", s_path, os.path.join(ROOT, "genomics-rs_amd", "csrc", "gx_kernels.hip")], check=True)
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
for k, v in steady:
    c = collections.Counter(v)
    valu = sum(n for op, n in c.items() if op.startswith("v_"))
    print(f"{k}: {len(v)} insts, VALU {valu} ({valu / 8:.2f} per cell), SALU {sum(n for op, n in c.items() if op.startswith('s_'))}")
if steady:
    c = collections.Counter(steady[-1][1])
    for op, n in c.most_common(30):
        print(f"   {op:26s}{n}")
    if os.environ.get("GX_ISA_JSON"):
        import json
        valu = {op: n for op, n in c.items() if op.startswith("v_")}
        with open(os.environ["GX_ISA_JSON"], "w") as f:
            json.dump({"kernel": m.group(1), "block": steady[-1][0], "cells_per_lane": 8, "valu": valu,
                       "valu_total": sum(valu.values()),
                       "dual_rate": sum(n for op, n in valu.items() if op in ("v_add_u32_e32", "v_sub_u32_e32")),
                       "source": "tools/isa_mix.py (steady-state 4-step group: 4 steps x 2 rows per lane)"}, f, indent=1)
