#!/usr/bin/env python3
"""Instruction counts of a kernel's large basic blocks, from a device-only
assembly build (hipcc --cuda-device-only -S):

    python tools/isa_blocks.py <file.s> <kernel-name-regex> [min-insts] [--dump BLOCK]

Prints, for every basic block of at least min-insts instructions (default 60),
the counts of VALU (v_*; DPP forms separately), SALU (s_*, without s_nop),
s_nop, LDS (ds_*), VMEM (buffer_/global_) and waitcnt instructions.  Used for
the split column step (gx_cs2.hip): the core wave's 4-column group holds 24
v_max_i32_dpp (four 6-step scans), the side wave's likewise."""
import collections
import re
import sys


def blocks_of(path, pat):
    s = open(path).read()
    m = re.search(r"\n(" + pat + r"[A-Za-z0-9_]*):", s)
    if not m:
        sys.exit(f"no kernel matching {pat}")
    i = m.start()
    j = s.index(".Lfunc_end", i)
    out = collections.OrderedDict()
    cur = "entry"
    out[cur] = []
    for line in s[i:j].split("\n"):
        mm = re.match(r"^(\.LBB\d+_\d+):", line)
        if mm:
            cur = mm.group(1)
            out[cur] = []
            continue
        t = line.strip()
        if t and not t.startswith(";") and not t.startswith("."):
            out[cur].append(t)
    return m.group(1), out


def classify(ins):
    op = ins.split()[0]
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("v_"):
        return "dpp" if ("row_" in ins or "wave_" in ins or "quad_perm" in ins) else "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lim = int(sys.argv[3]) if len(sys.argv) > 3 and not sys.argv[3].startswith("--") else 60
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    name, blocks = blocks_of(path, pat)
    print(name)
    for k, v in blocks.items():
        if dump == k:
            print("\n".join(v))
        if len(v) < lim:
            continue
        c = collections.Counter(classify(x) for x in v)
        print(f"{k}: {len(v)} insts  valu {c['valu']} dpp {c['dpp']} salu {c['salu']} nop {c['nop']} "
              f"lds {c['lds']} vmem {c['vmem']} wait {c['wait']} other {c['other']}")


if __name__ == "__main__":
    main()
