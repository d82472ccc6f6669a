"""CPU: the C-ABI library loads and exports every symbol declared in
include/gx.h; host-only entry points (FASTA, config, Display) work without a
GPU.  No compute calls."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import COMPARISON, FASTA, GOLDEN, ROOT, read_fasta_records

HEADER = os.path.join(ROOT, "include", "gx.h")
LIB = os.path.join(ROOT, "genomics-rs_amd", "libgx_amd.so")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]*?\b(gx_\w+)\s*\(", text, re.M)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("gx_alignment_table", "gx_retrace", "gx_align", "gx_align_batch", "gx_table_export",
              "gx_fasta_load", "gx_config_load", "gx_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(gx):
    lib = gx.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gx_\w+)$", out, re.M))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    for s in declared_symbols():
        assert getattr(lib, s) is not None
    assert sorted(gx.EXPORTED) == declared_symbols()


def test_struct_layouts(gx):
    # #[repr(C)] AlignmentCell is 48 B (algo.rs:25-35); gx_step mirrors (u8, usize, usize)
    assert ctypes.sizeof(gx.CCell) == 48
    assert ctypes.sizeof(gx.CStep) == 24
    assert gx.CELL_DTYPE.itemsize == 48 and gx.STEP_DTYPE.itemsize == 24
    assert [int(c) for c in gx.AlignmentChoice] == [0, 1, 2, 3, 4, 5]


def test_version_and_error(gx):
    assert b"gfx950" in gx.lib().gx_version()
    with pytest.raises(gx.GxError):
        gx.get_config("/nonexistent/config.toml")
    assert b"Could not read config file" in gx.lib().gx_last_error()


def test_fasta_loader_matches_oracle(gx):
    """from_fasta (sequence.rs:45-95): product loader == oracle restatement
    on every FASTA fixture."""
    files = [os.path.join(FASTA, f) for f in sorted(os.listdir(FASTA))] + \
            [os.path.join(COMPARISON, f) for f in sorted(os.listdir(COMPARISON))]
    for path in files:
        sc = gx.SequenceContainer()
        sc.from_fasta(path)
        want = read_fasta_records(path)
        got = [(s.name.encode(), s.sequence.encode()) for s in sc.sequences]
        assert got == want, path


def test_fasta_appends_and_edge_cases(gx, tmp_path):
    p = tmp_path / "e.fasta"
    p.write_bytes(b"orphan\n>  a b \r\nAC GT \n\n   \n>b\n\tAAA\t\n>empty\n")
    sc = gx.SequenceContainer()
    sc.from_fasta(str(p))
    sc.from_fasta(str(p))                       # appends (sequence.rs:94)
    assert [(s.name, s.sequence) for s in sc.sequences] == [("a b", "AC GT"), ("b", "AAA"), ("empty", "")] * 2
    q = tmp_path / "bad.fasta"
    q.write_bytes(b">a\nAC\n\xff\xfe\nGG\n")
    sc = gx.SequenceContainer()
    sc.from_fasta(str(q))
    assert [(s.name, s.sequence) for s in sc.sequences] == [("a", "AC")]
    sc = gx.SequenceContainer()
    sc.from_fasta(str(tmp_path / "missing.fasta"))   # swallowed (sequence.rs:84-86)
    assert sc.sequences == []


def test_config_loader(gx, tmp_path):
    c = gx.get_config(os.path.join(GOLDEN, "config.toml"))
    assert (c.scores.s_match, c.scores.s_mismatch, c.scores.g, c.scores.h) == (1, -2, -1, -5)
    p = tmp_path / "c.toml"
    p.write_text("# comment\ntitle = 'x'\n[scores]\ns_match = +2 # two\ns_mismatch = -1_0\ng = -1\nh = -3\n"
                 "extra = 7\n[other]\ng = 99\n")
    c = gx.get_config(str(p))
    assert (c.scores.s_match, c.scores.s_mismatch, c.scores.g, c.scores.h) == (2, -10, -1, -3)
    p.write_text("scores = { s_match = 1, s_mismatch = -2, g = -2, h = -5 }\n")
    c = gx.get_config(str(p))
    assert (c.scores.g, c.scores.h) == (-2, -5)
    for bad in ("[scores]\ns_match = 1\ns_mismatch = -2\ng = -1\n",          # missing h
                "[scores]\ns_match = 1.5\ns_mismatch = -2\ng = -1\nh = -5\n",   # not an integer
                "[scores]\ns_match = 1\ns_match = 2\ns_mismatch = -2\ng = -1\nh = -5\n"):
        p.write_text(bad)
        with pytest.raises(gx.GxError):
            gx.get_config(str(p))


def _display_restatement(s1, s2, alignment, score, matches, mismatches, ext, opens):
    """Python restatement of display.rs:9-127 (the writeln! output)."""
    W = 200
    out, a1, al, a2 = [], "", "", ""
    i1 = i2 = hl = ai = 0
    for c, _, _ in reversed(alignment):
        if hl > W:
            out.append(f"\n\n{ai - W}-{ai}:\n\n{a1}\n{al}\n{a2}\n")
            a1 = al = a2 = ""
            hl = 0
        if c in ("Insert", "OpenInsert"):
            a1 += "-"
        elif i1 < len(s1):
            a1 += s1[i1]; i1 += 1
        al += {"Match": "|", "Mismatch": "x", "Insert": " ", "Delete": " "}.get(c, "%")
        if c in ("Delete", "OpenDelete"):
            a2 += "-"
        elif i2 < len(s2):
            a2 += s2[i2]; i2 += 1
        hl += 1
        ai += 1
    out.append(f"\n\n{ai - len(a1)}-{ai}:\n\n{a1}\n{al}\n{a2}\n")
    out.append(f"\n\nAlignment Score: {score}\n")
    for lab, v in (("Matches", matches), ("Mismatches", mismatches), ("Gap Extensions", ext),
                   ("Opening Gaps", opens)):
        out.append(f"{lab}: {v}/{ai} ({v / ai * 100:.2f}%)\n")
    pid = matches / ai * 100
    pid_s = repr(pid)
    if pid_s.endswith(".0"):
        pid_s = pid_s[:-2]          # Rust Display of an integral f64 omits ".0"
    out.append(f"Percent Identity {pid_s}%\n")
    return "".join(out)


def test_display_matches_restatement(gx, oracle):
    import json
    with open(os.path.join(GOLDEN, "oracle_vectors.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases[:40]:
        aln = [(x[0], x[1], x[2]) for x in c["alignment"]]
        a = gx.AlignedSequences(gx.Sequence("s1", c["s1"]), gx.Sequence("s2", c["s2"]),
                                [(gx.AlignmentChoice[x[0]], x[1], x[2]) for x in aln], c["score"],
                                c["stats"][0], c["stats"][1], c["stats"][2], c["stats"][3])
        want = _display_restatement(c["s1"], c["s2"], aln, c["score"], *c["stats"])
        assert str(a) == want, c["name"]


def _table_restatement(s1, s2, alignment, planes, color):
    """Python restatement of print_alignment_table + print_scores_table
    (display.rs:131-220): the stdout text for one alignment."""
    n, m = len(s1), len(s2)
    if not (n < 200 and m < 2000):
        return ""
    glyph = {"Match": ("M", "\x1b[32m"), "Mismatch": ("X", "\x1b[31m"), "Insert": ("I", "\x1b[34m"),
             "Delete": ("D", "\x1b[36m"), "OpenInsert": ("I", "\x1b[1;34m"), "OpenDelete": ("D", "\x1b[1;36m")}
    out = ["\nSequence Table (S1 columns, S2 rows):\n\n", " " + s2 + "\n"]
    for i in range(n):
        row = s1[i]
        for j in range(m):
            hit = next((c for c, x, y in alignment if x == i + 1 and y == j + 1), None)
            if hit is None:
                row += "."
            else:
                g, st = glyph[hit]
                row += f"{st}{g}\x1b[0m" if color else g
        out.append(row + "\n")
    for title, k in (("Delete Scores", 1), ("Insert Scores", 0), ("Sub Scores", 2)):
        out.append(title + "\n")
        out.append(". \t" + "".join(f"{j}\t" for j in range(m + 1)) + "\n")
        for i in range(n + 1):
            vals = ["-inf" if v <= -9223372036854775700 else str(int(v)) for v in planes[k][i]]
            out.append(f"{i}\t" + "".join(v + "\t" for v in vals) + "\n")
    return "".join(out)


@pytest.mark.parametrize("is_local", [False, True])
def test_alignment_table_print_matches_restatement(gx, oracle, is_local):
    """print_alignment_table (display.rs:131-220, printed by retrace at
    algo.rs:438): host formatter == restatement, on oracle planes (plain and
    coloured), including the too-large cut-off."""
    cases = [(b"BANANA", b"MISSISSIPPI"), (b"ACGGTTACGATTACA", b"ACGTTAGGATTTACGA"),
             (b"ACGT" * 49 + b"AC", b"ACGA" * 40)]
    for s1, s2 in cases:
        o = oracle.align(s1, s2, (1, -2, -1, -5), is_local=is_local, want_planes=True)
        aln = o.alignment()
        a = gx.AlignedSequences(gx.Sequence("s1", s1.decode()), gx.Sequence("s2", s2.decode()),
                                [(gx.AlignmentChoice[c], i, j) for c, i, j in aln], o.score,
                                o.matches, o.mismatches, o.gap_extensions, o.opening_gaps)
        planes = [o.planes[k] for k in range(3)]
        for color in (False, True):
            want = _table_restatement(s1.decode(), s2.decode(), aln, planes, color)
            assert gx.format_alignment_table(a, planes, color) == want
    big = gx.AlignedSequences(gx.Sequence("s1", "A" * 200), gx.Sequence("s2", "A"), [], 0, 0, 0, 0, 0)
    assert gx.format_alignment_table(big, [None] * 3) == ""


def _d8_rule(sm, smm, g, h, local):
    """Independent restatement of the compact-plane range proof."""
    if g > 0 or h > 0:
        return 12
    a = g + h
    U = max(0, max(sm, smm) - a)
    lo = min(g, min(sm, smm) - U, 2 * a - U)
    hi = max(U - a, max(sm, smm) - 2 * a, U - 2 * a)
    return 3 if lo >= -128 and hi <= 127 else 12


@pytest.mark.parametrize("scores", [(1, -2, -1, -5), (1, -2, -2, -5), (2, -3, -2, -4), (5, -4, 0, -10),
                                    (10, -10, -5, -20), (1, -1, 0, 0), (30, -30, -10, -40), (3, 1, -1, -2),
                                    (40, -1, -1, -1), (20, -20, -10, -25), (1, -2, 1, -5)])
@pytest.mark.parametrize("local", [False, True])
def test_plane_bytes_per_cell(gx, scores, local, monkeypatch):
    """Host-only: which score-plane format a batch launch picks (no GPU call)."""
    monkeypatch.delenv("GX_PLANES32", raising=False)
    assert gx.plane_bytes_per_cell(gx.Scores(*scores), local) == _d8_rule(*scores, local)
    monkeypatch.setenv("GX_PLANES32", "1")
    assert gx.plane_bytes_per_cell(gx.Scores(*scores), local) == 12


@pytest.mark.parametrize("local", [False, True], ids=["global", "local"])
def test_plan_layout(gx, local, monkeypatch):
    """Host-only: the layout rule (gx_api_plan.cpp fill_layout).  BASELINE configs
    2 and 3 take the latency layouts; a wide batch takes layout 0; columns
    past the 24-bit landing-column range of the 64-row strip layouts (the
    skeleton holds E + 64 in 24 bits, gx_kernels.hip tb_chase_kernel; a
    strip's int32 plane must stay inside one buffer descriptor) never take
    layout 3 or the column step, forced or not."""
    for k in ("GX_LAYOUT", "GX_CS2", "GX_BAND_WAVES"):
        monkeypatch.delenv(k, raising=False)
    sc = gx.Scores(1, -2, -1, -5)
    covid, brca2 = (29903, 29882), (11382, 10346)
    assert gx.plan_layout(sc, False, [covid]) == 3
    # tracked fills (max cell + matches_at_max): layout 3 at its untracked
    # pace since round 6 (the side waves keep the first maximum only, the LCS
    # runs as bit rows in workgroups of their own, gx_lcs.h), so the BASELINE
    # pairs take it in both modes
    assert gx.plan_layout(sc, False, [covid], track=True) == 3
    assert gx.plan_layout(sc, True, [brca2], track=True) == 3
    assert gx.plan_layout(sc, local, [(64, 30000)], track=True) == 3
    assert gx.plan_layout(sc, local, [(1024, 30000)], track=True) == 3
    assert gx.plan_layout(sc, True, [brca2]) == 1
    assert gx.plan_layout(sc, local, [(64, 30000)]) == 3
    assert gx.plan_layout(sc, local, [(30000, 30000)] * 80) == 0
    big = (64, (1 << 24) - 100)
    assert gx.plan_layout(sc, local, [big]) == 0
    monkeypatch.setenv("GX_LAYOUT", "3")
    assert gx.plan_layout(sc, local, [big]) == 0
    assert gx.plan_layout(sc, local, [(64, (1 << 24) - 129)]) == 3
    monkeypatch.setenv("GX_LAYOUT", "1")
    assert gx.plan_layout(sc, local, [big]) == 0
    # h > 0 (the folded gap opening needs h <= 0) and wide substitution scores
    # (the ramp-up's virtual-column drift) keep layout 3 off
    monkeypatch.setenv("GX_LAYOUT", "3")
    assert gx.plan_layout(gx.Scores(1, -2, -1, 2), local, [covid]) != 3
    assert gx.plan_layout(gx.Scores(1 << 23, -(1 << 23), -1, -5), local, [(4, 4)]) != 3
    assert gx.plan_layout(gx.Scores(1 << 20, -(1 << 20), -1, -5), local, [(4, 4)]) == 3


def test_display_log_lines():
    """display.rs:12-18 and 139-144: the Display and table renderings log the
    reference's info / warn lines on stderr under GX_LOG (CPU only: the
    formatting is host code)."""
    import subprocess
    import sys
    code = r'''
import ctypes, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import gxamd as gx
L = gx.lib()
for n in (5, 300):
    a = b"A" * n
    steps = np.zeros(n, gx.STEP_DTYPE)
    for k in range(n):
        steps[k]["choice"] = 0; steps[k]["i"] = n - k; steps[k]["j"] = n - k
    res = gx.CResult(n, n, 0, 0, 0, n, 0, 0, 0, 0, 0, 0, 0)
    buf = ctypes.create_string_buffer(1 << 16)
    need = ctypes.c_size_t(0)
    assert L.gx_format_alignment(a, n, a, n, steps.ctypes.data, n, ctypes.byref(res), buf, len(buf), ctypes.byref(need)) == 0
    pl = np.zeros((n + 1) * (n + 1), np.int64)
    L.gx_format_table(a, n, a, n, steps.ctypes.data, n, pl.ctypes.data, pl.ctypes.data, pl.ctypes.data, 0, buf, len(buf), None)
'''
    import os
    from conftest import ROOT
    env = dict(os.environ, GX_LOG="info")
    p = subprocess.run([sys.executable, "-c", code, os.path.join(ROOT, "genomics-rs_amd")], capture_output=True,
                       text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    err = p.stderr
    assert "[gx INFO] Original Sequences:\n[gx INFO] AAAAA\n[gx INFO] AAAAA\n" in err
    assert "[gx WARN] Sequences are too long to display." in err
    assert "[gx INFO] Computing sequence table visualization..." in err
    assert "[gx WARN] Sequence table too large to visualize" in err
    env["GX_LOG"] = "off"
    p = subprocess.run([sys.executable, "-c", code, os.path.join(ROOT, "genomics-rs_amd")], capture_output=True,
                       text=True, env=env, timeout=120)
    assert p.returncode == 0 and "[gx " not in p.stderr
