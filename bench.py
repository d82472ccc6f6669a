#!/usr/bin/env python3
"""bench.py -- GCUPS of the MI355X affine-gap aligner on synthetic 30k x 30k
DNA pairs (BASELINE.json metric), 1..8 GPUs, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs-per-gpu P]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A STEP is one pass of the hot path over one batch: for each of the P
synthetic 30k x 30k pairs resident on this GPU, the full-table fill that
writes the three score planes (alignment_table, algo.rs:151-282; stored as
exact per-cell byte differences when the scores allow it, gx_api_plan.cpp
d8_planes_ok, else int32) plus
the traceback (retrace, algo.rs:287-441) down to the labelled alignment on
the host.  Inputs are staged in HBM before the timed region; the K timed
steps run as one pipelined call (step k's host labelling overlaps step k+1's
fill on the device; all K complete inside the timed region).  Each rank
aligns its own pairs (weak scaling); RCCL (torch.distributed "nccl") carries
only the barrier, the max-over-ranks time and the gather of per-pair
results.  value = all ranks' cells / max-over-ranks time (GCUPS).

P defaults to the pairs whose planes fill ~220 GB of HBM, at most 80 (80 x 30k
with compact planes, 20 with int32 planes).

roofline: the fill kernel's score-plane writes, B bytes per cell (3 compact,
12 int32); achieved = B * cells / average fill-kernel time
from HIP events on the kernel's own stream.  With compact planes the fill is
issue-bound rather than HBM-bound: no_plane_fill times the same batch without
plane stores (the kernel's compute ceiling) for comparison.  cpu_baseline: the reference-layout C
restatement (oracle/, 48-B cells, column-major, i-outer/j-inner, one core)
on the first R rows of the same synthetic pair.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))

PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
MEASURED_HBM_GBS = 6290.0  # float4 copy ceiling (same source)
PLANE_BUDGET = 220e9       # bytes of score planes per GPU the default batch is sized to (288 GiB HBM)
MAX_DEFAULT_PAIRS = 80     # 80 x 30k at 15-strip bands = 1,280 bands = 5 full rounds on 256 CUs
SCORES = (1, -2, -1, -5)   # config.toml:1-5


def splitmix64_bases(seed: int, length: int) -> bytes:
    """bytes i.i.d. over ACGT from SplitMix64, base = "ACGT"[x >> 62]."""
    with np.errstate(over="ignore"):
        k = np.arange(1, length + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return np.frombuffer(b"ACGT", np.uint8)[(z >> np.uint64(62)).astype(np.int64)].tobytes()


def synth_pair(k: int, length: int):
    return (splitmix64_bases(0x5EED0001 + 0x10000 * k, length),
            splitmix64_bases(0x5EED0002 + 0x10000 * k, length))


def related_pair(k: int, length: int):
    """SURVEY.md 8(d) M1 "related" variant: s1 = synthetic pair k's s1; s2 =
    s1 with ~10 % substitutions and ~1 % indels of length 1-10, drawn from a
    SplitMix64 stream seeded 0x5EED0003 + 0x10000 k.  Per position of s1: u =
    top 53 bits of the next draw; u < 0.01: an indel (next draw y: length 1 +
    y % 10; bit 32 of y set: delete that many bases of s1, else insert that
    many random bases before the current one); u < 0.11: substitute a
    different base ("ACGT"[(b + 1 + y % 3) % 4]); else copy."""
    s1 = splitmix64_bases(0x5EED0001 + 0x10000 * k, length)
    state = (0x5EED0003 + 0x10000 * k) & 0xFFFFFFFFFFFFFFFF
    M = 0xFFFFFFFFFFFFFFFF

    def draw():
        nonlocal state
        state = (state + 0x9E3779B97F4A7C15) & M
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    code = {65: 0, 67: 1, 71: 2, 84: 3}
    out = bytearray()
    i = 0
    p_indel, p_sub = int(0.01 * 2 ** 53), int(0.11 * 2 ** 53)
    while i < length:
        u = draw() >> 11
        if u < p_indel:
            y = draw()
            n = 1 + y % 10
            if (y >> 32) & 1:
                i += n
                continue
            for _ in range(n):
                out.append(b"ACGT"[draw() >> 62])
            out.append(s1[i])
        elif u < p_sub:
            out.append(b"ACGT"[(code[s1[i]] + 1 + draw() % 3) % 4])
        else:
            out.append(s1[i])
        i += 1
    return s1, bytes(out)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(s1: bytes, s2: bytes, target_s: float, is_local: bool):
    """Reference-layout restatement timed on this host, one core, on the first
    R rows of the pair (bounded sample; the per-row access pattern -- a
    (n+1)*48-B column stride per j step -- is that of the full table)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/measurement infrastructure, CPU baseline only
    import tempfile
    path = os.path.join(tempfile.mkdtemp(prefix="gx_cpu_"), "liboracle_native.so")
    try:
        oracle.build(native=True, out=path)
        kind_note = "gcc -O3 -march=native"
    except Exception as e:  # no compiler: fall back to the shipped portable build
        log("cpu_baseline: native build failed (%s); using oracle/liboracle.so" % e)
        oracle.build()
        path = oracle.LIB_PATH
        kind_note = "gcc -O3 -march=x86-64-v3"
    try:
        allowed = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {sorted(allowed)[0]})
    except Exception:
        allowed = None
    # grow the sample until one run takes >= half the target (the per-row cost
    # falls as rows share pages of the column-major table, so extrapolating
    # from a few rows would overshoot); the touched part of the table stays
    # under ~24 GB
    max_rows = min(len(s1) + 1, int(24e9 / (48 * (len(s2) + 1))))
    rows = 64
    while True:
        t0 = time.perf_counter()
        cells, ck = oracle.ref_layout_fill_rows(s1, s2, rows, SCORES, is_local, lib_path=path)
        dt = time.perf_counter() - t0
        if dt >= target_s / 2 or rows >= max_rows:
            break
        rows = int(min(max_rows, rows * min(8.0, max(2.0, target_s / max(dt, 1e-3)))))
    if allowed:
        try:
            os.sched_setaffinity(0, allowed)
        except Exception:
            pass
    return {
        "value": round(cells / dt / 1e9, 6),
        "unit": "GCUPS",
        "cores": 1,
        "kind": "port",
        "sample": f"alignment_table fill, reference layout (48-B AoS cells, column-major (n+1)x(m+1), "
                  f"i-outer/j-inner, int64; C restatement, {kind_note}) over the first {rows - 1} interior rows "
                  f"x {len(s2)} columns of synthetic pair 0 ({len(s1)}x{len(s2)}); {cells} cells in {dt:.2f} s",
        "seconds": round(dt, 3),
        "cpu": _cpu_model(),
    }


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def load_traffic(workload: str, twin: bool = False):
    """HBM bytes per fill launch from the committed PMC profile of this
    workload and fill kernel (profiles/pmc_fill_*.json, made by
    tools/gpu_profile.sh + tools/rocpd_summary.py)."""
    for name in sorted(os.listdir(os.path.join(ROOT, "profiles")), reverse=True) if os.path.isdir(
            os.path.join(ROOT, "profiles")) else []:
        if name.startswith("pmc_fill") and name.endswith(".json"):
            try:
                with open(os.path.join(ROOT, "profiles", name)) as f:
                    d = json.load(f)
                if d.get("workload") == workload and ("fill_pk_kernel" in d.get("kernel", "")) == twin:
                    return d.get("hbm_bytes_per_launch"), name
            except Exception:
                continue
    return None, None


def load_valu(workload: str, twin: bool = False):
    """VALU issue profile of this workload's fill (profiles/valu_fill_*.json,
    made by tools/gpu_valu.sh + tools/valu_summary.py): VALU instructions per
    cell (SQ_INSTS_VALU), the shader clock under this load and the VALU
    lane-operation ceiling at the fill's instruction mix, measured by
    tools/valu_probe.hip -- the bound of the compact-plane fill."""
    d = os.path.join(ROOT, "profiles")
    for name in sorted(os.listdir(d), reverse=True) if os.path.isdir(d) else []:
        if name.startswith("valu_fill") and name.endswith(".json"):
            try:
                with open(os.path.join(d, name)) as f:
                    v = json.load(f)
                if "ceiling" not in v:
                    continue
                for case in ("planes", "noplanes"):
                    c = v.get(case, {})
                    if c.get("workload") == workload and ("fill_pk_kernel" in c.get("kernel", "")) == twin:
                        return {"valu_insts_per_cell": c["valu_insts_per_cell"],
                                "valu_issue_frac": c["valu_issue_frac"], "clock_ghz": c["clock_ghz"],
                                "peak_tops": c["valu_lane_ops_peak_tops"],
                                "cpi_fill_mix": v["ceiling"]["cpi_fill_mix"],
                                "dual_issued_fraction": c["dual_issued_fraction"], "source": name}
            except Exception:
                continue
    return None


def cpu_baseline_parallel(pairs, threads: int, target_s: float, is_local: bool):
    """The same reference-layout restatement on `threads` host cores at once,
    one independent pair per thread (the batch shape the GPU runs; the
    reference's own CLI aligns one pair at a time): each thread fills the first
    R rows of its pair, R sized so all tables stay under ~48 GB, timed
    wall-clock.  ctypes releases the GIL for the duration of each fill."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/measurement infrastructure, CPU baseline only
    import tempfile
    import threading
    path = os.path.join(tempfile.mkdtemp(prefix="gx_cpu_"), "liboracle_native.so")
    try:
        oracle.build(native=True, out=path)
    except Exception:
        oracle.build()
        path = oracle.LIB_PATH
    threads = max(1, min(threads, len(pairs)))
    cpus = sorted(os.sched_getaffinity(0))[:threads]
    threads = len(cpus)
    m = max(len(b) for _, b in pairs[:threads])
    max_rows = int(48e9 / threads / (48 * (m + 1)))
    rows = 64
    while True:
        res = [None] * threads

        def work(k):
            try:
                os.sched_setaffinity(0, {cpus[k]})   # this thread only (Linux: per-thread affinity)
            except Exception:
                pass
            a, b = pairs[k]
            res[k] = oracle.ref_layout_fill_rows(a, b, min(rows, len(a) + 1), SCORES, is_local, lib_path=path)[0]

        ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = time.perf_counter() - t0
        if dt >= target_s / 2 or rows >= max_rows:
            break
        rows = int(min(max_rows, rows * min(8.0, max(2.0, target_s / max(dt, 1e-3)))))
    cells = sum(res)
    return {
        "value": round(cells / dt / 1e9, 6), "unit": "GCUPS", "cores": threads, "kind": "port",
        "sample": f"the cpu_baseline restatement on {threads} cores at once, one synthetic pair per core "
                  f"(pairs 0-{threads - 1}), first {rows - 1} interior rows x {m} columns each; {cells} cells in "
                  f"{dt:.2f} s wall",
        "seconds": round(dt, 3),
    }


def fasta_pair(gx, which: str):
    """BASELINE configs 2 and 3: the reference's own FASTA pairs (copied under
    tests/golden), loaded with the from_fasta mirror."""
    g = os.path.join(ROOT, "tests", "golden")
    cont = gx.SequenceContainer()
    if which == "covid":
        cont.from_fasta(os.path.join(g, "comparison_data", "Covid_Wuhan.fasta"))
        cont.from_fasta(os.path.join(g, "comparison_data", "Covid_USA-CA4.fasta"))
    else:
        cont.from_fasta(os.path.join(g, "fasta", "Human-Mouse-BRCA2-cds.fasta"))
    return cont.sequences[0].sequence.encode(), cont.sequences[1].sequence.encode()


def config_record(gx, ctx, which: str, steps: int, tracked: bool = False):
    """BASELINE configs 2 (Covid_Wuhan x Covid_USA-CA4, global) and 3 (Human x
    Mouse BRCA2, local): the reference's align call (main.rs:143-150), one pair
    per call, resident in HBM, with int32 score planes and traceback, `steps`
    timed passes (bench.py's own clock), then one untimed pass with device
    plane checksums compared with tests/golden/large_digests.json (score,
    statistics, alignment sha256, the three plane checksums).  tracked: the
    fill also keeps alignment_table's running max cell and matches_at_max
    (algo.rs:258-262, 279), as the drop-in alignment_table call does; both are
    checked too."""
    a, b = fasta_pair(gx, which)
    local = which == "brca2"
    scores = gx.Scores(*SCORES)
    st = gx.StagedPairs([(a, b)], ctx=ctx)
    st.run(scores, local, True, max_cell=tracked)
    t0 = time.perf_counter()
    res, fms = st.run(scores, local, True, steps=steps, max_cell=tracked)
    el = time.perf_counter() - t0
    finfo = ctx.fill_info()
    cells = len(a) * len(b)
    out = {"workload": f"{'Covid_Wuhan x Covid_USA-CA4' if which == 'covid' else 'Human x Mouse BRCA2 cds'} "
                       f"({len(a)}x{len(b)}), {'local SW' if local else 'global NW'}, scores {SCORES}, "
                       f"{plane_desc(finfo['plane_bytes_per_cell'])}"
                       + (", max cell + matches_at_max tracked (alignment_table)" if tracked else ""),
           "gcups": round(cells * steps / el / 1e9, 3), "ms_per_step": round(el / steps * 1e3, 3),
           "fill_ms_avg": round(fms, 3), "fill_gcups": round(cells / (fms * 1e-3) / 1e9, 3), "steps": steps,
           "fill_launch": finfo}
    bpc = finfo["plane_bytes_per_cell"]
    ach = bpc * cells / (fms * 1e-3) / 1e9
    out["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                       "frac": round(ach / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_cell": bpc,
                       "note": "a single pair is latency-bound (the strip chain), not HBM-bound; DESIGN.md 6.6"}
    with open(os.path.join(ROOT, "tests", "golden", "large_digests.json")) as f:
        gold = {c["name"]: c for c in json.load(f)["cases"]}
    g = gold["brca2/local" if local else "covid_wuhan_usa/global"]
    res, _ = st.run(scores, local, True, plane_sums=True, max_cell=tracked)
    if ctx.fill_info() != finfo:
        raise RuntimeError(f"{which}: the parity pass took a different launch: {ctx.fill_info()} != {finfo}")
    sums = [int(x) for x in st.plane_sums()[0, 0]]
    r = res[0]
    ok = (r.score == g["score"] and [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps] == g["stats"]
          and r.n_steps == g["n_steps"] and alignment_sha256(st.steps(0)) == g["alignment_sha256"]
          and sums == [int(x) for x in g["plane_sums"]])
    if tracked:
        ok = ok and [r.max_cell_i, r.max_cell_j] == list(g["max_cell"]) and r.matches_at_max == g["matches_at_max"]
    if not ok:
        raise RuntimeError(f"{which}: result differs from tests/golden/large_digests.json")
    out["parity"] = {"bit_exact": True, "fields": "score, statistics, alignment sha256, I/D/S plane checksums"
                                                  + (", max cell, matches_at_max" if tracked else ""),
                     "source": "tests/golden/large_digests.json (oracle)"}
    return out


LOCAL_BATCH_PAIRS = 64   # tests/golden/make_golden.py LOCAL_RELATED


def local_batch_record(gx, ctx, steps: int):
    """A Smith-Waterman batch (BASELINE config 3's mode at config 2's size):
    the first 64 related 30k pairs (SURVEY 8(d) M1's variant, s2 = s1 with ~10 %
    substitutions and ~1 % indels, so every pair has a long local alignment)
    aligned locally (algo.rs:231-248 with the 0 floor, last-max start
    algo.rs:310-322), resident in HBM, score planes + traceback + labelled
    alignment per step -- the local twin fill (gx_fill_pk.hip LOCAL) when the
    host admits it.  `steps` timed passes, then one untimed pass whose every
    pair is compared with tests/golden/synthetic_related_local_L30000.json
    (score, statistics, alignment sha256, the three plane checksums)."""
    pairs = [related_pair(k, 30000) for k in range(LOCAL_BATCH_PAIRS)]
    scores = gx.Scores(*SCORES)
    ctx.trim()   # the headline batch's cached plane buffers (~175 GB) back to the device
    st = gx.StagedPairs(pairs, ctx=ctx)
    st.run(scores, True, True, steps=2)   # (both pipeline slots' buffers allocated before the timed steps)
    t0 = time.perf_counter()
    _, fms = st.run(scores, True, True, steps=steps)
    el = time.perf_counter() - t0
    finfo = ctx.fill_info()
    cells = sum(len(a) * len(b) for a, b in pairs)
    bpc = finfo["plane_bytes_per_cell"]
    ach = bpc * cells / (fms * 1e-3) / 1e9
    out = {"workload": f"{len(pairs)} related 30k pairs (SURVEY 8(d) M1 variant), local SW, scores {SCORES}, "
                       f"{plane_desc(bpc)}",
           "gcups": round(cells * steps / el / 1e9, 3), "ms_per_step": round(el / steps * 1e3, 3),
           "fill_ms_avg": round(fms, 3), "fill_gcups": round(cells / (fms * 1e-3) / 1e9, 3), "steps": steps,
           "fill_launch": finfo,
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(ach / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_cell": bpc,
                        "note": "plane bytes of the fill; the local twin fill is VALU-bound like the global one "
                                "(DESIGN.md 6.7)"}}
    path = os.path.join(ROOT, "tests", "golden", "synthetic_related_local_L30000.json")
    with open(path) as f:
        gold = {c["k"]: c for c in json.load(f)["cases"]}
    mine = {p: gold[p] for p in range(len(pairs))}
    # every timed pass (the launch that was measured), then two more passes
    # through the same pipeline with device plane checksums of each pass
    timed_checked = check_passes(st.pass_results(), mine, 0, 0, "local_batch timed")
    passes = 2
    st.run(scores, True, True, steps=passes, plane_sums=True)
    if ctx.fill_info() != finfo:
        raise RuntimeError(f"local_batch: the parity passes took a different launch than the timed call: "
                           f"{ctx.fill_info()} != {finfo}")
    check_passes(st.pass_results(), mine, 0, 0, "local_batch parity")
    sums = st.plane_sums()
    for p in range(len(pairs)):
        c = gold[p]
        if alignment_sha256(st.steps(p)) != c["alignment_sha256"]:
            raise RuntimeError(f"local_batch: pair {p} alignment differs from the oracle digest")
        for k in range(passes):
            if [int(x) for x in sums[k, p]] != [int(x) for x in c["plane_sums"]]:
                raise RuntimeError(f"local_batch: pass {k}, pair {p} score planes differ from the oracle's checksums")
    out["parity"] = {"pairs_checked": len(pairs), "bit_exact": True, "timed_passes_checked": timed_checked,
                     "parity_passes": passes, "fill_groups": finfo.get("groups"),
                     "fields": "every timed pass: score, statistics, length; two more passes through the same "
                               "launch: score, statistics, length, I/D/S plane checksums of each pass, "
                               "alignment sha256",
                     "source": os.path.relpath(path, ROOT)}
    return out


def allvsall_share(gx, rank: int, world: int):
    """BASELINE config 4: rank r's longest-processing-time share of the 45
    pairs i<j of the comparison_data genomes (files in name order, the same
    plan on every rank, so no scatter is needed for the bench; the product's
    gxamd.all_vs_all broadcasts the sequences instead).  Returns (pairs, all
    ranks' total cells)."""
    cont = gx.SequenceContainer()
    d = os.path.join(ROOT, "tests", "golden", "comparison_data")
    for f in sorted(os.listdir(d)):
        if f.endswith(".fasta"):
            cont.from_fasta(os.path.join(d, f))
    seqs = [x.sequence.encode() for x in cont.sequences]
    pairs = gx.all_pairs(len(seqs), with_self=False)
    w = [float(len(seqs[i])) * len(seqs[j]) for i, j in pairs]
    mine = gx.lpt_partition(w, world)[rank]
    return [(seqs[pairs[p][0]], seqs[pairs[p][1]]) for p in mine], int(sum(w)), [tuple(pairs[p]) for p in mine]


def allvsall_digests(ij):
    """{pair index on this rank: oracle digest} for the rank's all-vs-all
    pairs (tests/golden/allvsall_digests.json: score, statistics, alignment
    sha256, plane checksums per genome pair i, j), and the file's path."""
    path = os.path.join(ROOT, "tests", "golden", "allvsall_digests.json")
    with open(path) as f:
        d = json.load(f)
    by = {(c["i"], c["j"]): c for c in d["cases"]}
    return {p: by[tuple(x)] for p, x in enumerate(ij) if tuple(x) in by}, os.path.relpath(path, ROOT)


def plane_desc(bytes_per_cell) -> str:
    if bytes_per_cell == 1.5:
        return ("score planes (exact per-cell 12-bit codes of the differences S - I, D - I; I replayed along the "
                "row; 1.5 B/cell) + traceback")
    if bytes_per_cell == 3:
        return "score planes (exact per-cell byte differences, 3 B/cell) + traceback"
    return f"score planes (int32, {bytes_per_cell} B/cell) + traceback"


def rank_pairs(rank: int, pairs_per_rank: int, length: int, related: bool = False):
    """Weak-scaling shard: rank r aligns synthetic pairs r*P .. r*P+P-1 (no
    data-path collective; every rank generates its own inputs)."""
    gen = related_pair if related else synth_pair
    return [gen(rank * pairs_per_rank + p, length) for p in range(pairs_per_rank)]


# Inputs of a multi-GPU run above this many bytes are synthesised by each rank
# itself instead of scattered from rank 0 (config 5 at 1024 x 64k x 8 ranks
# would be 1 GB of sequences generated on one host thread)
SCATTER_MAX_BYTES = 1 << 30


def scatter_inputs(dist, rank: int, world: int, workload: str, P: int, L: int, related: bool, device: str):
    """North star: "RCCL over xGMI used only to scatter pairs and gather
    scores".  Rank 0 holds the job's inputs -- the 10 comparison_data genomes
    (config 4; read from FASTA on rank 0 only) or every rank's synthetic pairs
    -- and sends them to all ranks with gxamd._broadcast_bytes_list (three
    broadcasts: count, lengths, packed bytes; RCCL over xGMI for device =
    "cuda", gloo on CPU tensors in tests); each rank keeps its share: its LPT
    share of the 45 pairs, or pairs r*P .. r*P+P-1.  Untimed (before the
    timed region, which starts with the inputs resident in HBM).  Returns
    (pairs, all ranks' cells, (i, j) of each pair or None, info)."""
    import gxamd as gx
    t0 = time.perf_counter()
    ij = None
    if workload == "allvsall":
        seqs = None
        if rank == 0:
            cont = gx.SequenceContainer()
            d = os.path.join(ROOT, "tests", "golden", "comparison_data")
            for f in sorted(os.listdir(d)):
                if f.endswith(".fasta"):
                    cont.from_fasta(os.path.join(d, f))
            seqs = [x.sequence.encode() for x in cont.sequences]
        seqs = gx._broadcast_bytes_list(dist, seqs, device)
        allp = gx.all_pairs(len(seqs), with_self=False)
        w = [float(len(seqs[i])) * len(seqs[j]) for i, j in allp]
        mine = gx.lpt_partition(w, world)[rank]
        pairs = [(seqs[allp[p][0]], seqs[allp[p][1]]) for p in mine]
        ij = [tuple(allp[p]) for p in mine]
        n_total, nbytes = int(sum(w)), sum(len(x) for x in seqs)
        what = f"the {len(seqs)} comparison_data genomes; each rank keeps its LPT share of the {len(allp)} pairs"
    else:
        if 2 * L * P * world > SCATTER_MAX_BYTES:
            pairs = rank_pairs(rank, P, L, related)
            cells = sum(len(a) * len(b) for a, b in pairs)
            return pairs, cells * world, None, {"mode": "local synthesis", "bytes": 0, "ms": 0.0,
                                                "reason": f"inputs above {SCATTER_MAX_BYTES} B: each rank "
                                                          f"synthesises its own shard"}
        items = None
        if rank == 0:
            items = [x for r in range(world) for a, b in rank_pairs(r, P, L, related) for x in (a, b)]
        items = gx._broadcast_bytes_list(dist, items, device)
        mine = items[2 * P * rank: 2 * P * (rank + 1)]
        pairs = [(mine[2 * k], mine[2 * k + 1]) for k in range(P)]
        n_total = sum(len(items[2 * k]) * len(items[2 * k + 1]) for k in range(P * world))
        nbytes = sum(len(x) for x in items)
        what = f"{P * world} synthetic pairs; each rank keeps pairs r*{P} .. r*{P}+{P - 1}"
    if device == "cuda":
        import torch
        torch.cuda.synchronize()
    dist.barrier()
    ms = (time.perf_counter() - t0) * 1e3
    return pairs, n_total, ij, {"mode": "scatter from rank 0", "bytes": int(nbytes), "ms": round(ms, 3),
                                "collective": "3 broadcasts (count, lengths, packed bytes) from rank 0, "
                                              + ("RCCL over xGMI" if device == "cuda" else "gloo"),
                                "inputs": what}


def combine_over_ranks(dist, elapsed: float, rows, device: str):
    """Max-over-ranks time and all-gather of per-pair (score, steps, matches)
    rows.  `dist` is torch.distributed (RCCL on the GPU box, gloo in tests) or
    None for a single process."""
    if dist is None:
        return elapsed, [list(map(tuple, rows))]
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # ranks may hold different pair counts (all-vs-all LPT shares): pad to the
    # largest share with a count column so that all_gather sees equal shapes
    cnt = torch.tensor([len(rows)], dtype=torch.int64, device=device)
    cap = cnt.clone()
    dist.all_reduce(cap, op=dist.ReduceOp.MAX)
    mine = torch.zeros((int(cap.item()), 3), dtype=torch.int64, device=device)
    if rows:
        mine[: len(rows)] = torch.tensor(rows, dtype=torch.int64, device=device).reshape(-1, 3)
    gathered = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    counts = [torch.zeros_like(cnt) for _ in range(dist.get_world_size())]
    dist.all_gather(gathered, mine)
    dist.all_gather(counts, cnt)
    return float(t.item()), [[tuple(int(x) for x in r) for r in g.cpu().tolist()[: int(c.item())]]
                             for g, c in zip(gathered, counts)]


def alignment_sha256(steps) -> str:
    import hashlib
    h = hashlib.sha256()
    h.update(bytes(steps["choice"].astype(np.uint8)))
    h.update(steps["i"].astype("<u8").tobytes())
    h.update(steps["j"].astype("<u8").tobytes())
    return h.hexdigest()


def golden_digests(rank: int, P: int, L: int, related: bool = False):
    """{pair index on this rank: oracle digest} from tests/golden/synthetic(_related)_L{L}.json
    (score, statistics, alignment sha256, plane checksums), and the file's path."""
    path = os.path.join(ROOT, "tests", "golden", f"synthetic_related_L{L}.json" if related else f"synthetic_L{L}.json")
    if not os.path.exists(path):
        return {}, None
    with open(path) as f:
        golden = {c["k"]: c for c in json.load(f)["cases"]}
    return {p: golden[rank * P + p] for p in range(P) if rank * P + p in golden}, os.path.relpath(path, ROOT)


def check_passes(pass_res, mine, rank: int, P: int, what: str):
    """Every pass's per-pair results (gx_staged_pass_results) against the
    oracle digests: score, statistics, alignment length.  Raises on any
    difference; returns the number of passes checked."""
    for k, row in enumerate(pass_res):
        for p, c in mine.items():
            r = row[p]
            got = (r.score, [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps], r.n_steps)
            want = (c["score"], c["stats"], c["n_steps"])
            if got != want:
                raise RuntimeError(f"parity ({what}): pass {k}, pair {rank * P + p} differs from the oracle digest: "
                                   f"{got} != {want}")
    return len(pass_res)


def verify_against_golden(staged, ctx, scores, is_local, keep_planes, rank: int, P: int, L: int, related: bool,
                          timed_info: dict, passes: int = 2):
    """Parity of the benchmarked launch itself: `passes` more (untimed)
    pipelined passes of the same staged batch through the same launch as the
    timed call (fill_info must equal the timed call's: layout, band width,
    plane format, twin fill, fill groups -- the overlapped two-group pipeline
    when the timed call took it), with on-device plane checksums of every
    pass.  Every pair that has an oracle digest (tests/golden/synthetic_L{L}.json)
    must match it bit for bit: each pass's score, statistics, length and three
    plane checksums, and the last pass's alignment sha256.  Raises on any
    difference.  Returns (pairs checked, source, fill_info of the pass)."""
    mine, src = golden_digests(rank, P, L, related)
    if is_local or not mine:
        return 0, src, None
    return verify_passes(staged, ctx, scores, is_local, keep_planes, mine, src, rank, P, timed_info, passes)


def verify_passes(staged, ctx, scores, is_local, keep_planes, mine, src, rank: int, P: int, timed_info: dict,
                  passes: int):
    """verify_against_golden's check for digests `mine` ({pair index: digest})."""
    staged.run(scores, is_local, keep_planes, steps=passes, plane_sums=keep_planes)
    info = ctx.fill_info()
    if info != timed_info:
        raise RuntimeError(f"parity pass took a different launch than the timed call: {info} != {timed_info}")
    check_passes(staged.pass_results(), mine, rank, P, "parity pass")
    sums = staged.plane_sums() if keep_planes else None
    for p, c in mine.items():
        if alignment_sha256(staged.steps(p)) != c["alignment_sha256"]:
            raise RuntimeError(f"parity: pair {rank * P + p} alignment differs from the oracle digest")
        for k in range(passes if keep_planes else 0):
            if [int(x) for x in sums[k, p]] != [int(x) for x in c["plane_sums"]]:
                raise RuntimeError(f"parity: pass {k}, pair {rank * P + p} score planes differ from the oracle's "
                                   f"checksums")
    return len(mine), src, info


def simulate_world(args, gx, ctx):
    """Predicted N-GPU scaling from one GPU: every rank's shard of the
    workload (LPT share of the 45 all-vs-all pairs, or rank r's synthetic
    pairs) timed on this GPU in turn, K steps each after one warm-up, plus the
    whole workload at N = 1.  Since shards share nothing on the data path,
    the N-GPU step time is the slowest shard's; prints one JSON line.  Not a
    measurement of N GPUs (no xGMI, no concurrent HBM/power load)."""
    W = args.simulate_world
    scores = gx.Scores(*SCORES)
    strong = args.workload == "allvsall"

    checked = [0, 0]

    def shard(r, w):
        if strong:
            pr, _, ij = allvsall_share(gx, r, w)
            return pr, ij
        P = args.pairs_per_gpu or 8
        return rank_pairs(r, P, args.length), None

    def timed(pairs, ij):
        st = gx.StagedPairs(pairs, ctx=ctx)
        keep = args.planes if strong else not args.no_planes
        st.run(scores, False, keep)
        t0 = time.perf_counter()
        st.run(scores, False, keep, steps=args.steps)
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        if strong and not args.no_verify:
            # every timed pass of the shard against the oracle digests
            mine, _ = allvsall_digests(ij)
            if len(mine) != len(pairs):
                raise RuntimeError("all-vs-all pairs without an oracle digest")
            checked[0] += check_passes(st.pass_results(), mine, 0, 0, "simulated shard") * len(mine)
            checked[1] += len(mine)
        return ms

    per = []
    for r in range(W):
        pr, ij = shard(r, W)
        per.append({"rank": r, "pairs": len(pr), "cells": sum(len(a) * len(b) for a, b in pr),
                    "ms_per_step": round(timed(pr, ij), 3)})
        log(f"simulated rank {r}/{W}: {per[-1]}")
    full, ij1 = shard(0, 1)
    t1 = timed(full, ij1)
    cells1 = sum(len(a) * len(b) for a, b in full)
    tmax = max(p["ms_per_step"] for p in per)
    cells_w = sum(p["cells"] for p in per)
    eff = t1 / (W * tmax) if strong else per[0]["ms_per_step"] / tmax
    print(json.dumps({
        "metric": "GCUPS (DP cell updates/s) at 30k×30k NW, 1/2/4/8 MI355X; % HBM roofline",
        "simulated_world": W, "scaling": "strong" if strong else "weak",
        "workload": "all-vs-all of the 10 comparison_data genomes (45 pairs i<j), LPT shares" if strong else
                    f"synthetic {args.length}x{args.length} pairs, {per[0]['pairs']} per rank",
        "per_rank": per, "n1": {"pairs": len(full), "ms_per_step": round(t1, 3),
                                "gcups": round(cells1 / t1 / 1e6, 3)},
        "predicted": {"ms_per_step": tmax, "gcups": round(cells_w / tmax / 1e6, 3),
                      "efficiency": round(eff, 4),
                      "basis": "each rank's shard timed alone on one MI355X; N-GPU step = slowest shard "
                               "(no data-path collective)"},
        "parity": ({"pair_passes_checked": checked[0], "pairs_checked": checked[1], "bit_exact": True,
                    "fields": "score, statistics, alignment length of every pair, every timed pass",
                    "source": "tests/golden/allvsall_digests.json (oracle)"} if strong and checked[1] else None),
        "steps": args.steps}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs-per-gpu", type=int,
                    default=int(os.environ["GX_BENCH_PAIRS"]) if "GX_BENCH_PAIRS" in os.environ else None,
                    help="default: as many as fill ~220 GB with score planes (80 compact / 20 int32 at 30k)")
    ap.add_argument("--length", type=int, default=30000)
    ap.add_argument("--local", action="store_true", help="Smith-Waterman mode (default: global NW)")
    ap.add_argument("--no-planes", action="store_true", help="score+traceback only (not the headline)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="cores of the all-cores CPU baseline (the GPU box's CPU share is 16; 1 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the parity pass against the oracle digests")
    ap.add_argument("--workload", choices=["synthetic", "allvsall", "covid", "brca2"], default="synthetic",
                    help="allvsall: BASELINE config 4, the 45 pairs i<j of the 10 comparison_data genomes, "
                         "LPT-sharded over the ranks (traceback-only fill unless --planes); covid: config 2, "
                         "Covid_Wuhan x Covid_USA-CA4 global; brca2: config 3, the Human x Mouse BRCA2 cds pair "
                         "local (one copy per rank)")
    ap.add_argument("--planes", action="store_true", help="allvsall: also write the score planes")
    ap.add_argument("--related", action="store_true",
                    help="synthetic: the SURVEY 8(d) M1 related variant (s2 = s1 with ~10%% substitutions and ~1%% "
                         "indels; a long non-trivial traceback)")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="1 GPU only: time every rank's shard of an N-GPU run in turn and print the predicted "
                         "N-GPU step time and scaling efficiency (not the headline line)")
    ap.add_argument("--config-steps", type=int, default=5,
                    help="synthetic, 1 GPU: also time BASELINE configs 2 and 3 (the single-pair align calls) "
                         "with this many steps (0: skip)")
    ap.add_argument("--single-pair-steps", type=int, default=5,
                    help="also time BASELINE config 2's shape alone (one pair, latency), 1 GPU only; 0 = skip")
    ap.add_argument("--int32-steps", type=int, default=2,
                    help="also time the batch with int32 score planes (12 B/cell, HBM roofline), 1 GPU only; 0 = skip")
    ap.add_argument("--no-plane-steps", type=int, default=2,
                    help="also time the batch without plane stores (compute ceiling), 1 GPU only; 0 = skip")
    ap.add_argument("--local-batch-steps", type=int, default=3,
                    help="synthetic, 1 GPU: also time a local (SW) batch of 32 related 30k pairs (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend="nccl")       # RCCL over xGMI
        dist = tdist

    import gxamd as gx
    ctx = gx.Context(gx.device_for_rank(local_rank))
    if args.simulate_world > 1 and world == 1:
        simulate_world(args, gx, ctx)
        ctx.close()
        return
    P, L = args.pairs_per_gpu, args.length
    scores = gx.Scores(*SCORES)
    if P is None:
        pb = 0 if args.no_planes else gx.plane_bytes_per_cell(scores, args.local)
        P = max(1, min(MAX_DEFAULT_PAIRS, int(PLANE_BUDGET // (max(pb, 3) * L * (L + 64)))))
    ij = None
    scatter = None
    if world > 1 and args.workload in ("allvsall", "synthetic"):
        # the inputs come from rank 0 (north_star: RCCL scatters the pairs)
        pairs, n_total, ij, scatter = scatter_inputs(dist, rank, world, args.workload, P, L, args.related, "cuda")
        if args.workload == "allvsall":
            P = len(pairs)
            keep_planes = args.planes
            args.single_pair_steps = 0
        else:
            keep_planes = not args.no_planes
    elif args.workload == "allvsall":
        pairs, n_total, ij = allvsall_share(gx, rank, world)
        P = len(pairs)
        keep_planes = args.planes
        args.single_pair_steps = 0
    elif args.workload in ("covid", "brca2"):
        pairs = [fasta_pair(gx, args.workload)]
        P = 1
        args.local = args.workload == "brca2"
        keep_planes = not args.no_planes
        args.single_pair_steps = 0
    else:
        pairs = rank_pairs(rank, P, L, args.related)
        keep_planes = not args.no_planes
    staged = gx.StagedPairs(pairs, ctx=ctx)             # inputs resident in HBM
    cells_rank = sum(len(a) * len(b) for a, b in pairs)

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        # (two pipelined passes: the same launches, streams and pooled buffers
        # as the timed call, so it allocates nothing)
        staged.run(scores, args.local, keep_planes, steps=2)
    barrier()
    fill_ms = []
    tb_us = []
    t0 = time.perf_counter()
    # the K steps in one library call: pipelined one step deep (step k's host
    # labelling overlaps step k+1's fill); every step's fill, traceback and
    # labelling completes inside the timed region
    res, fms = staged.run(scores, args.local, keep_planes, steps=args.steps)
    fill_ms.append(fms)
    tb_us.append(res[0].retrace_us)
    barrier()
    elapsed = time.perf_counter() - t0
    finfo = ctx.fill_info()
    # every timed pass's results against the oracle digests (after the timed region)
    timed_passes = staged.pass_results()
    if len(timed_passes) != args.steps:
        raise RuntimeError(f"{len(timed_passes)} pass records for {args.steps} timed steps")
    timed_checked = 0
    if args.workload == "synthetic" and not args.local and not args.no_verify:
        mine, _ = golden_digests(rank, P, L, args.related)
        if mine:
            timed_checked = check_passes(timed_passes, mine, rank, P, "timed passes")
    elif args.workload == "allvsall" and not args.local and not args.no_verify:
        mine, _ = allvsall_digests(ij)
        if len(mine) != P:
            raise RuntimeError(f"{P - len(mine)} of this rank's all-vs-all pairs have no oracle digest")
        timed_checked = check_passes(timed_passes, mine, rank, P, "timed passes")
    else:   # no digests: every pass must at least agree with the last
        for k, row in enumerate(timed_passes):
            if [(r.score, r.n_steps, r.matches) for r in row] != [(r.score, r.n_steps, r.matches) for r in res]:
                raise RuntimeError(f"timed pass {k} differs from the last pass")
    bytes_per_cell = finfo["plane_bytes_per_cell"]

    # max over ranks (time) and gather of per-pair results, over RCCL
    elapsed, _gathered = combine_over_ranks(dist, elapsed, [[r.score, r.n_steps, r.matches] for r in res], "cuda")
    total_cells = cells_rank * world
    if args.workload == "allvsall":
        total_cells = n_total
    ms_per_step = elapsed / args.steps * 1e3
    gcups = total_cells * args.steps / elapsed / 1e9
    avg_fill_ms = float(np.mean(fill_ms))
    mode_s = f"{'local SW' if args.local else 'global NW'}, scores {SCORES}, " \
             f"{plane_desc(bytes_per_cell) if keep_planes else 'traceback only (no planes)'}"
    if args.workload == "allvsall":
        workload = f"all-vs-all of the 10 comparison_data genomes (45 pairs i<j, 29,644-30,123 nt), " \
                   f"LPT-sharded over {world} GPU(s), {mode_s}"
    elif args.workload == "covid":
        workload = f"Covid_Wuhan x Covid_USA-CA4 ({len(pairs[0][0])}x{len(pairs[0][1])}), one pair per GPU, {mode_s}"
    elif args.workload == "brca2":
        workload = f"Human x Mouse BRCA2 cds ({len(pairs[0][0])}x{len(pairs[0][1])}), one pair per GPU, {mode_s}"
    else:
        workload = (f"synthetic related {L}-nt DNA pairs (SplitMix64 s1, s2 = s1 with ~10% substitutions and ~1% "
                    f"indels), {P} per GPU, {mode_s}") if args.related else \
                   f"synthetic {L}x{L} DNA pairs (SplitMix64), {P} per GPU, {mode_s}"
    fill_bytes = bytes_per_cell * cells_rank
    achieved = fill_bytes / (avg_fill_ms * 1e-3) / 1e9
    twin = bool(finfo.get("twin"))
    kname = "gx::fill_pk_kernel (twin fill)" if twin else "gx::fill_kernel"
    traffic, traffic_src = load_traffic(workload, twin)
    valu = load_valu(workload, twin)
    hbm = {"bound": "hbm", "achieved": round(achieved, 1) if keep_planes else None,
           "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "frac": round(achieved / PEAK_HBM_GBS, 4) if keep_planes else None,
           "frac_of_measured_copy_ceiling": round(achieved / MEASURED_HBM_GBS, 4) if keep_planes else None,
           "traffic": traffic, "traffic_source": traffic_src,
           "kernel": kname, "fill_ms_avg": round(avg_fill_ms, 3),
           "algorithmic_bytes_per_cell": bytes_per_cell,
           "algorithmic_bytes_per_launch": fill_bytes}
    if finfo.get("groups", 1) == 2:
        # the overlapped batch: a pass is two concurrent fill
        # launches; "launch" figures are per pass, the time is the fill
        # pipeline's per pass, the PMC profile the same kernel run one launch a pass
        hbm["fill_launches_per_pass"] = 2
    if valu is not None and keep_planes and bytes_per_cell in (1.5, 3):
        # compact planes / twin codes: the fill is bound by VALU issue, not HBM -- lane-ops
        # per launch (VALU/cell x cells, SQ_INSTS_VALU profile) over the live
        # fill time, against the probe-measured ceiling at the fill's mix
        ach = valu["valu_insts_per_cell"] * cells_rank / (avg_fill_ms * 1e-3) / 1e12
        roofline = {"bound": "valu", "achieved": round(ach, 3), "peak": valu["peak_tops"], "unit": "TOP/s",
                    "frac": round(ach / valu["peak_tops"], 4), "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": kname, "fill_ms_avg": round(avg_fill_ms, 3),
                    "algorithmic_ops_per_cell": valu["valu_insts_per_cell"],
                    "algorithmic_ops_per_launch": round(valu["valu_insts_per_cell"] * cells_rank),
                    "ops": "VALU lane-operations (wave64 VALU instructions x 64; a packed 16-bit twin "
                           "instruction updates two pairs' cells)",
                    "peak_basis": f"1024 SIMDs x 64 lanes x {valu['clock_ghz']} GHz / {valu['cpi_fill_mix']} cycles "
                                  f"per wave64 VALU instruction at the fill's mix (tools/valu_probe.hip)",
                    "source": valu["source"], "hbm": hbm}
        if finfo.get("groups", 1) == 2:
            roofline["fill_launches_per_pass"] = 2
    else:
        roofline = hbm

    out = {
        "metric": "GCUPS (DP cell updates/s) at 30k×30k NW, 1/2/4/8 MI355X; % HBM roofline",
        "value": round(gcups, 3),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.workload == "allvsall" else "weak",
        "vs_baseline": None,
        "dtype": "int16x2 (two pairs per register, exact, relative to int32 block bases)" if twin else "int32",
        "data": "synthetic" if args.workload == "synthetic" else "reference FASTA data (tests/golden)",
        "config": {"workload": workload, "pairs_per_gpu": P, "seq_len": L if args.workload == "synthetic" else None,
                   "cells_per_step": total_cells, "parallelism": f"pairs sharded over {world} GPU(s)"},
        "roofline": roofline,
        "fill_launch": finfo,
        "valu": valu,
        "fill_gcups_per_gpu": round(cells_rank / (avg_fill_ms * 1e-3) / 1e9, 3),
        "traceback_us_pair0": int(np.mean(tb_us)),
    }
    if scatter is not None:
        out["scatter"] = scatter
    if args.workload == "synthetic" and not args.no_verify:
        vpasses = 2 if args.steps >= 2 else 1
        checked, src, vinfo = verify_against_golden(staged, ctx, scores, args.local, keep_planes, rank, P, L,
                                                    args.related, finfo, vpasses)
        if dist is not None:
            import torch
            t = torch.tensor([checked], dtype=torch.int64, device="cuda")
            dist.all_reduce(t)
            checked = int(t.item())
        out["parity"] = {"pairs_checked": checked, "pairs_total": P * world, "bit_exact": True,
                         "fields": "score, statistics, alignment sha256" + (", I/D/S plane checksums" if keep_planes
                                                                            else ""),
                         "source": src,
                         "timed_passes_checked": timed_checked,
                         "timed_pass_fields": "score, statistics, alignment length of every pair with a digest, "
                                              "every timed pass",
                         "pass": f"{vpasses} extra untimed pipelined passes through the timed call's launch "
                                 f"(fill_info identical: layout {finfo['layout']}, band width {finfo['band_waves']}, "
                                 f"{finfo['plane_bytes_per_cell']} B/cell, twin {finfo['twin']}, "
                                 f"{finfo['groups']} fill group(s) per pass"
                                 + (", the overlapped two-group pipeline" if finfo.get('groups') == 2 else "")
                                 + "); plane checksums of every pass, alignment sha256 of the last"}
    if args.workload == "allvsall" and not args.local and not args.no_verify:
        # every pair of this rank's share against the oracle digests of the 45
        # genome pairs (tests/golden/allvsall_digests.json); gathered over ranks
        vpasses = 2 if args.steps >= 2 else 1
        mine, src = allvsall_digests(ij)
        checked, src, _ = verify_passes(staged, ctx, scores, False, keep_planes, mine, src, rank, P, finfo, vpasses)
        pairs_total = P
        if dist is not None:
            import torch
            t = torch.tensor([checked, P], dtype=torch.int64, device="cuda")
            dist.all_reduce(t)
            checked, pairs_total = int(t[0].item()), int(t[1].item())
        out["parity"] = {"pairs_checked": checked, "pairs_total": pairs_total, "bit_exact": True,
                         "fields": "score, statistics, alignment sha256" + (", I/D/S plane checksums" if keep_planes
                                                                            else ""),
                         "source": src, "timed_passes_checked": timed_checked,
                         "timed_pass_fields": "score, statistics, alignment length of every pair, every timed pass",
                         "pass": f"{vpasses} extra untimed pipelined passes through the timed call's launch "
                                 f"(fill_info identical); plane checksums of every pass, alignment sha256 of the last"}
    if world == 1 and keep_planes and bytes_per_cell == 1.5 and args.no_plane_steps > 0:
        # the same batch with the per-pair byte planes (3 B/cell, the table format)
        os.environ["GX_PLANES_W16"] = "0"
        try:
            staged.run(scores, args.local, True)
            _, fms3 = staged.run(scores, args.local, True, steps=args.no_plane_steps)
            fi3 = ctx.fill_info()
        finally:
            del os.environ["GX_PLANES_W16"]
        out["byte_planes"] = {"fill_ms_avg": round(fms3, 3),
                              "fill_gcups_per_gpu": round(cells_rank / (fms3 * 1e-3) / 1e9, 3),
                              "steps": args.no_plane_steps, "fill_launch": fi3}
    if world == 1 and keep_planes and bytes_per_cell in (1.5, 3) and args.int32_steps > 0:
        # the same batch with int32 score planes (12 B/cell, the HBM-bound
        # format of SURVEY 8(d)); batches beyond the free HBM run in chunks
        os.environ["GX_PLANES32"] = "1"
        try:
            staged.run(scores, args.local, True)
            t2 = time.perf_counter()
            _, fms2 = staged.run(scores, args.local, True, steps=args.int32_steps)
            e2 = time.perf_counter() - t2
            fi2 = ctx.fill_info()
        finally:
            del os.environ["GX_PLANES32"]
        a2 = 12 * cells_rank / (fms2 * 1e-3) / 1e9
        out["int32_planes"] = {"gcups": round(cells_rank * args.int32_steps / e2 / 1e9, 3),
                               "ms_per_step": round(e2 / args.int32_steps * 1e3, 3),
                               "fill_ms_avg": round(fms2, 3), "steps": args.int32_steps,
                               "chunks": fi2["chunks"], "fill_launch": fi2,
                               "roofline": {"bound": "hbm", "achieved": round(a2, 1), "peak": PEAK_HBM_GBS,
                                            "unit": "GB/s", "frac": round(a2 / PEAK_HBM_GBS, 4),
                                            "frac_of_measured_copy_ceiling": round(a2 / MEASURED_HBM_GBS, 4),
                                            "algorithmic_bytes_per_cell": 12}}
    if world == 1 and keep_planes and args.no_plane_steps > 0:
        # the same batch without plane stores: the fill's compute ceiling
        staged.run(scores, args.local, False)
        _, fms0 = staged.run(scores, args.local, False, steps=args.no_plane_steps)
        out["no_plane_fill"] = {"fill_ms_avg": round(fms0, 3),
                                "fill_gcups_per_gpu": round(cells_rank / (fms0 * 1e-3) / 1e9, 3),
                                "planes_fill_frac": round(fms0 / avg_fill_ms, 4), "steps": args.no_plane_steps}
    if world == 1 and args.single_pair_steps > 0 and P > 1:
        # one 30k x 30k pair per step (configs[1]'s shape): the latency view of the same kernel
        one = gx.StagedPairs(pairs[:1], ctx=ctx)
        one.run(scores, args.local, keep_planes)
        t1 = time.perf_counter()
        _, fms1 = one.run(scores, args.local, keep_planes, steps=args.single_pair_steps)
        e1 = time.perf_counter() - t1
        f1 = [fms1]
        c1 = len(pairs[0][0]) * len(pairs[0][1])
        out["single_pair"] = {"gcups": round(c1 * args.single_pair_steps / e1 / 1e9, 3),
                              "ms_per_step": round(e1 / args.single_pair_steps * 1e3, 3),
                              "fill_ms_avg": round(float(np.mean(f1)), 3), "steps": args.single_pair_steps}
        del one
    if world == 1 and args.workload == "synthetic" and args.config_steps > 0:
        # BASELINE configs 2 and 3, the drop-in single-pair align calls, timed here
        out["config2"] = config_record(gx, ctx, "covid", args.config_steps)
        out["config3"] = config_record(gx, ctx, "brca2", args.config_steps)
        # the same calls with alignment_table's max cell + matches_at_max kept
        out["config2_tracked"] = config_record(gx, ctx, "covid", args.config_steps, tracked=True)
        out["config3_tracked"] = config_record(gx, ctx, "brca2", args.config_steps, tracked=True)
    if world == 1 and args.workload == "synthetic" and args.local_batch_steps > 0 and not args.local:
        out["local_batch"] = local_batch_record(gx, ctx, args.local_batch_steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if len(pairs[0][1]) > 40000:
            # the reference layout needs (n+1)(m+1) x 48 B (197 GB at 64k)
            out["cpu_baseline"] = {"value": None, "unit": "GCUPS", "cores": 1, "kind": "port",
                                   "sample": "N/A: the reference-layout table of one pair exceeds host memory "
                                             "(SURVEY.md 8(d))"}
        else:
            out["cpu_baseline"] = cpu_baseline(pairs[0][0], pairs[0][1], args.cpu_seconds, args.local)
            if args.cpu_threads > 1:
                out["cpu_baseline_all_cores"] = cpu_baseline_parallel(pairs, args.cpu_threads, args.cpu_seconds / 2,
                                                                      args.local)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
