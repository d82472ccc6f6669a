"""Generate the committed golden fixtures from the CPU oracle.

    python tests/golden/make_golden.py [--large]

oracle_vectors.json : full outputs (alignment vectors) for small inputs --
                      config 1 (s1.fasta x s2.fasta), the multi-record
                      test_data files, both modes, both scoring configs.
large_digests.json  : (--large) digests for the big pairs: BRCA2 (config 3)
                      and Covid_Wuhan x Covid_USA-CA4 (config 2): score,
                      stats, start, max_cell, matches_at_max, n_steps, the
                      sha256 of the alignment vector and weighted checksums
                      of the three score planes.

The oracle (oracle/gx_oracle.c) is pinned by the reference's own vectors
(tests/test_oracle.py).  The FASTA inputs are the reference's data files,
copied under tests/golden/fasta and tests/golden/comparison_data.
"""
import argparse
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as o  # noqa: E402

CONFIG = (1, -2, -1, -5)
TEST = (1, -2, -2, -5)


def recs(path):
    with open(path, "rb") as f:
        return o.fasta_parse(f.read())


def alignment_digest(choices, si, sj):
    h = hashlib.sha256()
    h.update(bytes(choices.astype("uint8")))
    h.update(si.astype("<u8").tobytes())
    h.update(sj.astype("<u8").tobytes())
    return h.hexdigest()


def small_cases():
    cases = []
    fa = os.path.join(HERE, "fasta")
    pairs = [("config1_s1_s2", recs(os.path.join(fa, "s1.fasta"))[0][1], recs(os.path.join(fa, "s2.fasta"))[0][1])]
    for name in ("test1", "test2_short", "test3_short", "test4", "Opsin1_colorblindness_gene"):
        r = recs(os.path.join(fa, name + ".fasta"))
        pairs.append((name, r[0][1], r[1][1]))
    # s3 x s4 and simple x repeat (single-record files paired, as config 1)
    pairs.append(("s3_s4", recs(os.path.join(fa, "s3.fasta"))[0][1], recs(os.path.join(fa, "s4.fasta"))[0][1]))
    pairs.append(("simple_repeat", recs(os.path.join(fa, "simple.fasta"))[0][1],
                  recs(os.path.join(fa, "repeat.fasta"))[0][1]))
    for name, a, b in pairs:
        for loc in (False, True):
            for sc in (CONFIG, TEST):
                r = o.align(a, b, sc, is_local=loc)
                assert r.status == 0
                cases.append({
                    "name": f"{name}/{'local' if loc else 'global'}/{sc}",
                    "s1": a.decode("latin-1"), "s2": b.decode("latin-1"), "scores": list(sc), "is_local": loc,
                    "score": r.score, "stats": [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps],
                    "start": list(r.start), "max_cell": list(r.max_cell), "matches_at_max": r.matches_at_max,
                    "alignment": [list(x) for x in r.alignment()],
                })
    return cases


def large_cases():
    fa = os.path.join(HERE, "fasta")
    cd = os.path.join(HERE, "comparison_data")
    brca = recs(os.path.join(fa, "Human-Mouse-BRCA2-cds.fasta"))
    wuhan = recs(os.path.join(cd, "Covid_Wuhan.fasta"))[0][1]
    usa = recs(os.path.join(cd, "Covid_USA-CA4.fasta"))[0][1]
    jobs = [("brca2", brca[0][1], brca[1][1], True), ("brca2", brca[0][1], brca[1][1], False),
            ("covid_wuhan_usa", wuhan, usa, False), ("covid_wuhan_usa", wuhan, usa, True)]
    out = []
    for name, a, b, loc in jobs:
        r = o.align_lean(a, b, CONFIG, is_local=loc)
        assert r.status == 0
        out.append({
            "name": f"{name}/{'local' if loc else 'global'}", "n": len(a), "m": len(b), "is_local": loc,
            "scores": list(CONFIG), "score": r.score,
            "stats": [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps],
            "start": list(r.start), "max_cell": list(r.max_cell), "matches_at_max": r.matches_at_max,
            "n_steps": int(len(r.choices)), "alignment_sha256": alignment_digest(r.choices, r.steps_i, r.steps_j),
            "plane_sums": [str(x) for x in r.extra["plane_sums"]],
        })
        print(out[-1]["name"], out[-1]["score"], out[-1]["n_steps"], flush=True)
    return out


def _allvsall_job(job):
    i, j, a, b = job
    r = o.align_lean(a, b, CONFIG, is_local=False)
    assert r.status == 0
    return {"i": i, "j": j, "n": len(a), "m": len(b), "score": r.score,
            "stats": [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps],
            "n_steps": int(len(r.choices)), "alignment_sha256": alignment_digest(r.choices, r.steps_i, r.steps_j),
            "plane_sums": [int(x) for x in r.extra["plane_sums"]]}


def allvsall_cases(workers: int):
    """BASELINE config 4: every pair i <= j of the comparison_data records (files
    in name order), global NW under config.toml scores."""
    from multiprocessing import Pool
    cd = os.path.join(HERE, "comparison_data")
    names, seqs = [], []
    for f in sorted(os.listdir(cd)):
        if f.endswith(".fasta"):
            for name, seq in recs(os.path.join(cd, f)):
                names.append(name.decode("utf-8") if isinstance(name, bytes) else name)
                seqs.append(seq)
    jobs = [(i, j, seqs[i], seqs[j]) for j in range(len(seqs)) for i in range(j + 1)]
    jobs.sort(key=lambda x: -len(x[2]) * len(x[3]))
    with Pool(workers) as pool:
        out = pool.map(_allvsall_job, jobs, chunksize=1)
    out.sort(key=lambda c: (c["j"], c["i"]))
    return names, out


def splitmix64_bases(seed: int, length: int) -> bytes:
    """SURVEY.md 8(d) synthetic DNA (the same generator as bench.py): bytes
    i.i.d. over ACGT from SplitMix64, base = "ACGT"[x >> 62]."""
    import numpy as np
    with np.errstate(over="ignore"):
        k = np.arange(1, length + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return np.frombuffer(b"ACGT", np.uint8)[(z >> np.uint64(62)).astype(np.int64)].tobytes()


def synth_pair(k: int, length: int):
    """Synthetic pair k of length L (bench.py synth_pair: seeds 0x5EED0001/2 + 0x10000 k)."""
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


# Synthetic batches digested by --synthetic: BASELINE configs[1]'s shape (the
# bench's own 30k pairs, rank 0's 80 at N = 1) and configs[4] (1024 x 1k, and
# samples of the 4k / 16k / 64k batches).
SYNTH_SETS = {30000: 80, 1024: 1024, 4096: 256, 16384: 256, 65536: 1}


def _synth_job(job):
    length, k = job[:2]
    a, b = (related_pair if len(job) > 2 and job[2] else synth_pair)(k, length)
    r = o.align_lean(a, b, CONFIG, is_local=len(job) > 3 and job[3])
    assert r.status == 0
    return length, {"k": k, "n": len(a), "m": len(b), "score": r.score,
                    "stats": [r.matches, r.mismatches, r.gap_extensions, r.opening_gaps],
                    "n_steps": int(len(r.choices)), "alignment_sha256": alignment_digest(r.choices, r.steps_i, r.steps_j),
                    "plane_sums": [str(x) for x in r.extra["plane_sums"]]}


# The local (Smith-Waterman) batch of bench.py's `local_batch` record: the
# first LOCAL_RELATED related 30k pairs (a long local alignment each).
LOCAL_RELATED = 64


# Local related pairs of 64k (round-4 verdict item 7: the local twin fill on
# values beyond 2^15): the first LOCAL_RELATED_64K related_pair(k, 65536).
LOCAL_RELATED_64K = 16


def synthetic_cases(workers: int, lengths, related: bool = False, local: bool = False):
    """Oracle digests of the synthetic batches (related: the SURVEY 8(d) M1
    "related" variant, s2 derived from s1, 80 pairs at 30k; local: its first
    LOCAL_RELATED pairs aligned locally, LOCAL_RELATED_64K at 64k)."""
    from multiprocessing import Pool
    count = lambda L: (LOCAL_RELATED_64K if L == 65536 else LOCAL_RELATED) if local else SYNTH_SETS[L]
    jobs = [(L, k, related, local) for L in lengths for k in range(count(L))]
    jobs.sort(key=lambda x: -x[0])
    out = {L: [] for L in lengths}
    with Pool(workers) as pool:
        for n_done, (L, rec) in enumerate(pool.imap_unordered(_synth_job, jobs, chunksize=1), 1):
            out[L].append(rec)
            if L >= 16384 or n_done % 128 == 0:
                print(f"synthetic L={L} k={rec['k']} done ({n_done}/{len(jobs)})", flush=True)
    for L in lengths:
        out[L].sort(key=lambda c: c["k"])
        name = f"synthetic_related{'_local' if local else ''}_L{L}.json" if related else f"synthetic_L{L}.json"
        src = (f"tests/golden/make_golden.py --related-local{' --length 65536' if L == 65536 else ''} "
               f"(oracle_align_lean, LOCAL, config.toml scores; pair k = related_pair(k, {L}), k < {count(L)})") if local else ("tests/golden/make_golden.py --related (oracle_align_lean, global, config.toml scores; pair k = "
               "related_pair(k): s1 of synthetic pair k, s2 derived with seed 0x5EED0003 + 0x10000 k)") if related else \
              ("tests/golden/make_golden.py --synthetic (oracle_align_lean, global, config.toml "
               "scores; pair k = splitmix64 seeds 0x5EED0001/2 + 0x10000 k, bench.py synth_pair)")
        with open(os.path.join(HERE, name), "w") as f:
            json.dump({"_source": src,
                       "length": L, "scores": list(CONFIG), "cases": out[L]}, f, indent=0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true")
    ap.add_argument("--allvsall", action="store_true")
    ap.add_argument("--synthetic", type=str, default=None,
                    help="comma-separated lengths of SYNTH_SETS to digest, or 'all'")
    ap.add_argument("--related", action="store_true", help="the related 30k batch (SURVEY 8(d) M1 variant)")
    ap.add_argument("--related-local", action="store_true",
                    help="local digests of the first 64 related 30k pairs (bench.py local_batch), or 16 at --length 65536")
    ap.add_argument("--length", type=int, default=30000, help="--related-local: pair length (30000 or 65536)")
    ap.add_argument("--workers", type=int, default=7)
    args = ap.parse_args()
    o.build()
    if args.related_local:
        synthetic_cases(args.workers, [args.length], related=True, local=True)
        return
    if args.related:
        synthetic_cases(args.workers, [30000], related=True)
        return
    if args.synthetic:
        lengths = sorted(SYNTH_SETS) if args.synthetic == "all" else [int(x) for x in args.synthetic.split(",")]
        synthetic_cases(args.workers, lengths)
        return
    if args.allvsall:
        names, cases = allvsall_cases(args.workers)
        with open(os.path.join(HERE, "allvsall_digests.json"), "w") as f:
            json.dump({"_source": "tests/golden/make_golden.py --allvsall (oracle_align_lean, global, "
                                  "config.toml scores)", "names": names, "scores": list(CONFIG),
                       "cases": cases}, f, indent=1)
        return
    with open(os.path.join(HERE, "oracle_vectors.json"), "w") as f:
        json.dump({"_source": "tests/golden/make_golden.py (oracle restatement, pinned by "
                              "tests/test_alignment.rs vectors)", "cases": small_cases()}, f)
    if args.large:
        with open(os.path.join(HERE, "large_digests.json"), "w") as f:
            json.dump({"_source": "tests/golden/make_golden.py --large (oracle_align_lean)",
                       "cases": large_cases()}, f, indent=1)


if __name__ == "__main__":
    main()
