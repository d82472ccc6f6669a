"""CPU, world_size 2 over gloo: bench.py's multi-GPU orchestration -- the
weak-scaling pair shards are disjoint and deterministic, the timing is the
max over ranks and the per-pair results are all-gathered in rank order
(pairs shard with no data-path collective)."""
import os
import socket
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench as b
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pairs = b.rank_pairs(rank, 3, 256)
    rows = [[len(x), len(y), 10 * rank + k] for k, (x, y) in enumerate(pairs)]
    t, gathered = b.combine_over_ranks(dist, 1.0 + rank, rows, "cpu")
    q.put((rank, t, gathered, [x for x, _ in pairs]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_shard_and_reduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted(q.get(timeout=180) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    expected = [[(256, 256, 0), (256, 256, 1), (256, 256, 2)], [(256, 256, 10), (256, 256, 11), (256, 256, 12)]]
    for rank, t, gathered, firsts in out:
        assert t == 2.0                              # max over ranks
        assert gathered == expected                  # rank-ordered all-gather, same on every rank
        assert firsts == [bench.synth_pair(3 * rank + k, 256)[0] for k in range(3)]
    # the two ranks' inputs are different pairs
    assert not set(out[0][3]) & set(out[1][3])


def _scatter_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench as b
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for workload, P, L in (("synthetic", 3, 300), ("allvsall", 0, 0)):
        pairs, n_total, ij, info = b.scatter_inputs(dist, rank, world, workload, P, L, False, "cpu")
        # the rest of bench.py's path with a stand-in for the GPU aligner:
        # per-pair rows, max-over-ranks time, rank-ordered gather
        rows = [[len(x) * 7 + len(y), len(x) + len(y), sum(x) % 1000] for x, y in pairs]
        t, gathered = b.combine_over_ranks(dist, 1.0 + rank, rows, "cpu")
        out[workload] = (pairs, n_total, ij, info, t, gathered)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_inputs_scattered_from_rank0():
    """bench.py's multi-GPU path (world 2, gloo on CPU tensors; RCCL over
    xGMI on the GPU box): rank 0 builds the inputs and broadcasts them
    (scatter_inputs), each rank keeps exactly the shard the local path would
    have built -- synthetic pairs r*P .. r*P+P-1, the LPT share of the 45
    comparison-genome pairs -- then the per-pair rows are gathered and the
    time is the max over ranks.  The line's scatter record counts the bytes."""
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
    import gxamd as gx
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted((q.get(timeout=240) for _ in range(2)), key=lambda x: x[0])
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, o in out:
        pairs, n_total, ij, info, t, gathered = o["synthetic"]
        assert pairs == bench.rank_pairs(rank, 3, 300)
        assert n_total == 2 * 3 * 300 * 300 and ij is None and t == 2.0
        assert info["mode"] == "scatter from rank 0" and info["bytes"] == 2 * 3 * 2 * 300 and "gloo" in info["collective"]
        want = [[(len(x) * 7 + len(y), len(x) + len(y), sum(x) % 1000) for x, y in bench.rank_pairs(r, 3, 300)]
                for r in range(2)]
        assert gathered == want
        pairs, n_total, ij, info, t, gathered = o["allvsall"]
        local_pairs, local_total, local_ij = bench.allvsall_share(gx, rank, 2)
        assert pairs == local_pairs and n_total == local_total and ij == local_ij
        assert info["bytes"] == sum(len(a) for a in {x for p in bench.allvsall_share(gx, 0, 1)[0] for x in p})
    # the two ranks' all-vs-all shares are disjoint and cover the 45 pairs
    both = out[0][1]["allvsall"][2] + out[1][1]["allvsall"][2]
    assert sorted(both) == sorted(gx.all_pairs(10, with_self=False))


def test_single_process_combine_is_identity():
    t, g = bench.combine_over_ranks(None, 3.5, [[1, 2, 3]], "cpu")
    assert t == 3.5 and g == [[(1, 2, 3)]]


def test_synthetic_inputs_follow_survey_seeds():
    # SplitMix64, seed 0x5EED0001 (s1) / 0x5EED0002 (s2), base = "ACGT"[x >> 62]
    s1, s2 = bench.synth_pair(0, 64)
    assert set(s1) <= set(b"ACGT") and set(s2) <= set(b"ACGT") and s1 != s2
    x = (0x5EED0001 + 0x9E3779B97F4A7C15) & (2 ** 64 - 1)
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & (2 ** 64 - 1)
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & (2 ** 64 - 1)
    x ^= x >> 31
    assert s1[0] == b"ACGT"[x >> 62]


# ---- all-vs-all (BASELINE config 4): broadcast scatter, LPT shares, gather ----

def _fake_align(pairs, scores, is_local):
    """Deterministic stand-in for the GPU aligner (plumbing test only)."""
    return [[len(a) * 1000 + len(b), len(a), len(b), 0, 0, len(a) + len(b)] for a, b in pairs]


def _avsa_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import gxamd as gx
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seqs = [gx.Sequence(f"s{k}", "ACGT"[k % 4] * (50 + 37 * k)) for k in range(7)]
    # only rank 0 holds the sequences: the others receive them through the broadcast
    cont = gx.SequenceContainer(seqs if rank == 0 else [])
    calls = []

    def fn(pairs, scores, is_local):
        calls.append(len(pairs))
        return _fake_align(pairs, scores, is_local)

    res = gx.all_vs_all(cont, gx.Scores(), dist=dist, device="cpu", align_fn=fn)
    q.put((rank, res["pairs"], res["records"], res["lengths"], calls, res["names"]))
    dist.barrier()
    dist.destroy_process_group()


def test_all_vs_all_two_ranks_equals_single_process():
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
    import gxamd as gx
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_avsa_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted(q.get(timeout=180) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    seqs = [gx.Sequence(f"s{k}", "ACGT"[k % 4] * (50 + 37 * k)) for k in range(7)]
    single = gx.all_vs_all(gx.SequenceContainer(seqs), gx.Scores(), align_fn=_fake_align)
    assert len(single["pairs"]) == 28
    for rank, pairs, records, lengths, calls, names in out:
        assert pairs == single["pairs"] and records == single["records"]
        assert lengths == [50 + 37 * k for k in range(7)]
        assert names == [f"s{k}" for k in range(7)]     # broadcast with the sequences
    # the two shares are disjoint and cover every pair; LPT balances n*m
    shares = gx.lpt_partition([float(a * b) for a, b in
                               ((single["lengths"][i], single["lengths"][j]) for i, j in single["pairs"])], 2)
    assert sorted(shares[0] + shares[1]) == list(range(28))
    assert [o[4] for o in out] == [[len(shares[0])], [len(shares[1])]]
    loads = [sum(single["lengths"][single["pairs"][p][0]] * single["lengths"][single["pairs"][p][1]] for p in s)
             for s in shares]
    assert max(loads) / min(loads) < 1.1


def test_similarity_tsv_layout():
    sys.path.insert(0, os.path.join(ROOT, "genomics-rs_amd"))
    import gxamd as gx
    res = gx.all_vs_all(gx.SequenceContainer([gx.Sequence("a", "AC"), gx.Sequence("b", "ACG")]), gx.Scores(),
                        align_fn=_fake_align)
    # row r, column c filled for c <= r (main.rs:253-264, 343-359)
    assert gx.similarity_tsv(res) == "\t0\t1\t\n0\t2002\t0\t\n1\t2003\t3003\t\n"
    assert gx.similarity_tsv(res, "matches", blank_header=True) == " \t0\t1\t\n0\t2\t0\t\n1\t2\t3\t\n"


def _ragged_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench as b
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = [[rank, k, 7] for k in range(2 - rank)]     # rank 0: 2 pairs, rank 1: 1 pair
    q.put((rank,) + tuple(b.combine_over_ranks(dist, 0.5, rows, "cpu")))
    dist.barrier()
    dist.destroy_process_group()


def test_combine_over_ranks_ragged_shares():
    """All-vs-all LPT shares differ in size between ranks (45 pairs over 8 GPUs)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ragged_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = sorted(q.get(timeout=180) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, t, gathered in out:
        assert t == 0.5 and gathered == [[(0, 0, 7), (0, 1, 7)], [(1, 0, 7)]]


def test_related_pair_generators_agree():
    """bench.py and tests/golden/make_golden.py generate the same related pairs
    (SURVEY 8(d) M1 variant), whose digests the bench checks itself against."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden
    for k in (0, 5):
        a, b = bench.related_pair(k, 3000)
        assert (a, b) == make_golden.related_pair(k, 3000)
        assert a == bench.synth_pair(k, 3000)[0] and a != b and abs(len(a) - len(b)) < 300
