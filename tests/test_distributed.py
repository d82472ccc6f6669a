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
