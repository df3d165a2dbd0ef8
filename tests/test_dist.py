"""CPU, world_size 2 over gloo: the multi-GPU bench path.  Each rank owns a
disjoint set of whole tracks (weak scaling, no data-path collective); the
only collective is the max-over-ranks step clock.  Also checks that two
ranks encoding their shards produce exactly what one process encoding the
union produces (tracks are independent), using the oracle on CPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = bench.shard(world, rank, 3)
        import hashlib
        import oracle_port
        import signals
        digests = {}
        for t in ids:
            pcm = signals.make("tone", 4096 + 37 * t, 2, 16, seed=t)
            data, _ = oracle_port.encode(pcm, 2, 16, 44100, **oracle_port.PRESETS["8"])
            digests[t] = hashlib.sha256(data).hexdigest()
        elapsed = 1.0 + rank            # rank-specific clock
        mx = bench.reduce_max(torch, dist, elapsed, torch.device("cpu"))
        q.put((rank, ids, digests, mx))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_and_clock():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    all_ids = [t for _, ids, _, _ in res for t in ids]
    assert sorted(all_ids) == list(range(6)) and len(set(all_ids)) == 6
    assert all(mx == 2.0 for _, _, _, mx in res)
    # union of the shards == single-process encode of every track
    import hashlib
    import oracle_port
    import signals
    for _, _, digests, _ in res:
        for t, h in digests.items():
            pcm = signals.make("tone", 4096 + 37 * t, 2, 16, seed=t)
            data, _ = oracle_port.encode(pcm, 2, 16, 44100, **oracle_port.PRESETS["8"])
            assert hashlib.sha256(data).hexdigest() == h


def _rg_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_port
        import signals
        # this rank's tracks of one album: histograms summed locally, then
        # the album reduce of bench.py over the ranks
        local = np.zeros(12000, dtype=np.uint64)
        peak = 0.0
        for t in bench.shard(world, rank, 2):
            pcm = signals.make("tone", 30000 + 1000 * t, 2, 16, seed=t)
            A, pk = oracle_port.rg_title(pcm, 2, 16, 44100)
            local += A
            peak = max(peak, pk)
        hist = torch.tensor(local.astype(np.int64), dtype=torch.int32)
        pkt = torch.tensor([peak], dtype=torch.float64)
        bench.album_reduce(dist, world, hist, pkt)
        q.put((rank, hist.numpy().astype(np.uint32), float(pkt.item())))
    finally:
        dist.destroy_process_group()


def test_two_rank_album_reduce_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle_port
    import signals
    B = np.zeros(12000, dtype=np.uint64)
    peak = 0.0
    for t in range(4):
        A, pk = oracle_port.rg_title(signals.make("tone", 30000 + 1000 * t, 2, 16, seed=t),
                                     2, 16, 44100)
        B += A
        peak = max(peak, pk)
    for _, hist, pk in res:
        assert np.array_equal(hist, B.astype(np.uint32))
        assert pk == peak
        assert oracle_port.rg_gain(hist) == oracle_port.rg_gain(B.astype(np.uint32))


@pytest.mark.parametrize("scaling,tracks,want_total", [("weak", 3, 6), ("strong", 5, 5)])
def test_bench_spawns_ranks(scaling, tracks, want_total):
    """`python bench.py --gpus 2` spawns its own ranks (no torchrun) and the
    rank-0 line reports n_gpus, the scaling mode and the whole-job track
    count; --selftest swaps the GPU step for the CPU oracle (gloo)"""
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, bench.__file__, "--selftest", "--gpus", "2",
                        "--tracks", str(tracks), "--frames", "1", "--steps", "1",
                        "--warmup", "0", "--scaling", scaling],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == scaling and d["selftest"] is True
    assert d["tracks_total"] == want_total


def test_strong_shards_partition_the_batch():
    for world in (1, 2, 3, 8):
        ids = [t for r in range(world) for t in bench.shard(world, r, 1024, "strong")]
        assert ids == list(range(1024))
