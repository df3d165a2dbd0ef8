"""GPU: the pipelined device API (atg_flac_encode_device_async / _wait).

Batches enqueued with encode_device_async keep their MD5 chains split in two
parts one batch apart (md5.hip launch_track_md5 part 0 / part 1, engine.hip
batch_end), so a batch's STREAMINFO MD5 is only complete once a later batch
was enqueued or the batch was waited.  These tests keep several batches with
different PCM buffers and mixed track shapes in flight -- tracks shorter than
two MD5 blocks, odd PCM offsets (the unaligned finishing path), uneven
lengths, a synchronous encode in between -- and require every waited image
to equal the CPU port's byte for byte.  They also pin the slot contract of
include/atgpu.h: a fourth unwaited enqueue fails, results survive until
waited."""
import numpy as np
import pytest

import oracle_port
import signals

pytestmark = pytest.mark.gpu

FLAC8 = oracle_port.PRESETS["8"]


def _batch(seed, shapes):
    """shapes: list of (leading gap frames, track frames) -> (pcm int16,
    tracks, per-track int32 pcm)"""
    rng = np.random.default_rng(seed)
    parts, tracks, per, pos = [], [], [], 0
    for gap, n in shapes:
        if gap:
            parts.append(rng.integers(-99, 99, 2 * gap).astype(np.int16))
            pos += gap
        kind = ["tone", "noise", "chirp", "sine"][len(per) % 4]
        p = signals.make(kind, n, 2, 16, seed=int(rng.integers(1 << 30))) if n else \
            np.zeros(0, np.int32)
        parts.append(p.astype(np.int16))
        tracks.append((pos, n))
        per.append(p.astype(np.int32))
        pos += n
    return np.concatenate(parts), tracks, per


SHAPES = [
    [(0, 4096 * 3 + 5), (1, 7), (0, 31), (3, 4096 * 2), (0, 1), (5, 9000), (0, 0), (2, 300)],
    [(1, 4096 * 4), (0, 4096 * 4), (1, 100), (0, 15), (1, 16), (0, 17), (7, 12345)],
    [(0, 64), (0, 4096), (1, 4097), (0, 4096 * 5 + 4095)],
]


def _dev(torch, arr):
    return torch.from_numpy(arr.copy()).to("cuda")


def _check(eng, torch, d_out, res, per, label):
    host = d_out.cpu().numpy()
    for t, (r, p) in enumerate(zip(res, per)):
        want, _ = oracle_port.encode(p, 2, 16, 44100, **FLAC8)
        got = host[r.out_offset:r.out_offset + r.bytes].tobytes()
        assert got == want, "%s track %d (%d frames): GPU %d B vs port %d B" % (
            label, t, len(p) // 2, len(got), len(want))


def test_async_batches_split_md5_match_port(gpu_engine):
    import torch
    from audiotools import _atgpu
    eng = gpu_engine
    opts = _atgpu.make_options(**FLAC8)
    batches = [_batch(100 + i, s) for i, s in enumerate(SHAPES)]
    dev = []
    for pcm, tracks, per in batches:
        d_pcm = _dev(torch, pcm)
        _, cap = eng.bounds(opts, tracks, 2, 16)
        dev.append((d_pcm, torch.empty(cap, dtype=torch.uint8, device="cuda"), cap))
    torch.cuda.synchronize()
    # three batches in flight, waited oldest first
    tickets = []
    for (d_pcm, d_out, cap), (_, tracks, _) in zip(dev, batches):
        tickets.append(eng.encode_device_async(opts, d_pcm.data_ptr(), _atgpu.PCM_S16, tracks,
                                               2, 16, 44100, d_out.data_ptr(), cap))
    for i, t in enumerate(tickets):
        res = eng.wait(t)
        _check(eng, torch, dev[i][1], res, batches[i][2], "pipelined batch %d" % i)
    # waited in reverse order, with a synchronous encode in between
    t0 = eng.encode_device_async(opts, dev[0][0].data_ptr(), _atgpu.PCM_S16, batches[0][1],
                                 2, 16, 44100, dev[0][1].data_ptr(), dev[0][2])
    t1 = eng.encode_device_async(opts, dev[1][0].data_ptr(), _atgpu.PCM_S16, batches[1][1],
                                 2, 16, 44100, dev[1][1].data_ptr(), dev[1][2])
    res2 = eng.encode_device(opts, dev[2][0].data_ptr(), _atgpu.PCM_S16, batches[2][1],
                             2, 16, 44100, dev[2][1].data_ptr(), dev[2][2])
    _check(eng, torch, dev[2][1], res2, batches[2][2], "sync between async")
    res1 = eng.wait(t1)
    res0 = eng.wait(t0)
    _check(eng, torch, dev[1][1], res1, batches[1][2], "async waited first")
    _check(eng, torch, dev[0][1], res0, batches[0][2], "async waited last")


def test_fourth_enqueue_refused_results_survive(gpu_engine):
    import torch
    from audiotools import _atgpu
    eng = gpu_engine
    eng.set_inflight(3)  # the contract at a fixed depth (the default is automatic)
    opts = _atgpu.make_options(**FLAC8)
    pcm, tracks, per = _batch(7, [(0, 4096 * 2 + 11), (1, 333)])
    d_pcm = _dev(torch, pcm)
    _, cap = eng.bounds(opts, tracks, 2, 16)
    outs = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in range(4)]
    torch.cuda.synchronize()
    ts = [eng.encode_device_async(opts, d_pcm.data_ptr(), _atgpu.PCM_S16, tracks, 2, 16,
                                  44100, outs[k].data_ptr(), cap) for k in range(3)]
    with pytest.raises(_atgpu.ATGError) as e:
        eng.encode_device_async(opts, d_pcm.data_ptr(), _atgpu.PCM_S16, tracks, 2, 16, 44100,
                                outs[3].data_ptr(), cap)
    assert e.value.status == _atgpu.ATG_ERR_INVALID
    with pytest.raises(_atgpu.ATGError):   # the host pipeline refuses too
        eng.encode(opts, pcm, tracks, 2, 16, 44100)
    # the first ticket's results were not lost
    _check(eng, torch, outs[0], eng.wait(ts[0]), per, "ticket 0")
    t3 = eng.encode_device_async(opts, d_pcm.data_ptr(), _atgpu.PCM_S16, tracks, 2, 16, 44100,
                                 outs[3].data_ptr(), cap)
    for k, t in ((1, ts[1]), (2, ts[2]), (3, t3)):
        _check(eng, torch, outs[k], eng.wait(t), per, "ticket %d" % k)
    with pytest.raises(_atgpu.ATGError):   # waited twice after its slot was reused
        eng.wait(ts[0])
    eng.set_inflight(0)


@pytest.mark.parametrize("n_tracks,frames,want", [(4, 64, 32), (1024, 8, 12), (3, 1, 12)])
def test_automatic_depth(n_tracks, frames, want):
    """the default (automatic) depth: the first pipelined batch on an idle
    engine sets it from its longest track's MD5 chain against its kernel
    time (engine.hip auto_depth) -- 4 one-MiB tracks (a narrow rank batch)
    32, 1024 short tracks 12, a tiny batch 12; the depth's contract holds
    (D unwaited enqueues, the next refused), every batch's images are the
    same bytes (the first batch's checked against the port), and a host
    job sets the rotation back to 3"""
    import torch
    from audiotools import _atgpu
    eng = _atgpu.Engine(0)
    opts = _atgpu.make_options(**FLAC8)
    pcm, tracks, per = _batch(900 + n_tracks, [(0, 4096 * frames)] * n_tracks)
    d_pcm = _dev(torch, pcm)
    _, cap = eng.bounds(opts, tracks, 2, 16)
    outs = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in range(want)]
    torch.cuda.synchronize()
    table = _atgpu.TrackTable(tracks)

    def enq(k):
        return eng.encode_device_async(opts, d_pcm.data_ptr(), _atgpu.PCM_S16, table, 2, 16,
                                       44100, outs[k].data_ptr(), cap)

    ts = [enq(0)]
    assert eng.inflight() == want
    ts += [enq(k) for k in range(1, want)]
    with pytest.raises(_atgpu.ATGError):
        enq(0)
    res = [eng.wait(t) for t in ts]
    first = outs[0].cpu().numpy()
    imgs = [first[r.out_offset:r.out_offset + r.bytes].tobytes() for r in res[0]]
    for t in range(min(n_tracks, 4)):
        want_img, _ = oracle_port.encode(per[t], 2, 16, 44100, **FLAC8)
        assert imgs[t] == want_img, "track %d" % t
    for k in range(1, want):
        host = outs[k].cpu().numpy()
        assert all(host[r.out_offset:r.out_offset + r.bytes].tobytes() == imgs[t]
                   for t, r in enumerate(res[k])), "batch %d" % k
    eng.encode(opts, pcm, tracks, 2, 16, 44100)
    assert eng.inflight() == 3
    eng.close()


def test_async_batches_new_frame_lengths_fresh_engine():
    """a fresh engine (empty window table), three batches enqueued back to
    back whose tracks end in frame lengths no earlier batch had: every
    batch uploads new Tukey windows on its own slot stream, and the table
    grows (the buffer is replaced) while earlier LPC kernels may still run
    (engine.hip prepare_windows, ev_win).  Each image equals the port's"""
    import torch
    from audiotools import _atgpu
    eng = _atgpu.Engine(0)
    opts = _atgpu.make_options(**FLAC8)
    shapes = [[(0, 4096 * 2 + 1000 + 37 * k + 100 * b) for k in range(6)] for b in range(3)]
    batches = [_batch(300 + i, s) for i, s in enumerate(shapes)]
    dev = []
    for pcm, tracks, per in batches:
        _, cap = eng.bounds(opts, tracks, 2, 16)
        dev.append((_dev(torch, pcm), torch.empty(cap, dtype=torch.uint8, device="cuda"), cap))
    torch.cuda.synchronize()
    tickets = [eng.encode_device_async(opts, d_pcm.data_ptr(), _atgpu.PCM_S16, tracks, 2, 16,
                                       44100, d_out.data_ptr(), cap)
               for (d_pcm, d_out, cap), (_, tracks, _) in zip(dev, batches)]
    for i, t in enumerate(tickets):
        _check(eng, torch, dev[i][1], eng.wait(t), batches[i][2], "fresh-engine batch %d" % i)


def _batch32(seed, shapes, bps):
    """int32 containers of `bps`-bit samples (the rolled s32 path)"""
    rng = np.random.default_rng(seed)
    parts, tracks, per, pos = [], [], [], 0
    for gap, n in shapes:
        if gap:
            parts.append(rng.integers(-99, 99, 2 * gap).astype(np.int32))
            pos += gap
        p = signals.make(["noise", "tone", "chirp"][len(per) % 3], n, 2, bps,
                         seed=int(rng.integers(1 << 30))) if n else np.zeros(0, np.int32)
        parts.append(p.astype(np.int32))
        tracks.append((pos, n))
        per.append(p.astype(np.int32))
        pos += n
    return np.concatenate(parts), tracks, per


@pytest.mark.parametrize("depth", [4, 8, 16, 32])
def test_rolled_md5_many_in_flight_match_port(depth):
    """atg_engine_set_inflight(depth >= 4): every batch's MD5 chain runs in
    depth - 2 slices on the engine's MD5 stream, all batches' slices in one
    launch per enqueue (md5.hip k_track_md5_roll).  Batches of 16-bit and
    24-bit (int32 container) PCM, mixed shapes incl. unaligned and
    sub-block tracks, more batches than slots, waited oldest first and out
    of order: every image equals the port's; a (depth + 1)-th unwaited
    enqueue is refused; the default depth comes back"""
    import torch
    from audiotools import _atgpu
    eng = _atgpu.Engine(0)
    eng.set_inflight(depth)
    opts = _atgpu.make_options(**FLAC8)
    jobs = []
    for i in range(depth + 3):
        if i % 3 == 2:
            pcm, tracks, per = _batch32(500 + i, SHAPES[i % 3], 24)
            fmt, bps = _atgpu.PCM_S32, 24
        else:
            pcm, tracks, per = _batch(500 + i, SHAPES[i % 3])
            fmt, bps = _atgpu.PCM_S16, 16
        _, cap = eng.bounds(opts, tracks, 2, bps)
        jobs.append((_dev(torch, pcm), torch.empty(cap, dtype=torch.uint8, device="cuda"), cap,
                     tracks, per, fmt, bps))
    torch.cuda.synchronize()

    def check(j, res, label):
        d_pcm, d_out, cap, tracks, per, fmt, bps = j
        host = d_out.cpu().numpy()
        for t, (r, p) in enumerate(zip(res, per)):
            want, _ = oracle_port.encode(p, 2, bps, 44100, **FLAC8)
            got = host[r.out_offset:r.out_offset + r.bytes].tobytes()
            assert got == want, "%s track %d" % (label, t)

    def enq(j):
        d_pcm, d_out, cap, tracks, per, fmt, bps = j
        return eng.encode_device_async(opts, d_pcm.data_ptr(), fmt, tracks, 2, bps, 44100,
                                       d_out.data_ptr(), cap)

    pending = []
    for i, j in enumerate(jobs):
        pending.append((i, enq(j)))
        if len(pending) == depth:
            k, t = pending.pop(0)
            check(jobs[k], eng.wait(t), "rolled batch %d" % k)
    # the slot contract at this depth
    with pytest.raises(_atgpu.ATGError):
        while True:
            pending.append((0, enq(jobs[0])))
    # drain newest first: waits that cannot count on later enqueues
    for k, t in reversed(pending):
        check(jobs[k], eng.wait(t), "rolled batch %d (drain)" % k)
    eng.set_inflight(3)
    ts = [enq(jobs[k]) for k in range(3)]
    for k, t in enumerate(ts):
        check(jobs[k], eng.wait(t), "depth 3 again, batch %d" % k)
    for bad in (2, 33):  # the rotation is 3..32 batches
        with pytest.raises(_atgpu.ATGError):
            eng.set_inflight(bad)
    eng.close()
