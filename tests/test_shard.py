"""The multi-GPU product path on CPU: batches sharded by track
over the node's GPUs, and ReplayGain's album reduce.

* shard_ranges: contiguous groups balanced by frames;
* replaygain.album_scan over 3 mocked devices: each shard's GPU call is
  replaced by the CPU oracle (oracle/replaygain_port.c), so the sharding,
  the mono/stereo buffer layout and the SUM / MAX album reduce are checked
  against the title-by-title oracle album;
* replaygain.album_allreduce at world size 2 over gloo: the histogram SUM
  and peak MAX every rank gets equal the single-process album."""
import os
import socket
import threading

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_port
import signals
from audiotools import _atgpu, replaygain


def test_shard_ranges():
    assert _atgpu.shard_ranges([1] * 10, 3) == [(0, 3), (3, 6), (6, 10)]
    assert _atgpu.shard_ranges([5, 1, 1, 1, 1, 1], 2) == [(0, 1), (1, 6)]
    assert _atgpu.shard_ranges([1, 1], 8) == [(0, 1), (1, 2)]
    assert _atgpu.shard_ranges([], 4) == []
    for n in range(1, 9):
        w = list(np.random.default_rng(n).integers(1, 1000, 37))
        r = _atgpu.shard_ranges(w, n)
        assert len(r) == n and r[0][0] == 0 and r[-1][1] == 37
        assert all(a[1] == b[0] and a[0] < a[1] for a, b in zip(r, r[1:] + [(37, 38)]))
        # no shard more than one track's weight above the even share
        assert max(sum(w[a:b]) for a, b in r) <= sum(w) / n + max(w)


def test_batch_devices_env(monkeypatch):
    for var in ("ATG_DEVICE", "LOCAL_RANK", "ATG_SHARD_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("ATG_DEVICE_COUNT", "4")
    assert _atgpu.batch_devices() == [0, 1, 2, 3]
    monkeypatch.setenv("LOCAL_RANK", "2")
    assert _atgpu.batch_devices() == [2]
    monkeypatch.setenv("ATG_SHARD_DEVICES", "0,0")
    assert _atgpu.batch_devices() == [0, 0]


def _titles():
    out = []
    for k in range(7):
        ch = 1 if k % 3 == 1 else 2
        n = 44100 // 4 + 911 * k
        x = signals.make("tone", n, ch, 16, seed=40 + k).astype(np.int32)
        sizes = [4096] * (n // 4096) + ([n % 4096] if n % 4096 else [])
        # the reads' arrays, as replaygain._read_title keeps them
        parts = np.split(x, np.cumsum(sizes)[:-1] * ch) if k % 2 else x
        out.append((parts, sizes, ch, 16))
    out.insert(3, None)  # a title that read nothing
    return out


class _FakeDevice(object):
    """device memory and replaygain_device's contract on the host: the GPU
    call is the CPU oracle (oracle/replaygain_port.c) per title"""

    def __init__(self):
        self.mem, self.next = {}, 1 << 40
        self.lock = threading.Lock()  # the shards run on threads of their own

    def _find(self, p):
        with self.lock:
            base = max(b for b in self.mem if b <= p)
            return self.mem[base], p - base

    def device_alloc(self, n):
        with self.lock:
            p = self.next
            self.mem[p] = np.zeros(max(4, int(n)), dtype=np.uint8)
            self.next += 1 << 36
            return p

    def device_free(self, p):
        with self.lock:
            del self.mem[p]

    def copy_to_device(self, d, src):
        buf, o = self._find(d)
        b = np.ascontiguousarray(src).view(np.uint8).reshape(-1)
        buf[o:o + len(b)] = b

    def copy_to_host(self, dst, d):
        buf, o = self._find(d)
        dst.view(np.uint8).reshape(-1)[:] = buf[o:o + dst.nbytes]
        return dst

    def replaygain_device(self, d_pcm, tracks, n_albums=0, d_album_hist=None):
        class R(object):
            pass
        buf, o = self._find(d_pcm)
        x = buf[o:].view(np.int32)
        res, hist, peak = [], np.zeros(12000, dtype=np.uint64), 0.0
        for t in tracks:
            a = t.pcm_offset * t.channels
            A, pk = oracle_port.rg_title(x[a:a + t.pcm_frames * t.channels], t.channels,
                                         t.bits_per_sample, t.sample_rate)
            r = R()
            r.title_gain, r.title_peak = oracle_port.rg_gain(A), pk
            res.append(r)
            hist += A
            peak = max(peak, pk)
        self.copy_to_device(d_album_hist, hist.astype(np.uint32))
        return res, [peak]


def test_album_scan_sharded_matches_oracle(monkeypatch):
    dev = _FakeDevice()
    monkeypatch.setattr(_atgpu, "replaygain_device", dev.replaygain_device)
    monkeypatch.setattr(_atgpu, "batch_devices", lambda: [0, 1, 2])
    monkeypatch.setattr(_atgpu, "shard_object", lambda kind, i, d: dev)
    # small staging buffers: the titles are uploaded over several chunks
    monkeypatch.setattr(_atgpu, "staging", lambda key, n: np.zeros(n, dtype=np.uint8))
    monkeypatch.setattr(replaygain, "STAGE_BYTES", 1)
    titles = _titles()
    gains, hist, peak = replaygain.album_scan(titles, 44100)
    want_hist, want_peak = np.zeros(12000, dtype=np.uint64), 0.0
    for t, g in zip(titles, gains):
        if t is None:
            assert g == (0.0, 0.0)
            continue
        A, pk = oracle_port.rg_title(np.concatenate(replaygain._parts(t[0])), t[2], 16, 44100)
        assert g == (oracle_port.rg_gain(A), pk)
        want_hist += A
        want_peak = max(want_peak, pk)
    assert np.array_equal(hist, want_hist) and peak == want_peak


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        titles = [t for t in _titles() if t is not None][rank::world]
        hist, peak = np.zeros(12000, dtype=np.uint64), 0.0
        for x, _, ch, bps in titles:
            A, pk = oracle_port.rg_title(np.concatenate(replaygain._parts(x)), ch, bps, 44100)
            hist += A
            peak = max(peak, pk)
        h, p = replaygain.album_allreduce(hist, peak)
        th = torch.as_tensor(hist.astype(np.int32))
        tp = torch.tensor([peak], dtype=torch.float64)
        replaygain.album_allreduce(th, tp)  # in place, the tensor form
        q.put((rank, h, p, th.numpy().astype(np.uint32), float(tp.item())))
    finally:
        dist.destroy_process_group()


def test_album_allreduce_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_hist, want_peak = np.zeros(12000, dtype=np.uint64), 0.0
    for x, _, ch, bps in [t for t in _titles() if t is not None]:
        A, pk = oracle_port.rg_title(np.concatenate(replaygain._parts(x)), ch, bps, 44100)
        want_hist += A
        want_peak = max(want_peak, pk)
    for _, h, p, th, tp in got:
        assert np.array_equal(h, want_hist) and p == want_peak
        assert np.array_equal(th, want_hist.astype(np.uint32)) and tp == want_peak
    assert oracle_port.rg_gain(got[0][1].astype(np.uint32)) == \
        oracle_port.rg_gain(want_hist.astype(np.uint32))
