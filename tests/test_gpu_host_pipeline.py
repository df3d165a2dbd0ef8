"""GPU: the chunked, overlapped host-memory encode (atg_flac_encode_host):
tracks are cut into chunks of ~chunk_bytes of PCM
(atg_engine_set_host_chunk_bytes), staged through
pinned buffers, and chunk c's upload / encode / chunk c-1's download
overlap.  Every image and frame offset must equal the CPU port's, whatever
the chunking, track order in memory or explicit frame sizes."""
import os

import numpy as np
import pytest

import oracle_port

pytestmark = pytest.mark.gpu


DEFAULT_CHUNK = 512 << 20


@pytest.fixture
def chunked():
    """the session engine; its chunk size is restored afterwards"""
    from audiotools import _atgpu
    eng = _atgpu.engine()
    yield eng, _atgpu
    eng.set_host_chunk_bytes(DEFAULT_CHUNK)


def _tracks(rng, n, lo, hi):
    lens = [int(rng.integers(lo, hi)) for _ in range(n)]
    parts = []
    for k, m in enumerate(lens):
        t = np.arange(m)
        x = (6000 * np.sin(2 * np.pi * (180 + 40 * k) * t / 44100)).astype(np.int64)
        x = np.stack([x, (x * 3) // 4 + rng.integers(-300, 300, m)], 1)
        parts.append(np.clip(x, -32768, 32767).astype(np.int16).reshape(-1))
    return lens, parts


@pytest.mark.parametrize("chunk_mb", ["1", "3", "4096"])
def test_chunked_host_encode_matches_port(chunk_mb, chunked):
    eng, A = chunked
    eng.set_host_chunk_bytes(int(chunk_mb) << 20)
    rng = np.random.default_rng(int(chunk_mb))
    lens, parts = _tracks(rng, 19, 20000, 160000)
    # tracks stored out of order, with gaps between them
    order = rng.permutation(len(parts))
    buf, where, pos = [], {}, 0
    for k in order:
        buf.append(np.zeros(2 * int(rng.integers(0, 50)), np.int16))
        pos += len(buf[-1]) // 2
        where[int(k)] = pos
        buf.append(parts[k])
        pos += lens[k]
    pcm = np.concatenate(buf)
    tracks = [(where[k], lens[k]) for k in range(len(parts))]
    opts = A.make_options(**oracle_port.PRESETS["8"])
    out, res, offs, fpcm = eng.encode(opts, pcm, tracks, 2, 16, 44100)
    for k in range(len(parts)):
        want, woffs = oracle_port.encode(parts[k].astype(np.int32), 2, 16, 44100,
                                         **oracle_port.PRESETS["8"])
        r = res[k]
        assert bytes(out[r.out_offset:r.out_offset + r.bytes]) == want, k
        got = [(int(offs[r.first_frame + i]), int(fpcm[r.first_frame + i]))
               for i in range(r.n_frames)]
        assert got == woffs, k


def test_chunked_host_encode_explicit_frame_sizes(chunked):
    eng, A = chunked
    eng.set_host_chunk_bytes(1 << 20)
    rng = np.random.default_rng(5)
    lens, parts = _tracks(rng, 6, 150000, 200000)
    pcm = np.concatenate(parts)
    tracks, base = [], 0
    for k, m in enumerate(lens):
        sizes = []
        left = m
        while left:
            s = min(left, int(rng.choice([1152, 4096, 777])))
            sizes.append(s)
            left -= s
        tracks.append((base, m, sizes) if k % 2 else (base, m))
        base += m
    opts = A.make_options(**oracle_port.PRESETS["8"])
    out, res, offs, fpcm = eng.encode(opts, pcm, tracks, 2, 16, 44100)
    eng.set_host_chunk_bytes(4096 << 20)
    out1, res1, offs1, fpcm1 = eng.encode(opts, pcm, tracks, 2, 16, 44100)
    assert np.array_equal(offs, offs1) and np.array_equal(fpcm, fpcm1)
    for k in range(len(parts)):
        r, r1 = res[k], res1[k]
        img = bytes(out[r.out_offset:r.out_offset + r.bytes])
        # chunked == one chunk, byte for byte
        assert img == bytes(out1[r1.out_offset:r1.out_offset + r1.bytes]), k
        got = [(int(offs[r.first_frame + i]), int(fpcm[r.first_frame + i]))
               for i in range(r.n_frames)]
        # the port's encode of the same reads (explicit frame sizes,
        # flac.c:244-274, 412-518), byte for byte
        want, woffs = oracle_port.encode(parts[k].astype(np.int32), 2, 16, 44100,
                                         frame_sizes=tracks[k][2] if k % 2 else None,
                                         **oracle_port.PRESETS["8"])
        assert img == want, k
        assert got == woffs, k
        if k % 2:
            assert [n for _, n in got] == tracks[k][2]


@pytest.mark.parametrize("pin_in,pin_out", [(True, True), (True, False), (False, True)])
def test_pinned_buffers_direct_dma(pin_in, pin_out, chunked):
    """page-locked PCM / output (atg_host_alloc) move by DMA without the
    staging copies; images are packed back to back in `out` and equal the
    port's, whatever the chunking (1 MB chunks: the three-stage ring wraps)"""
    eng, A = chunked
    eng.set_host_chunk_bytes(1 << 20)
    rng = np.random.default_rng(11 + 2 * pin_in + pin_out)
    lens, parts = _tracks(rng, 23, 1000, 120000)
    host = np.concatenate(parts)
    pcm = A.pinned_empty(host.shape, np.int16) if pin_in else host
    pcm[:] = host
    tracks, pos = [], 0
    for m in lens:
        tracks.append((pos, m))
        pos += m
    opts = A.make_options(**oracle_port.PRESETS["8"])
    _, nb = eng.bounds(opts, tracks, 2, 16)
    out = A.pinned_empty(nb, np.uint8) if pin_out else None
    out, res, offs, fpcm = eng.encode(opts, pcm, tracks, 2, 16, 44100, out=out)
    end = 0
    for k in range(len(parts)):
        r = res[k]
        assert r.out_offset == (end + 15) // 16 * 16      # packed, 16-byte aligned
        end = r.out_offset + r.bytes
        want, woffs = oracle_port.encode(parts[k].astype(np.int32), 2, 16, 44100,
                                         **oracle_port.PRESETS["8"])
        assert bytes(out[r.out_offset:r.out_offset + r.bytes]) == want, k
        got = [(int(offs[r.first_frame + i]), int(fpcm[r.first_frame + i]))
               for i in range(r.n_frames)]
        assert got == woffs, k


@pytest.mark.parametrize("pinned", [True, False])
def test_async_host_jobs_overlap(pinned, chunked):
    """atg_flac_encode_host_async: three jobs queued back to back share the
    chunk pipeline (a job's first chunks ride behind the previous job's
    last ones; 1 MB chunks wrap the three stages within and across jobs);
    waited in order, then a fourth waited before it could overlap.  Every
    job's images and frame tables equal the synchronous call's, which are
    the port's (test_chunked_host_encode_matches_port)."""
    eng, A = chunked
    eng.set_host_chunk_bytes(1 << 20)
    opts = A.make_options(**oracle_port.PRESETS["8"])
    jobs, want = [], []
    for seed in range(4):
        rng = np.random.default_rng(40 + seed)
        lens, parts = _tracks(rng, 7 + 3 * seed, 1000, 150000)
        host = np.concatenate(parts)
        pcm = A.pinned_empty(host.shape, np.int16) if pinned else host
        pcm[:] = host
        tracks, pos = [], 0
        for m in lens:
            tracks.append((pos, m))
            pos += m
        _, nb = eng.bounds(opts, tracks, 2, 16)
        out = A.pinned_empty(nb, np.uint8) if pinned else None
        jobs.append((pcm, tracks, out))
        o, r, f, p = eng.encode(opts, pcm, tracks, 2, 16, 44100)
        want.append(([bytes(o[x.out_offset:x.out_offset + x.bytes]) for x in r],
                     f.copy(), p.copy()))
    queued = [eng.encode_async(opts, pcm, tracks, 2, 16, 44100, out=out)
              for pcm, tracks, out in jobs[:3]]
    got = [j.wait() for j in queued]
    got.append(eng.encode_async(opts, *jobs[3][:2], 2, 16, 44100, out=jobs[3][2]).wait())
    for k, (out, res, offs, fpcm) in enumerate(got):
        imgs = [bytes(out[x.out_offset:x.out_offset + x.bytes]) for x in res]
        assert imgs == want[k][0], k
        assert np.array_equal(offs, want[k][1]) and np.array_equal(fpcm, want[k][2]), k


def test_async_host_job_refuses_device_batches(chunked, gpu_engine):
    """a host job in flight and an unwaited device batch exclude each other
    (they share the engine's slots); a ticket is waited once"""
    eng, A = chunked
    eng.set_host_chunk_bytes(1 << 20)
    rng = np.random.default_rng(3)
    lens, parts = _tracks(rng, 9, 50000, 150000)
    pcm = np.concatenate(parts)
    tracks, pos = [], 0
    for m in lens:
        tracks.append((pos, m))
        pos += m
    opts = A.make_options(**oracle_port.PRESETS["8"])
    job = eng.encode_async(opts, pcm, tracks, 2, 16, 44100)
    with pytest.raises(A.ATGError):
        eng.encode_device_async(opts, 0, A.PCM_S16, tracks, 2, 16, 44100, 0, 0)
    out, res, _, _ = job.wait()
    assert all(r.bytes for r in res)
    with pytest.raises(A.ATGError):
        A._check(eng.lib, eng.lib.atg_flac_encode_host_wait(eng.handle, job.ticket))
