"""GPU parity for the ALAC read() walk (alac_decode.hip k_adec_chain: a
wave per track checks 64 chained frameset predictions a step, then walks
on serially), status and PCM against the CPU oracle's read() loop
(oracle/alac_port.c, pinned to the reference decoder by the golden vectors
in test_gpu_alac.py).

One long stream (151 framesets of 256 frames: the wave's first, second and
third steps) decoded in one batch as several tracks, each taking the fast
steps and the serial walk at a different point:

* the whole stream with its `stsz` hints (every step fast, the last partial);
* remaining_frames ending inside the second step (the walk stops mid-wave);
* a hint wrong at frameset 70 (the predictions after it all miss: fast to
  70, then every frameset parsed inline);
* a start at frameset 10 with the hints from there, and with the hints from
  the stream's start (nothing matches: the serial walk from the start);
* no hints at all.
"""
import numpy as np
import pytest

import oracle_port as op
import signals

pytestmark = pytest.mark.gpu

BLOCK = 256
N = BLOCK * 150 + 37


def _stream():
    from audiotools import m4a
    x = signals.make("tone", N, 2, 16, seed=31)
    mdat, fs = op.alac_encode(x, 2, 16, block_size=BLOCK)
    img = m4a.m4a_file(2, 16, 44100, BLOCK, N, mdat, fs, create_date=0)
    return x, img


def test_walk_fast_and_serial():
    from audiotools import _atgpu
    x, img = _stream()
    st, info, _, sizes = _atgpu.alac_read_info(img)
    assert st == 0 and len(sizes) == 151
    sizes = [int(v) for v in sizes]
    start10 = info.mdat_offset + sum(sizes[:10])
    bad = list(sizes)
    bad[70] += 4
    cases = [
        ("full", None, None, sizes),
        ("remaining_mid_wave", None, BLOCK * 100 + 5, sizes),
        ("hint_wrong_at_70", None, None, bad),
        ("start10_hints", start10, N - 10 * BLOCK, sizes[10:]),
        ("start10_hints_from_0", start10, N - 10 * BLOCK, sizes),
        ("no_hints", None, None, None),
    ]
    pad = (-len(img)) % 4
    blob = b"".join([img + b"\0" * pad] * len(cases))
    tracks = [_atgpu.alac_dec_track(k * (len(img) + pad), len(img), info,
                                    start=None if s is None else s,
                                    remaining=r, frameset_bytes=h)
              for k, (_, s, r, h) in enumerate(cases)]
    # alac_dec_track's start is relative to the image, as info.mdat_offset
    pcm, res, _, _ = _atgpu.alac_decoder().decode(blob, tracks)
    rc, oinfo, _ = op.alac_read_info(img)
    assert rc == 0 and oinfo.mdat_offset == info.mdat_offset
    for (name, s, r, _), rr in zip(cases, res):
        want = op.alac_decode(img, oinfo, start=s, remaining=r)
        got = pcm[rr.sample_offset:rr.sample_offset + rr.pcm_frames * 2]
        assert rr.status == want["code"], (name, rr.status, want["code"])
        assert np.array_equal(got, want["pcm"]), name
    # the full decode is the source
    assert np.array_equal(pcm[res[0].sample_offset:res[0].sample_offset + 2 * N], x)
