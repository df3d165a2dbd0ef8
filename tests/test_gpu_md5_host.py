"""Engine host-MD5 mode (engine.hip want_host_md5 / start_host_md5): the
STREAMINFO MD5 of a device batch hashed by host threads from a D2H copy of
the PCM instead of GPU chains.  The images must be the bytes the port
(pinned to the reference encoder) writes, whichever side hashed, for every
container width the engine takes, synchronous and pipelined.
"""
import numpy as np
import pytest

import oracle_port
import signals

pytestmark = pytest.mark.gpu

FLAC8 = dict(oracle_port.PRESETS["8"])


def _device_batch(torch, pcms, bps):
    dt = torch.int16 if bps <= 16 else torch.int32
    host = np.concatenate(pcms).astype(np.int16 if bps <= 16 else np.int32)
    return torch.from_numpy(host).to("cuda").to(dt).contiguous()


def _encode(eng, torch, pcms, ch, bps, rate, asynchronous=False, reps=1):
    from audiotools import _atgpu
    opts = _atgpu.make_options(**FLAC8)
    tracks, start = [], 0
    for p in pcms:
        tracks.append((start, len(p) // ch))
        start += len(p) // ch
    d = _device_batch(torch, pcms, bps)
    fmt = _atgpu.PCM_S16 if bps <= 16 else _atgpu.PCM_S32
    _, cap = eng.bounds(opts, tracks, ch, bps)
    outs = [torch.zeros(cap, dtype=torch.uint8, device="cuda") for _ in range(reps)]
    torch.cuda.synchronize()
    if asynchronous:
        tickets = [eng.encode_device_async(opts, d.data_ptr(), fmt, tracks, ch, bps, rate,
                                           o.data_ptr(), cap) for o in outs]
        results = [eng.wait(t) for t in tickets]
    else:
        results = [eng.encode_device(opts, d.data_ptr(), fmt, tracks, ch, bps, rate,
                                     o.data_ptr(), cap) for o in outs]
    images = []
    for o, res in zip(outs, results):
        host = o.cpu().numpy()
        images.append([host[r.out_offset:r.out_offset + r.bytes].tobytes() for r in res])
    return images


@pytest.mark.parametrize("ch,bps", [(2, 16), (6, 24), (1, 8), (2, 24)])
@pytest.mark.parametrize("asynchronous", [False, True])
def test_host_md5_images_equal_port(ch, bps, asynchronous):
    import torch
    from audiotools import _atgpu
    pcms = [signals.make("tone", 4096 * 5 + 77, ch, bps, seed=3),
            signals.make("noise", 4096 * 2, ch, bps, seed=4),
            signals.make("silence", 300, ch, bps, seed=5)]
    eng = _atgpu.Engine(0, md5="host")
    try:
        imgs = _encode(eng, torch, pcms, ch, bps, 48000, asynchronous, reps=3 if asynchronous else 1)
    finally:
        eng.close()
    for batch in imgs:
        for p, img in zip(pcms, batch):
            want, _ = oracle_port.encode(p, ch, bps, 48000, **FLAC8)
            assert img == want


def test_auto_picks_host_for_long_tracks_and_matches_gpu():
    """config-5 shape in small: few long 5.1 24-bit tracks take the host
    side under "auto"; the images equal the GPU-hashed ones and the port's"""
    import torch
    from audiotools import _atgpu
    ch, bps, rate = 6, 24, 48000
    n = 48000 * 4  # 4.6 MB of MD5 input per track: a ~55 ms GPU chain
    pcms = [signals.make("tone", n, ch, bps, seed=10 + k) for k in range(3)]
    got = {}
    for mode in ("auto", "gpu"):
        eng = _atgpu.Engine(0, md5=mode)
        try:
            got[mode] = _encode(eng, torch, pcms, ch, bps, rate, asynchronous=True, reps=2)
            kt = eng.kernel_times()
        finally:
            eng.close()
        if mode == "auto":
            auto_kt = kt
    assert got["auto"] == got["gpu"]
    for p, img in zip(pcms, got["auto"][0]):
        want, _ = oracle_port.encode(p, ch, bps, rate, **FLAC8)
        assert img == want
    assert "track_md5" in auto_kt


@pytest.mark.parametrize("ch,bps", [(2, 16), (6, 24)])
def test_host_md5_groups_of_sixteen(ch, bps):
    """more tracks than one host task takes (16 per task, hashed side by
    side): 37 tracks of uneven lengths, so the groups differ in size and
    every stream ends at its own byte"""
    import torch
    from audiotools import _atgpu
    pcms = [signals.make("tone" if k % 3 else "noise", 700 + 311 * k, ch, bps, seed=20 + k)
            for k in range(37)]
    eng = _atgpu.Engine(0, md5="host")
    try:
        (batch,) = _encode(eng, torch, pcms, ch, bps, 44100)
    finally:
        eng.close()
    for p, img in zip(pcms, batch):
        want, _ = oracle_port.encode(p, ch, bps, 44100, **FLAC8)
        assert img == want
