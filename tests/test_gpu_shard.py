"""GPU: the multi-device product path on one MI355X.

ATG_SHARD_DEVICES="0,0,0" makes the batch entry points take their sharded
path with three shards (three engines / decoders) on device 0: the images,
decoded PCM and ReplayGain results must equal the unsharded call's, and the
unsharded call's equal the oracle's.  The device choice of the drop-in
entry points reaches device 0 on a one-GPU box."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_port
import signals

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Reader(object):
    def __init__(self, x, ch, bps, rate=44100):
        self.x, self.channels, self.bits_per_sample, self.sample_rate = x, ch, bps, rate
        self.channel_mask, self.pos = 0x3 if ch == 2 else 0x4, 0

    def read(self, n):
        from audiotools import pcm
        a = self.x[self.pos:self.pos + n * self.channels]
        self.pos += len(a)
        return pcm.FrameList._wrap(np.asarray(a, dtype=np.int32), self.channels,
                                   self.bits_per_sample)

    def close(self):
        pass


def _pcms(n=7):
    return [signals.make(["tone", "noise", "chirp"][k % 3], 4096 * (k % 4 + 1) + 99 * k, 2, 16,
                         seed=70 + k) for k in range(n)]


def test_encode_decode_batch_sharded(tmp_path, monkeypatch):
    from audiotools import decoders, encoders
    pcms = _pcms()
    opts = dict(oracle_port.PRESETS["8"])
    args = (opts["block_size"], opts["max_lpc_order"], opts["min_residual_partition_order"],
            opts["max_residual_partition_order"])
    kw = dict(mid_side=opts["mid_side"], exhaustive_model_search=opts["exhaustive_model_search"])
    runs = {}
    for shards in ("", "0,0,0"):
        monkeypatch.setenv("ATG_SHARD_DEVICES", shards)
        fns = [str(tmp_path / ("%s_%d.flac" % (shards or "one", k))) for k in range(len(pcms))]
        offs = encoders.encode_flac_batch(fns, [_Reader(p, 2, 16) for p in pcms], *args, **kw)
        imgs = [open(f, "rb").read() for f in fns]
        runs[shards] = (offs, imgs, decoders.decode_flac_batch(imgs))
    assert runs[""][0] == runs["0,0,0"][0] and runs[""][1] == runs["0,0,0"][1]
    for p, img in zip(pcms, runs[""][1]):
        want, _ = oracle_port.encode(p, 2, 16, 44100, **opts)
        assert img == want
    for a, b, p in zip(runs[""][2], runs["0,0,0"][2], pcms):
        assert a[0] == b[0] == 0
        assert np.array_equal(a[2], b[2]) and np.array_equal(a[2], p.astype(np.int32))


def test_calculate_replay_gain_sharded(monkeypatch):
    import audiotools
    from audiotools import replaygain

    class T(object):
        def __init__(self, x, ch):
            self.x, self.ch = x, ch

        def sample_rate(self):
            return 44100

        def channels(self):
            return self.ch

        def total_frames(self):
            return len(self.x) // self.ch

        def to_pcm(self):
            return _Reader(self.x, self.ch, 16)

    tracks = [T(signals.make("tone", 44100 // 2 + 777 * k, 1 + (k % 2), 16, seed=k), 1 + (k % 2))
              for k in range(9)]
    got = {}
    for shards in ("", "0,0,0,0"):
        monkeypatch.setenv("ATG_SHARD_DEVICES", shards)
        got[shards] = [g[1:] for g in audiotools.calculate_replay_gain(tracks)]
    assert got[""] == got["0,0,0,0"]
    # the title-by-title object the reference drives gives the same numbers
    monkeypatch.setenv("ATG_SHARD_DEVICES", "")
    rg = replaygain.ReplayGain(44100)
    titles = [rg.title_gain(t.to_pcm()) for t in tracks]
    album = rg.album_gain()
    assert [g[:2] for g in got[""]] == titles
    assert all(g[2:] == album for g in got[""])
    hists = [oracle_port.rg_title(t.x, t.ch, 16, 44100)[0] for t in tracks]
    assert album[0] == oracle_port.rg_gain(np.sum(hists, axis=0).astype(np.uint32))


def test_device_choice_reaches_device_0(tmp_path):
    env = {k: v for k, v in os.environ.items()
           if k not in ("ATG_DEVICE", "LOCAL_RANK", "ATG_SHARD_DEVICES", "ATG_DEVICE_COUNT")}
    env["ATG_RR_FILE"] = str(tmp_path / "rr")
    code = ("import sys; sys.path.insert(0, %r); from audiotools import _atgpu; "
            "e = _atgpu.engine(); print(_atgpu.visible_devices(), _atgpu.default_device(), "
            "e.device)" % os.path.join(ROOT, "python-audio-tools_amd"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         check=True).stdout.split()
    n, d, e = (int(x) for x in out)
    assert 0 <= d < n and e == d
    if n == 1:
        assert d == 0
