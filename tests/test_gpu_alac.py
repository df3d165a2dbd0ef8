"""GPU parity: libatgpu's ALAC encoder (alac_encode.hip) against the
reference encoder's recorded output (tests/golden/alac_vectors.json: sha256
of the mdat atoms oracle/_ref/alacenc wrote) and against the CPU oracle
(oracle/alac_port.c) on seeded batches; the encode_alac / ALACAudio
interface."""
import hashlib
import io
from collections import defaultdict

import numpy as np
import pytest

import alac_cases
import oracle_port as op
import signals

pytestmark = pytest.mark.gpu
G = alac_cases.load()


def _gpu_encode(pcms, channels, bps, **opts):
    from audiotools import _atgpu
    enc = _atgpu.alac_encoder()
    o = enc.options(**opts)
    tracks, start = [], 0
    for p in pcms:
        tracks.append((start, len(p) // channels))
        start += len(p) // channels
    pcm = np.concatenate(pcms).astype(np.int16 if bps <= 16 else np.int32)
    out, res, fsb = enc.encode(o, pcm, tracks, channels, bps)
    mdats = [out[r.out_offset:r.out_offset + r.bytes].tobytes() for r in res]
    sizes = [[int(x) for x in fsb[r.first_frameset:r.first_frameset + r.n_framesets]]
             for r in res]
    return mdats, sizes, res


def _groups():
    g = defaultdict(list)
    for v in G["encoder"]:
        g[(v["channels"], v["bps"], v["block_size"])].append(v)
    return sorted(g.items())


@pytest.mark.parametrize("key,vecs", _groups(), ids=lambda x: str(x) if isinstance(x, tuple)
                         else None)
def test_encoder_vectors_batch(key, vecs):
    ch, bps, bs = key
    pcms = [alac_cases.enc_pcm(v) for v in vecs]
    mdats, sizes, res = _gpu_encode(pcms, ch, bps, block_size=bs)
    for v, m, fs, r in zip(vecs, mdats, sizes, res):
        assert r.status == 0
        assert hashlib.sha256(m).hexdigest() == v["sha256"], v["name"]
        assert len(fs) == v["framesets"] and sum(fs) + 8 == len(m)
        assert r.pcm_frames == v["n"]


@pytest.mark.parametrize("ch,bps", [(2, 16), (2, 24), (1, 16), (6, 24), (8, 16), (3, 24)])
def test_matches_oracle_mixed_batch(ch, bps):
    kinds = ["tone", "noise", "silence", "chirp", "sine", "wasted"]
    pcms = [signals.make(k, 4096 * (1 + i % 3) + 97 * i, ch, bps, seed=i + 10 * ch)
            for i, k in enumerate(kinds)]
    mdats, sizes, _ = _gpu_encode(pcms, ch, bps)
    for p, m, fs in zip(pcms, mdats, sizes):
        want, wfs = op.alac_encode(p, ch, bps)
        assert m == want and fs == wfs


def test_short_blocks_and_explicit_reads():
    """frames shorter than 10 samples are written uncompressed; a reader
    that returns odd-sized reads gets one frameset per read"""
    import audiotools
    from audiotools import encoders

    class OddReader(audiotools.FrameListReader):
        sizes = [4096, 7, 1000, 4096, 3]

        def read(self, n):
            k = self.sizes.pop(0) if self.sizes else n
            return audiotools.FrameListReader.read(self, k)

    x = signals.make("tone", 4096 + 7 + 1000 + 4096 + 3, 2, 16, seed=5)
    f = io.BytesIO()
    log, frames = encoders.encode_alac(f, OddReader(x, 44100, 2, 16, 3), 4096, 10, 40, 14)
    assert frames == len(x) // 2 and len(log) == 5
    # the reference encodes each read as one frameset: concatenating the
    # oracle's per-read mdats reproduces the frames
    body = b""
    pos = 0
    for n in [4096, 7, 1000, 4096, 3]:
        m, _ = op.alac_encode(x[2 * pos:2 * (pos + n)], 2, 16)
        body += m[8:]
        pos += n
    assert f.getvalue()[8:] == body


def test_encode_alac_errors():
    import audiotools
    from audiotools import encoders
    x = signals.make("tone", 100, 2, 8, seed=1)
    with pytest.raises(ValueError):
        encoders.encode_alac(io.BytesIO(), audiotools.FrameListReader(x, 44100, 2, 8), 4096, 10,
                             40, 14)
    with pytest.raises(TypeError):
        encoders.encode_alac("not a file", audiotools.FrameListReader(x, 44100, 2, 16), 4096,
                             10, 40, 14)
