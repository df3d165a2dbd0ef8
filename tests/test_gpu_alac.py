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


def _lw_groups():
    g = defaultdict(list)
    for v in G["leftweights"]:
        g[(v["channels"], v["bps"], v["lw_min"], v["lw_max"])].append(v)
    return sorted(g.items())


@pytest.mark.parametrize("key,vecs", _lw_groups(), ids=lambda x: str(x) if isinstance(x, tuple)
                         else None)
def test_leftweight_vectors_batch(key, vecs):
    """minimum/maximum_interlacing_leftweight ranges (alac.c:57-72,
    459-481): the GPU writes the recorded mdat bytes"""
    ch, bps, lo, hi = key
    pcms = [alac_cases.enc_pcm(v) for v in vecs]
    mdats, sizes, res = _gpu_encode(pcms, ch, bps, minimum_interlacing_leftweight=lo,
                                    maximum_interlacing_leftweight=hi)
    for v, m, fs, r in zip(vecs, mdats, sizes, res):
        assert r.status == 0
        assert hashlib.sha256(m).hexdigest() == v["sha256"], v["name"]
        assert len(fs) == v["framesets"]


def test_leftweight_errors():
    import audiotools
    from audiotools import _atgpu, encoders
    pcm = signals.make("tone", 5000, 2, 16, seed=1)
    for lo, hi in ((3, 2), (0, 256), (-1, 4)):
        with pytest.raises(ValueError):
            encoders.encode_alac(io.BytesIO(), audiotools.FrameListReader(pcm, 44100, 2, 16),
                                 4096, 10, 40, 14, lo, hi)
    enc = _atgpu.alac_encoder()
    with pytest.raises(_atgpu.ATGError):
        enc.encode(enc.options(minimum_interlacing_leftweight=5, maximum_interlacing_leftweight=4),
                   pcm.astype(np.int16), [(0, 2500)], 2, 16)


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


# ------------------------------------------------------------------ decoder
def _alac_batch(images, hints=True):
    from audiotools import _atgpu
    tracks, parts, infos, pos = [], [], [], 0
    for img in images:
        st, info, _, sizes = _atgpu.alac_read_info(img)
        infos.append((st, info))
        if st:
            continue
        pad = (-len(img)) % 4
        tracks.append(_atgpu.alac_dec_track(pos, len(img), info,
                                            frameset_bytes=sizes if hints else None))
        parts.append(img + b"\0" * pad)
        pos += len(img) + pad
    return tracks, b"".join(parts), infos


@pytest.mark.parametrize("hints", [True, False])
@pytest.mark.parametrize("s", G["decoder"], ids=lambda s: s["name"])
def test_decoder_vectors_batch(s, hints):
    """every clean / flipped / truncated image of a stream in one GPU batch:
    same status class, same PCM bytes as the reference decoder recorded"""
    from audiotools import _atgpu
    x = alac_cases.enc_pcm(s)
    mdat, fs = op.alac_encode(x, s["channels"], s["bps"])
    img = alac_cases.dec_image(s, mdat, fs)
    images = [alac_cases.mutate(img, c) for c in s["cases"]]
    tracks, blob, infos = _alac_batch(images, hints)
    pcm, res, _, _ = _atgpu.alac_decoder().decode(blob, tracks)
    k = 0
    for c, (st, info) in zip(s["cases"], infos):
        if st:
            assert c["rc"] == 1 and c["pcm_bytes"] == 0, c["name"]
            continue
        r = res[k]
        k += 1
        if r.status == _atgpu.AD_CHANNEL_MISMATCH:
            continue  # the Python path raises; the standalone has no check
        assert (r.status == 0) == (c["rc"] == 0), (c["name"], r.status, c["rc"])
        got = pcm[r.sample_offset:r.sample_offset + r.pcm_frames * info.channels]
        b = op.pcm_bytes(got, info.bits_per_sample)
        assert len(b) == c["pcm_bytes"], c["name"]
        assert hashlib.md5(b).hexdigest() == c["pcm_md5"], c["name"]
        # and sample for sample the CPU oracle's walk
        want = op.alac_decode(alac_cases.mutate(img, c))
        assert np.array_equal(got, want["pcm"]) and (want["code"] == r.status), c["name"]


def test_reference_fixture():
    import os
    from audiotools import decoders
    f = G["fixture"]
    fn = os.path.join(alac_cases.FIX, f["file"])
    d = decoders.ALACDecoder(fn)
    assert (d.channels, d.bits_per_sample, d.sample_rate, d.channel_mask) == (1, 16, 44100, 4)
    frames = []
    while True:
        fl = d.read(4096)
        if not len(fl):
            break
        frames.append(fl.samples)
    assert [len(x) for x in frames] == [20, 20]
    b = op.pcm_bytes(np.concatenate(frames), 16)
    assert hashlib.md5(b).hexdigest() == f["pcm_md5"]


@pytest.mark.parametrize("ch,bps", [(2, 16), (1, 24), (6, 24), (8, 16), (5, 16), (3, 24), (4, 16),
                                    (7, 24), (8, 24)])
def test_round_trip_gpu_encode_decode(ch, bps):
    from audiotools import decoders, m4a
    pcms = [signals.make(k, 4096 * (2 + i) + 13 * i, ch, bps, seed=i)
            for i, k in enumerate(["tone", "noise", "silence", "chirp"])]
    mdats, sizes, _ = _gpu_encode(pcms, ch, bps)
    imgs = [m4a.m4a_file(ch, bps, 44100, 4096, len(p) // ch, m, fs, create_date=3)
            for p, m, fs in zip(pcms, mdats, sizes)]
    out = decoders.decode_alac_batch(imgs)
    for p, (st, info, pcm) in zip(pcms, out):
        assert st == 0 and np.array_equal(pcm, p)


def test_alac_audio_from_pcm_seek_and_read(tmp_path):
    import audiotools
    from audiotools import m4a
    total = 44100 * 8 + 123
    x = signals.make("tone", total, 2, 16, seed=9)
    fn = str(tmp_path / "t.m4a")
    a = m4a.ALACAudio.from_pcm(fn, audiotools.FrameListReader(x, 44100, 2, 16, 3),
                               total_pcm_frames=total)
    assert (a.channels(), a.bits_per_sample(), a.total_frames()) == (2, 16, total)
    r = a.to_pcm()
    got = []
    while True:
        fl = r.read(4096)
        if not len(fl):
            break
        assert fl.frames <= 4096
        got.append(fl.samples)
    assert np.array_equal(np.concatenate(got), x)
    with pytest.raises(ValueError):
        r.seek(-1)
    # seektable: a chunk of 5 framesets per entry (m4a.py:1342-1381)
    assert r.seek(4096 * 7) == 4096 * 5
    rest = []
    while True:
        fl = r.read(4096)
        if not len(fl):
            break
        rest.append(fl.samples)
    assert np.array_equal(np.concatenate(rest), x[2 * 4096 * 5:])
    assert r.seek(0) == 0
    assert np.array_equal(r.read(4096).samples, x[:2 * 4096])
    r.close()
    with pytest.raises(ValueError):
        r.read(1)
    with pytest.raises(ValueError):
        r.seek(0)


def test_alac_decoder_errors(tmp_path):
    from audiotools import decoders, m4a
    x = signals.make("noise", 4096 * 3, 2, 16, seed=2)
    mdat, fs = op.alac_encode(x, 2, 16)
    img = m4a.m4a_file(2, 16, 44100, 4096, 4096 * 3, mdat, fs, create_date=1)
    fn = tmp_path / "cut.m4a"
    fn.write_bytes(img[:-100])
    d = decoders.ALACDecoder(str(fn))
    d.read(4096)
    d.read(4096)
    with pytest.raises(IOError):
        d.read(4096)
    fn.write_bytes(img[:20])
    with pytest.raises((IOError, ValueError)):
        decoders.ALACDecoder(str(fn))
    with pytest.raises(IOError):
        decoders.ALACDecoder(str(tmp_path / "missing.m4a"))
