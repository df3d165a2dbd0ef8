"""GPU parity: libatgpu's FLAC encoder vs the CPU oracle (byte-identical).

Runs on the MI355X box (`pytest -m gpu`).  Every case encodes the same
seeded PCM with the GPU engine (through the C ABI) and with the oracle
(oracle/flac_port.c, itself byte-identical to the reference encoder), and
requires identical .flac images, identical frame offset lists, and a clean
oracle decode round trip.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_port
import signals

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def gpu_encode_tracks(engine, pcms, channels, bps, rate, opts, frame_sizes=None):
    from audiotools import _atgpu
    o = _atgpu.make_options(**opts)
    tracks, parts, start = [], [], 0
    for i, p in enumerate(pcms):
        n = len(p) // channels
        fs = None if frame_sizes is None else frame_sizes[i]
        tracks.append((start, n, fs))
        parts.append(p)
        start += n
    pcm = np.concatenate(parts) if parts else np.zeros(0, np.int32)
    pcm = pcm.astype(np.int16 if bps <= 16 else np.int32)
    out, res, offs, fpcm = engine.encode(o, pcm, tracks, channels, bps, rate)
    images = []
    for r in res:
        img = out[r.out_offset:r.out_offset + r.bytes].tobytes()
        lst = [(int(offs[r.first_frame + i]), int(fpcm[r.first_frame + i]))
               for i in range(r.n_frames)]
        images.append((img, lst))
    return images


def check_batch(engine, pcms, channels, bps, opts, rate=44100):
    got = gpu_encode_tracks(engine, pcms, channels, bps, rate, opts)
    for p, (img, lst) in zip(pcms, got):
        want, wlst = oracle_port.encode(p, channels, bps, rate, **opts)
        assert img == want, ("GPU/oracle mismatch: %d vs %d bytes, ch=%d bps=%d opts=%r"
                             % (len(img), len(want), channels, bps, opts))
        assert lst == wlst
        dec, ch, b, r = oracle_port.decode(img)
        assert np.array_equal(dec, p)


@pytest.mark.parametrize("preset", ["8", "0", "1", "2", "3", "4", "5", "6", "7"])
@pytest.mark.parametrize("channels,bps", [(2, 16), (1, 16), (2, 24), (6, 16), (6, 24), (1, 8)])
def test_presets_vs_oracle(gpu_engine, preset, channels, bps):
    opts = dict(oracle_port.PRESETS[preset])
    B = opts["block_size"]
    rng = np.random.default_rng(int(preset) * 1000 + channels * 100 + bps)
    pcms = []
    for kind in ["tone", "sine", "noise", "silence", "chirp", "wasted"]:
        if kind == "wasted" and bps == 8:
            continue
        n = int(rng.integers(1, 3 * B)) if kind != "tone" else 3 * B + 17
        pcms.append(signals.make(kind, n, channels, bps, seed=int(rng.integers(1 << 30))))
    check_batch(gpu_engine, pcms, channels, bps, opts)


def test_small_and_fsd_streams(gpu_engine):
    opts = dict(block_size=1152, max_lpc_order=16, min_residual_partition_order=0,
                max_residual_partition_order=3, mid_side=True, adaptive_mid_side=True,
                exhaustive_model_search=True)
    for samples, ch, bps in signals.SHORT_STREAMS:
        check_batch(gpu_engine, [np.array(samples, np.int32)], ch, bps, opts)
    for bps in (8, 16, 24):
        pcms = [signals.fsd(p, 100, bps) for p in signals.PATTERNS]
        check_batch(gpu_engine, pcms, 1, bps, opts)
    check_batch(gpu_engine, [signals.wasted_bps16(1000)], 2, 16, opts)


@pytest.mark.parametrize("block_size", [16, 17, 19, 24, 32, 33, 192, 576, 1000, 4096])
def test_block_sizes_lpc_orders(gpu_engine, block_size):
    rng = np.random.default_rng(block_size)
    noise = rng.integers(-32768, 32768, 32).astype(np.int32)
    for disable in [{}, dict(disable_verbatim_subframes=True, disable_constant_subframes=True),
                    dict(disable_verbatim_subframes=True, disable_constant_subframes=True,
                         disable_fixed_subframes=True)]:
        for lpc in [0, 1, 2, 4, 8, 9, 12, 15, 16, 17, 31, 32]:
            opts = dict(block_size=block_size, max_lpc_order=lpc,
                        min_residual_partition_order=0, max_residual_partition_order=6,
                        mid_side=True, adaptive_mid_side=True, exhaustive_model_search=True)
            opts.update(disable)
            pcms = [np.tile(noise, 400)[:n] for n in (block_size * 3 + 1, 200, 7)]
            check_batch(gpu_engine, pcms, 1, 16, opts)


def test_fractional_lengths(gpu_engine):
    opts = dict(block_size=256, max_lpc_order=8, min_residual_partition_order=0,
                max_residual_partition_order=6)
    lens = [254, 255, 256, 257, 258, 510, 511, 512, 513, 1022, 1023, 1024, 1025, 4095, 4097]
    pcms = [signals.noise(n, 2, 16, n) for n in lens]
    check_batch(gpu_engine, pcms, 2, 16, opts)


def test_rates_and_headers(gpu_engine):
    opts = dict(oracle_port.PRESETS["8"])
    for rate in [8000, 9, 90, 12345, 44100, 90000, 96000, 192000, 700000]:
        pcms = [signals.make("tone", 9000, 2, 16, seed=rate)]
        got = gpu_encode_tracks(gpu_engine, pcms, 2, 16, rate, opts)
        want, _ = oracle_port.encode(pcms[0], 2, 16, rate, **opts)
        assert got[0][0] == want


def test_tone_flac_kat(gpu_engine):
    """reference known-answer fixture test/tone.flac (FLAC-8 frames)"""
    data = open(os.path.join(GOLDEN, "tone.flac"), "rb").read()
    pcm, ch, bps, rate = oracle_port.decode(data)
    blocks, frames = oracle_port.split_flac(data)
    img, _ = gpu_encode_tracks(gpu_engine, [pcm], ch, bps, rate,
                               oracle_port.PRESETS["8"])[0]
    gblocks, gframes = oracle_port.split_flac(img)
    assert gblocks[0][1] == blocks[0][1]          # STREAMINFO incl. MD5
    assert hashlib.sha256(gframes).hexdigest() == hashlib.sha256(frames).hexdigest()


def test_many_tracks_one_batch(gpu_engine):
    opts = dict(oracle_port.PRESETS["8"])
    pcms = [signals.make("tone", 4096 * 3 + k * 131, 2, 16, seed=k) for k in range(40)]
    check_batch(gpu_engine, pcms, 2, 16, opts)


def test_explicit_frame_sizes(gpu_engine):
    """frames cut exactly where pcmreader.read() returned (flac.c:244-274):
    block-size codes 0x6/0x7 + explicit sizes (flac.c:412-518), byte-equal to
    the port's encode of the same reads"""
    opts = dict(oracle_port.PRESETS["8"])
    pcm = signals.make("tone", 10000, 2, 16, seed=3)
    sizes = [4096, 1000, 4096, 808]
    got = gpu_encode_tracks(gpu_engine, [pcm], 2, 16, 44100, opts, frame_sizes=[sizes])
    img, lst = got[0]
    want, wlst = oracle_port.encode(pcm, 2, 16, 44100, frame_sizes=sizes, **opts)
    assert img == want
    assert lst == wlst and [n for _, n in lst] == sizes
    dec, ch, b, r = oracle_port.decode(img)
    assert np.array_equal(dec, pcm)


VECTORS = json.load(open(os.path.join(GOLDEN, "flac_vectors.json")))["vectors"]


def _golden_pcm(v):
    if v["kind"] == "fsd":
        mono = signals.fsd(signals.PATTERNS[v["seed"] % len(signals.PATTERNS)], v["n"],
                           v["bps"])
        return np.repeat(mono[:, None], v["channels"], 1).reshape(-1).astype(np.int32)
    return signals.make(v["kind"], v["n"], v["channels"], v["bps"], seed=v["seed"])


@pytest.mark.parametrize("preset", sorted(oracle_port.PRESETS))
def test_golden_vectors_reference_hashes(gpu_engine, preset):
    """every committed reference-encoder vector (tests/golden/make_golden.py:
    presets 0-8 x {1,2,6} ch x {8,16,24} bit incl. 5.1 24-bit, config 5's
    encoder shape) encoded on the GPU, one batch per format: sha256 equal to
    the reference encoder's"""
    by_fmt = {}
    for v in VECTORS:
        if v["preset"] == preset:
            by_fmt.setdefault((v["channels"], v["bps"]), []).append(v)
    assert (6, 24) in by_fmt and (6, 8) in by_fmt
    opts = dict(oracle_port.PRESETS[preset])
    for (ch, bps), vs in sorted(by_fmt.items()):
        got = gpu_encode_tracks(gpu_engine, [_golden_pcm(v) for v in vs], ch, bps, 44100, opts)
        for v, (img, _) in zip(vs, got):
            assert len(img) == v["bytes"], v["name"]
            assert hashlib.sha256(img).hexdigest() == v["sha256"], v["name"]


SIZED = json.load(open(os.path.join(GOLDEN, "flac_vectors_sized.json")))["vectors"]


@pytest.mark.parametrize("preset", ["8", "5", "2", "0"])
def test_sized_reads_golden(gpu_engine, preset):
    """the reference encoder's streams for short/long reads
    (tests/golden/make_golden_sized.py: 1-frame reads, reads longer than the
    block, standard-code sizes, an empty read ending the stream) -- one GPU
    batch per format, every image's sha256 equal to the reference's and the
    bytes equal to the port's"""
    cases = [v for v in SIZED if v["preset"] == preset]
    opts = dict(oracle_port.PRESETS[preset])
    by_fmt = {}
    for v in cases:
        by_fmt.setdefault((v["channels"], v["bps"]), []).append(v)
    for (ch, bps), vs in sorted(by_fmt.items()):
        pcms = []
        for v in vs:
            x = signals.make(v["kind"], v["n"], ch, bps, seed=v["seed"])
            pcms.append(x[:sum(v["frame_lengths"]) * ch])
        got = gpu_encode_tracks(gpu_engine, pcms, ch, bps, 44100, opts,
                                frame_sizes=[v["frame_lengths"] for v in vs])
        for v, p, (img, lst) in zip(vs, pcms, got):
            assert [n for _, n in lst] == v["frame_lengths"], v["name"]
            assert len(img) == v["bytes"], v["name"]
            assert hashlib.sha256(img).hexdigest() == v["sha256"], v["name"]
            want, wlst = oracle_port.encode(p, ch, bps, 44100,
                                            frame_sizes=v["read_sizes"], **opts)
            assert img == want and lst == wlst, v["name"]


@pytest.mark.parametrize("seed", range(4))
def test_random_frame_sizes_vs_port(gpu_engine, seed):
    """random cuts (1..9000 frames per read) over several formats and
    presets, many tracks per batch, against the port"""
    rng = np.random.default_rng(500 + seed)
    preset = ["8", "6", "3", "1"][seed]
    opts = dict(oracle_port.PRESETS[preset])
    ch, bps = [(2, 16), (6, 24), (1, 8), (2, 24)][seed]
    pcms, cuts = [], []
    for k in range(12):
        n = int(rng.integers(1, 40000))
        sizes = [int(x) for x in rng.integers(1, 9000, int(rng.integers(1, 8)))]
        cut = oracle_port.cut_frames(n, opts["block_size"], sizes)
        pcms.append(signals.make(["tone", "noise", "chirp", "sine"][k % 4], n, ch, bps,
                                 seed=seed * 100 + k))
        cuts.append(cut)
    got = gpu_encode_tracks(gpu_engine, pcms, ch, bps, 44100, opts, frame_sizes=cuts)
    for p, cut, (img, lst) in zip(pcms, cuts, got):
        want, wlst = oracle_port.encode(p, ch, bps, 44100, frame_sizes=cut, **opts)
        assert img == want and lst == wlst, (cut, len(p) // ch)


def test_unsupported_options_raise(gpu_engine):
    from audiotools import _atgpu
    o = _atgpu.make_options(block_size=65536, max_lpc_order=8,
                            min_residual_partition_order=0, max_residual_partition_order=6)
    pcm = np.zeros(200000, np.int16)
    with pytest.raises(_atgpu.ATGError) as e:
        gpu_engine.encode(o, pcm, [(0, 100000)], 2, 16, 44100)
    assert e.value.status == _atgpu.ATG_ERR_UNSUPPORTED


def test_encode_flac_api(tmp_path):
    """audiotools.encoders.encode_flac: reference signature and return value"""
    import audiotools
    from audiotools.encoders import encode_flac
    pcm = signals.make("tone", 30000, 2, 16, seed=9)
    reader = audiotools.BufferedPCMReader(audiotools.FrameListReader(pcm, 44100, 2, 16))
    fn = str(tmp_path / "a.flac")
    offsets = encode_flac(fn, reader, **oracle_port.PRESETS["8"])
    want, wlst = oracle_port.encode(pcm, 2, 16, 44100, **oracle_port.PRESETS["8"])
    assert open(fn, "rb").read() == want
    assert offsets == wlst


class _SizedReader(object):
    """a PCMReader whose read() returns the listed frame counts, then
    `block` frames at a time (each read is one FLAC frame, flac.c:244-274)"""

    def __init__(self, samples, rate, channels, bps, sizes=()):
        import audiotools
        self._r = audiotools.FrameListReader(samples, rate, channels, bps)
        self.sample_rate, self.channels, self.bits_per_sample = rate, channels, bps
        self.channel_mask = 0
        self.sizes = list(sizes)
        self.closed = False

    def read(self, n):
        return self._r.read(self.sizes.pop(0) if self.sizes else n)

    def close(self):
        self.closed = True


@pytest.mark.parametrize("ch,bps,n,sizes,seg", [
    (2, 16, 4096 * 20 + 77, (), 3),          # 7 segments of 3 frames
    (2, 16, 4096 * 9, (4096, 1000, 7, 4096, 4095, 1), 4),
    (6, 24, 4096 * 5 + 5, (), 2),
    (1, 8, 3000, (), 256),
    (2, 16, 0, (), 3),                       # empty stream
])
def test_encode_flac_streaming(tmp_path, ch, bps, n, sizes, seg):
    """encode_flac (the C extension) streams in segments of up to 256 frames
    (frame numbers continue across segments, the MD5 of each segment hashed
    on a host thread, STREAMINFO rewritten at the end): the file equals the
    oracle's encode of the same reads"""
    from audiotools import _encoders_c, encoders
    x = signals.make("tone", n, ch, bps, seed=n + ch) if n else np.zeros(0, np.int32)
    opts = dict(oracle_port.PRESETS["8"])
    r = _SizedReader(x, 44100, ch, bps, sizes)
    fn = str(tmp_path / "s.flac")
    old = _encoders_c._set_segment_frames(seg)
    try:
        lst = encoders.encode_flac(fn, r, **opts)
    finally:
        _encoders_c._set_segment_frames(old)
    assert r.closed
    got = open(fn, "rb").read()
    # the oracle cuts the same frames: explicit sizes
    cut, left = list(sizes), n - sum(sizes)
    while left > 0:
        cut.append(min(left, opts["block_size"]))
        left -= cut[-1]
    if sizes:
        img = _port_frames(x, ch, bps, cut, opts)
    else:
        img, wl = oracle_port.encode(x, ch, bps, 44100, **opts)
        assert lst == wl
    assert [m for _, m in lst] == cut
    assert got == img
    dec, _, _, _ = oracle_port.decode(got)
    assert np.array_equal(dec, x)


def _port_frames(x, ch, bps, cut, opts):
    """the port's stream for explicit frame sizes (flacport_encode_sizes,
    pinned to the reference encoder by tests/golden/flac_vectors_sized.json)"""
    return oracle_port.encode(x, ch, bps, 44100, frame_sizes=cut, **opts)[0]


def test_loud_side_channel_split_fold(gpu_engine):
    """stereo whose side channel L - R runs near +-65535 (anti-phase full
    scale, uncorrelated full-scale noise, a hard-clipped square pair): the
    side candidate's predictors leave the 32-bit fold's bound and take the
    split fold (flac_search16.hip eval_split) or the 64-bit loop; images
    byte-identical to the oracle at FLAC-8 and the low presets"""
    rng = np.random.default_rng(99)
    n = 4096 * 3 + 17
    t = np.arange(n)
    a = np.round(32767 * np.sin(2 * np.pi * 997 * t / 44100)).astype(np.int64)
    anti = np.stack([a, -a], 1).reshape(-1).clip(-32768, 32767).astype(np.int32)
    noise = rng.integers(-32768, 32768, 2 * n).astype(np.int32)
    sq = np.where((t // 37) % 2, 32767, -32768)
    square = np.stack([sq, -sq], 1).reshape(-1).clip(-32768, 32767).astype(np.int32)
    mix = (anti // 2 + noise // 2).clip(-32768, 32767).astype(np.int32)
    for preset in ("8", "5"):
        check_batch(gpu_engine, [anti, noise, square, mix], 2, 16,
                    dict(oracle_port.PRESETS[preset]))


def test_encode_frames_back_to_back_uploads(gpu_engine):
    """atg_flac_encode_frames twice on one engine with the same geometry and
    different PCM (4 MiB each): the second call's frames equal the port's
    for ITS PCM.  The upload and the LPC kernel sit on different streams
    (engine.hip: K1 on the slot stream), so an LPC kernel not ordered after
    the upload would analyse the first call's samples still in the device
    buffer"""
    from audiotools import _atgpu
    opts = dict(oracle_port.PRESETS["8"])
    n = 4096 * 256
    for k, seed in enumerate((5, 6, 7)):
        x = signals.make("tone" if k % 2 else "noise", n, 2, 16, seed=seed).astype(np.int16)
        got, sizes = gpu_engine.encode_frames(_atgpu.make_options(**opts), x, 2, 16, 44100)
        want = oracle_port.split_flac(oracle_port.encode(x.astype(np.int32), 2, 16, 44100,
                                                         **opts)[0])[1]
        assert bytes(got) == want, "call %d" % k
