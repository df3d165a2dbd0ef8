"""GPU parity: pcm_convert.hip (BPSConverter / Downmixer / Averager bodies)
bit-exact against the CPU oracle on the same inputs and dither bytes; the
Python converter classes over a PCMReader.  Parity unpinned (no reference
fixtures exist for these converters), oracle restated from
src/pcmconverter.c."""
import numpy as np
import pytest

import oracle_port as op

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("frames", [0, 1, 4095, 4096, 4097, 12345])
@pytest.mark.parametrize("ch,ib,ob", [(2, 24, 16), (2, 16, 8), (1, 16, 24), (6, 24, 16),
                                      (2, 8, 16), (3, 20, 12)])
def test_bps_matches_oracle(frames, ch, ib, ob):
    from audiotools import _atgpu
    rng = np.random.RandomState(frames + ch)
    x = rng.randint(-2 ** (ib - 1), 2 ** (ib - 1), size=frames * ch).astype(np.int32)
    dither = rng.bytes((frames * ch + 7) // 8 + 1)
    kw = dict(dither=dither) if ob < ib else {}
    got = _atgpu.pcm_convert(_atgpu.CONV_BPS, x, ch, ib, ob, **kw)
    want = op.convert(op.CONV_BPS, x, ch, ib, ob, dither=dither)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("ch,mask", [(6, 0), (6, 0x3F), (5, 0x37), (4, 0x33), (3, 0x7),
                                     (2, 0x3), (1, 0x4), (8, 0)])
def test_downmix_matches_oracle(ch, mask):
    from audiotools import _atgpu
    rng = np.random.RandomState(ch)
    x = rng.randint(-32768, 32768, size=ch * 9000).astype(np.int32)
    x[:ch * 10] = 32767  # clamping
    got = _atgpu.pcm_convert(_atgpu.CONV_DOWNMIX, x, ch, 16, channel_mask=mask)
    want = op.convert(op.CONV_DOWNMIX, x, ch, 16, mask=mask)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("ch", [2, 3, 6, 8])
def test_average_matches_oracle(ch):
    from audiotools import _atgpu
    rng = np.random.RandomState(10 + ch)
    x = rng.randint(-2 ** 23, 2 ** 23, size=ch * 7777).astype(np.int32)
    got = _atgpu.pcm_convert(_atgpu.CONV_AVERAGE, x, ch, 24)
    assert np.array_equal(got, op.convert(op.CONV_AVERAGE, x, ch, 24))


def test_converter_classes_over_reader():
    import audiotools
    from audiotools import pcmconverter
    rng = np.random.RandomState(5)
    frames = 10000
    x = rng.randint(-2 ** 23, 2 ** 23, size=frames * 2).astype(np.int32)
    stream = rng.bytes(8192)
    pos = [0]

    def dither(n):
        b = stream[pos[0]:pos[0] + n]
        pos[0] += n
        return b + b"\0" * (n - len(b))

    r = pcmconverter.BPSConverter(
        audiotools.FrameListReader(x, 44100, 2, 24, 0x3), 16, dither=dither)
    out = []
    while True:
        fl = r.read(4096)
        if not len(fl):
            break
        out.append(fl.samples)
    got = np.concatenate(out)
    assert np.array_equal(got, op.convert(op.CONV_BPS, x, 2, 24, 16, dither=stream))
    six = rng.randint(-32768, 32768, size=6 * 5000).astype(np.int32)
    d = pcmconverter.Downmixer(audiotools.FrameListReader(six, 48000, 6, 16, 0x3F))
    got = np.concatenate([d.read(4096).samples for _ in range(2)])
    assert np.array_equal(got, op.convert(op.CONV_DOWNMIX, six, 6, 16, mask=0x3F))
    a = pcmconverter.Averager(audiotools.FrameListReader(six, 48000, 6, 16, 0x3F))
    got = np.concatenate([a.read(4096).samples for _ in range(2)])
    assert np.array_equal(got, op.convert(op.CONV_AVERAGE, six, 6, 16))
