"""CPU: the converter oracle (oracle/pcmconv_port.c) against hand-computed
values and the invariants SURVEY.md 8(a) R4/R5 names.  Parity unpinned: the
reference holds no fixtures for these converters."""
import math

import numpy as np

import oracle_port as op


def test_bps_down_dither_order_and_invariant():
    rng = np.random.RandomState(1)
    frames, ch = 5000, 2
    x = rng.randint(-2 ** 23, 2 ** 23, size=frames * ch).astype(np.int32)
    dither = rng.bytes((frames * ch + 7) // 8)
    y = op.convert(op.CONV_BPS, x, ch, 24, 16, dither=dither)
    base = x >> 8
    assert set(np.unique(y ^ base)) <= {0, 1}
    # bit order: per 4096-frame read, channel by channel, MSB first
    bits = np.unpackbits(np.frombuffer(dither, dtype=np.uint8))
    want = np.empty_like(base)
    k = 0
    for f0 in range(0, frames, 4096):
        n = min(4096, frames - f0)
        for c in range(ch):
            idx = (np.arange(f0, f0 + n) * ch + c)
            want[idx] = base[idx] ^ bits[k:k + n]
            k += n
    assert np.array_equal(y, want)


def test_bps_up_is_shift():
    x = np.array([-32768, -1, 0, 1, 32767], dtype=np.int32)
    assert list(op.convert(op.CONV_BPS, x, 1, 16, 24)) == [v << 8 for v in x.tolist()]


def test_average_truncates_toward_zero():
    x = np.array([-3, 0, 3, 0, -5, -4, 7, 8], dtype=np.int32)  # 2 channels
    assert list(op.convert(op.CONV_AVERAGE, x, 2, 16)) == [-1, 1, -4, 7]


def _downmix_ref(six, bps):
    mono = 0.7 * (six[4] + six[5])
    lo, hi = -(1 << (bps - 1)), (1 << (bps - 1)) - 1
    rnd = lambda v: int(math.copysign(math.floor(abs(v) + 0.5), v))
    l = rnd(six[0] + 0.6 * mono + 0.7 * six[2])
    r = rnd(six[1] - 0.6 * mono + 0.7 * six[2])
    return [max(lo, min(hi, l)), max(lo, min(hi, r))]


def test_downmix_values_and_masks():
    rng = np.random.RandomState(2)
    x = rng.randint(-32768, 32768, size=6 * 200).astype(np.int32)
    y = op.convert(op.CONV_DOWNMIX, x, 6, 16)
    for f in range(200):
        assert list(y[2 * f:2 * f + 2]) == _downmix_ref(x[6 * f:6 * f + 6].tolist(), 16)
    # 5.0 layout (mask 0x37: fL fR fC bL bR, no LFE)
    x5 = rng.randint(-1000, 1000, size=5 * 50).astype(np.int32)
    y5 = op.convert(op.CONV_DOWNMIX, x5, 5, 16, mask=0x37)
    for f in range(50):
        a = x5[5 * f:5 * f + 5].tolist()
        assert list(y5[2 * f:2 * f + 2]) == _downmix_ref([a[0], a[1], a[2], 0, a[3], a[4]], 16)
    # clamping
    big = np.array([32767, 32767, 32767, 0, 32767, 32767], dtype=np.int32)
    assert list(op.convert(op.CONV_DOWNMIX, big, 6, 16)) == [32767, 28180]
    assert _downmix_ref(big.tolist(), 16) == [32767, 28180]
