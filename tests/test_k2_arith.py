"""CPU checks of the integer identities K2's folded residual arithmetic rests
on (csrc/flac_search16.hip, DESIGN 4a'''), over random and edge-case int32
accumulators and every shift the 16-bit search uses.

Reference residual: r = s - (sum c s >> sh), src/encoders/flac.c:1060-1126.
The fold gives acc with acc >> shv = n = ~r (arithmetic shift).  The biased
form (ATG_K2F_BIAS) keeps x = ((acc + 2^31) mod 2^32) >>> shv instead, sums
|r| as |x - (B - 1)| (B = 2^(31 - shv), one v_sad_u32) and recovers the Rice
code shift v >> kv in pass 2 as (n >> kv) ^ (n >> 31), n = x - B.
"""
import numpy as np


def _accs(rng, k):
    edge = np.array([-2**31, -2**31 + 1, -1, 0, 1, 2**31 - 1, -2**30, 2**30], dtype=np.int64)
    return np.concatenate([edge, rng.integers(-2**31, 2**31, size=k, dtype=np.int64)])


def test_biased_shift_is_offset_floor():
    rng = np.random.default_rng(7)
    acc = _accs(rng, 20000)
    for shv in range(0, 32):
        n = acc >> shv                                  # floor(acc / 2^shv)
        x = ((acc + 2**31) % 2**32) >> shv              # logical shift of the biased sum
        B = 1 << (31 - shv)
        assert np.array_equal(x, n + B)
        assert x.min() >= 0 and x.max() < 2 * B
        r = ~n                                          # n = ~r
        assert np.array_equal(np.abs(x - (B - 1)), np.abs(r))   # v_sad_u32(x, B - 1)


def test_pass2_code_shift_from_n():
    rng = np.random.default_rng(11)
    acc = _accs(rng, 20000)
    for shv in (0, 3, 12, 15, 20, 30, 31):
        n = acc >> shv
        v = n ^ (n >> 31)                               # |r| - [r < 0], the kept code
        assert np.all(v >= 0)
        for kv in range(0, 15):
            assert np.array_equal((n >> kv) ^ (n >> 31), v >> kv)


def test_warmup_sample_contributes_nothing():
    # lane 0's warm-up samples are forced to n = -1 (x = B - 1 in the biased
    # form, x = 2^31 - 1 with B = 2^31 in the split folds)
    for shv in range(0, 32):
        B = 1 << (31 - shv)
        x = B - 1
        assert abs(x - (B - 1)) == 0
        n = x - B
        assert n == -1 and ((n >> 5) ^ (n >> 31)) == 0
    x = (-1 & 0xFFFFFFFF) ^ 0x80000000
    assert x == 0x7FFFFFFF and x - 0x80000000 == -1
