"""CPU: the ReplayGain oracle (oracle/replaygain_port.c) on properties the
reference's algorithm fixes (window count, mono = duplicated stereo, 8-bit
input scaled by << 8, the 95th-percentile rule).  Parity unpinned: the
reference has no ReplayGain fixtures and replaygain.c is a Python-2 module."""
import math

import pytest

import numpy as np

import oracle_port as op


def tone(n, rate, ch, amp=0.5, bps=16):
    t = np.arange(n) / float(rate)
    x = amp * (np.sin(2 * np.pi * 441 * t) + 0.3 * np.sin(2 * np.pi * 4410 * t))
    x = np.round(x * (2 ** (bps - 1) - 1) / 1.3).astype(np.int32)
    return np.repeat(x[:, None], ch, 1).reshape(-1)


def test_window_count_and_gain_range():
    A, peak = op.rg_title(tone(441000, 44100, 2), 2, 16, 44100)
    assert A.sum() == 200          # 10 s / ceil(44100 * 0.05) = 2205-sample windows
    g = op.rg_gain(A)
    assert -30 < g < 30 and 0 < peak <= 1


def test_mono_is_duplicated_stereo():
    m = tone(50000, 48000, 1)
    s = np.repeat(m[:, None], 2, 1).reshape(-1)
    Am, pm = op.rg_title(m, 1, 16, 48000)
    As, ps = op.rg_title(s, 2, 16, 48000)
    assert np.array_equal(Am, As) and pm == ps


def test_8bit_is_shifted_16bit_filter_input():
    x8 = (tone(30000, 44100, 2, bps=8) // 2).astype(np.int32)
    A8, p8 = op.rg_title(x8, 2, 8, 44100)
    A16, p16 = op.rg_title(x8 << 8, 2, 16, 44100)
    assert np.array_equal(A8, A16)
    assert p8 == p16


def test_percentile_rule():
    A = np.zeros(12000, dtype=np.uint32)
    A[100] = 90
    A[5000] = 10                   # upper = ceil(100 * 0.05) = 5 -> bin 5000
    assert math.isclose(op.rg_gain(A), 64.82 - 50.0)
    assert math.isnan(op.rg_gain(np.zeros(12000, dtype=np.uint32)))


def test_rg_reader_oracle_invariants():
    m = op.rg_multiplier(-6.0, 0.9)
    assert math.isclose(m, 10 ** (-6.0 / 20), rel_tol=1e-15)
    assert op.rg_multiplier(3.0, 0.5) == 2.0          # amplifying gain -> 1 / peak
    rng = np.random.RandomState(3)
    x = rng.randint(-32768, 32768, size=2 * 5000).astype(np.int32)
    d = rng.bytes(2 * 5000 // 8 + 1)
    y = op.rg_apply(x, 2, 16, 2.0, 4096, d)
    base = np.clip(np.round(x.astype(np.float64) * 2.0), -32768, 32767).astype(np.int32)
    assert set(np.unique(y ^ base)) <= {0, 1}


def test_chunked_oracle_equals_default_for_4096_chunks():
    """the chunk-size form of the oracle reduces to the 4096-read form"""
    x = np.random.default_rng(3).integers(-30000, 30000, 2 * 20000).astype(np.int32)
    A0, p0 = op.rg_title(x, 2, 16, 44100)
    sizes = [4096] * 4 + [20000 - 4 * 4096]
    A1, p1 = op.rg_title(x, 2, 16, 44100, chunks=sizes)
    assert np.array_equal(A0, A1) and p0 == p1
    with pytest.raises(ValueError):
        op.rg_title(x, 2, 16, 44100, chunks=[100])
