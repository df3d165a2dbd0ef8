"""GPU parity for K2's packed pass-2 codes (flac_search16.hip PkStore /
ReSum, DESIGN 4a''''), byte for byte against the CPU oracle.

Pass 1 keeps the low 16 bits of each code (quiet lanes) or bits 8..23
(lanes the candidate's last finished job coded with k >= 9), and pass 2
uses them only when the wave's lane sums prove them exact; everything else
is recomputed.  These signals put each decision both ways inside one frame:

* bursts: loud noise in some 64-sample lane runs, near silence in others,
  so a wave mixes quiet and loud selectors and the hint of a lane can be
  wrong for the next order;
* a loud frame after a quiet one and the reverse (the hint is per frame);
* a pure tone whose low orders leave residuals past 2^15 while the high
  orders leave almost none (the hint from order 12 says quiet);
* samples with 1..7 wasted bits (shift + wasted bits past 15: B's low half
  is not zero, and past 23 the loud selector is refused);
* full-scale square waves and clipped noise (side channel past int16).
"""
import numpy as np
import pytest

import oracle_port
from test_gpu_flac import check_batch

pytestmark = pytest.mark.gpu

N = 4096 * 3 + 517  # three full frames and a short one


def _stereo(l, r):
    x = np.empty(2 * len(l), dtype=np.int32)
    x[0::2] = np.clip(l, -32768, 32767)
    x[1::2] = np.clip(r, -32768, 32767)
    return x


def _bursts(seed):
    g = np.random.default_rng(seed)
    amp = np.where((np.arange(N) // 64) % 3 == 0, 20000.0, 12.0)
    l = np.round(g.normal(0, 1, N) * amp)
    r = np.round(g.normal(0, 1, N) * amp[::-1])
    return _stereo(l, r)


def _frame_switch(seed):
    g = np.random.default_rng(seed)
    amp = np.where((np.arange(N) // 4096) % 2 == 0, 25.0, 15000.0)
    t = np.arange(N)
    l = np.round(3000 * np.sin(2 * np.pi * 440 * t / 44100) + g.normal(0, 1, N) * amp)
    r = np.round(g.normal(0, 1, N) * amp[::-1])
    return _stereo(l, r)


def _pure_tone(seed):
    t = np.arange(N)
    f = 3000.0 + 500.0 * seed
    l = np.round(30000 * np.sin(2 * np.pi * f * t / 44100))
    r = np.round(29000 * np.sin(2 * np.pi * f * 1.01 * t / 44100 + 0.3))
    return _stereo(l, r)


def _wasted(seed, w):
    g = np.random.default_rng(seed)
    t = np.arange(N)
    base = 32767 >> w
    l = np.round(base * 0.7 * np.sin(2 * np.pi * 220 * t / 44100) + g.normal(0, 3, N))
    r = np.round(base * 0.5 * np.sin(2 * np.pi * 330 * t / 44100) + g.normal(0, 40, N))
    l = np.clip(l, -(base + 1), base).astype(np.int64) << w
    r = np.clip(r, -(base + 1), base).astype(np.int64) << w
    return _stereo(l, r)


def _square_clip(seed):
    g = np.random.default_rng(seed)
    t = np.arange(N)
    l = np.where((t // 37) % 2 == 0, 32767, -32768).astype(np.float64)
    r = np.clip(np.round(g.normal(0, 30000, N)), -32768, 32767)
    return _stereo(l, r)


@pytest.mark.parametrize("seed", [1, 2])
def test_packed_codes_mixed_lanes(gpu_engine, seed):
    opts = dict(oracle_port.PRESETS["8"])
    check_batch(gpu_engine, [_bursts(seed), _frame_switch(seed), _pure_tone(seed)], 2, 16, opts)


def test_packed_codes_wasted_bits(gpu_engine):
    opts = dict(oracle_port.PRESETS["8"])
    check_batch(gpu_engine, [_wasted(3, w) for w in range(1, 8)], 2, 16, opts)


def test_packed_codes_full_scale(gpu_engine):
    opts = dict(oracle_port.PRESETS["8"])
    check_batch(gpu_engine, [_square_clip(4), _square_clip(5)], 2, 16, opts)


def test_packed_codes_mixed_batch(gpu_engine):
    # every kind in one batch: frames of different kinds share workgroups'
    # CUs and the hint never leaks across frames
    opts = dict(oracle_port.PRESETS["8"])
    pcms = [_bursts(7), _square_clip(8), _wasted(9, 5), _pure_tone(3), _frame_switch(9)]
    check_batch(gpu_engine, pcms, 2, 16, opts)
