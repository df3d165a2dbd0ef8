"""GPU parity for the wide-sample search's code-range check
(flac_search16.hip eval_fold_hl<true>), byte for byte against
the CPU oracle.

24-bit predictors whose codes cannot be bounded below 2^26 in advance
(|s| (1 + sum|c| / 2^sh) is past 2^25 for loud audio) are evaluated on the
folded 32-bit path and checked after pass 1; a job with a residual outside
[-2^25, 2^25) is redone with 64-bit sums.  These signals take each branch,
and both inside one frame:

* loud tones (0.7-0.95 full scale) with little noise: small residuals, the
  check passes;
* loud tones with one 64-sample run of full-scale noise: one lane's
  residuals leave the range, the whole job is redone wide;
* full-scale white noise: low orders fail the check, VERBATIM competes;
* a tone whose frames alternate loud / quiet (the bound passes in advance
  for the quiet frames);
* loud tones under heavy noise (sigma 2^16 .. 2^18): Rice parameters past
  14, so the partitions take RICE2's 5-bit parameters (the method is chosen
  after the partition search, as the reference does).
"""
import numpy as np
import pytest

import oracle_port
from test_gpu_flac import check_batch

pytestmark = pytest.mark.gpu

B = 4096
N = 3 * B + 211
FS = (1 << 23) - 1


def _interleave(chans):
    x = np.stack(chans, axis=1).reshape(-1)
    return np.clip(np.round(x), -FS - 1, FS).astype(np.int32)


def _tone(rng, n, amp, f):
    t = np.arange(n)
    return amp * FS * np.sin(2 * np.pi * f * t / 48000 + rng.uniform(0, 6.28)) + rng.normal(0, 40, n)


def _loud(rng, ch):
    return _interleave([_tone(rng, N, rng.uniform(0.7, 0.95), rng.uniform(80, 4000))
                        for _ in range(ch)])


def _burst(rng, ch):
    chans = []
    for c in range(ch):
        x = _tone(rng, N, 0.9, rng.uniform(80, 3000))
        at = int(rng.integers(0, 63)) * 64 + B * (c % 3)
        x[at:at + 64] = rng.uniform(-FS, FS, 64)
        chans.append(x)
    return _interleave(chans)


def _noise(rng, ch):
    return _interleave([rng.uniform(-FS, FS, N) for _ in range(ch)])


def _alternate(rng, ch):
    amp = np.where((np.arange(N) // B) % 2 == 0, 0.9, 0.002)
    return _interleave([_tone(rng, N, 1.0, rng.uniform(200, 2000)) * amp for _ in range(ch)])


def _rice2(rng, ch):
    return _interleave([_tone(rng, N, 0.5, rng.uniform(80, 3000)) +
                        rng.normal(0, 2.0 ** rng.uniform(16, 18), N) for _ in range(ch)])


@pytest.mark.parametrize("channels", [2, 6])
def test_code_range_check(gpu_engine, channels):
    rng = np.random.default_rng(0x24B + channels)
    pcms = [_loud(rng, channels), _burst(rng, channels), _noise(rng, channels),
            _alternate(rng, channels), _rice2(rng, channels)]
    check_batch(gpu_engine, pcms, channels, 24, dict(oracle_port.PRESETS["8"]), rate=48000)


def test_code_range_check_presets(gpu_engine):
    rng = np.random.default_rng(0x24C)
    pcms = [_loud(rng, 2), _burst(rng, 2)]
    for preset in ("5", "6", "7"):
        check_batch(gpu_engine, pcms, 2, 24, dict(oracle_port.PRESETS[preset]), rate=48000)
