"""GPU parity for the multi-wave frame pack (flac_frame.hip
k_frame_pack<T, false, NW>), byte for byte against the
CPU oracle.

A frame's subframes are packed by up to four waves at once, each starting
at the header plus the searched sizes of the subframes before it.  The
wave count follows the channel count (3 -> 3 waves, 4 -> 4, 5 -> 3 in two
rounds, 7 and 8 -> 4 in two rounds) and drops when the frame image and the
waves' staging pass the CU's LDS (7 and 8 channels of 24-bit: 3 waves);
neighbouring subframes share the words their bit ranges meet in.  Every
channel count 1-8 at 16 and 24 bits, with signals whose subframes take
every type (CONSTANT silence, VERBATIM noise, FIXED / LPC tones and
chirps, wasted bits) so subframe sizes and boundaries vary within a frame.
"""
import numpy as np
import pytest

import oracle_port
import signals
from test_gpu_flac import check_batch

pytestmark = pytest.mark.gpu


def _mixed(n, ch, bps, seed):
    # a different signal kind per channel: the subframes of one frame
    # differ in type and size, so the waves' starts are all different
    kinds = ["tone", "noise", "silence", "chirp", "sine", "wasted"]
    cols = []
    for c in range(ch):
        x = signals.make(kinds[(c + seed) % len(kinds)], n, 1, bps, seed=seed * 10 + c)
        cols.append(x.reshape(-1))
    return np.stack(cols, axis=1).reshape(-1)


@pytest.mark.parametrize("channels", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("bps", [16, 24])
def test_pack_waves_vs_oracle(gpu_engine, channels, bps):
    opts = dict(oracle_port.PRESETS["8"])
    n = 2 * 4096 + 1234
    pcms = [_mixed(n, channels, bps, s) for s in range(3)]
    pcms.append(signals.make("tone", n, channels, bps, seed=77))
    check_batch(gpu_engine, pcms, channels, bps, opts)


@pytest.mark.parametrize("preset", ["0", "3", "6"])
def test_pack_waves_presets(gpu_engine, preset):
    opts = dict(oracle_port.PRESETS[preset])
    n = 3 * opts["block_size"] + 99
    for channels, bps in ((5, 16), (8, 24)):
        check_batch(gpu_engine, [_mixed(n, channels, bps, 4)], channels, bps, opts)
