"""GPU parity for the large-frame path (csrc/flac_big.hip): block sizes
4097..65535 and residual partition orders 7..15, which the reference encoder
accepts (src/encoders/flac.c:1326-1505; test/test_formats.py:3798-3844
encodes 32768- and 65535-sample blocks of noise and silence).

Pinned twice: the 90 reference-encoder hashes of
tests/golden/flac_vectors_big.json (make_golden_big.py), and byte identity
with the CPU oracle on batches shaped like the reference's
test_noise_silence.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_port
import signals
from test_gpu_flac import check_batch, gpu_encode_tracks

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
VECS = json.load(open(os.path.join(GOLDEN, "flac_vectors_big.json")))["vectors"]


@pytest.mark.parametrize("part", range(6))
def test_golden_big_vectors(gpu_engine, part):
    for v in VECS[part::6]:
        pcm = signals.make(v["kind"], v["n"], v["channels"], v["bps"], seed=v["seed"])
        (img, _), = gpu_encode_tracks(gpu_engine, [pcm], v["channels"], v["bps"], 44100,
                                      v["opts"])
        assert len(img) == v["bytes"], v["name"]
        assert hashlib.sha256(img).hexdigest() == v["sha256"], v["name"]


@pytest.mark.parametrize("block_size", [32, 32768, 65535])
@pytest.mark.parametrize("channels", [1, 2, 4, 8])
def test_noise_silence(gpu_engine, block_size, channels):
    """test/test_formats.py:3798-3844: 65536 frames of random PCM and of
    silence, 8/16/24 bits, the disable-subframe variants, with and without
    the exhaustive model search"""
    for bps in (8, 16, 24):
        for disable in [{}, dict(disable_verbatim_subframes=True,
                                 disable_constant_subframes=True),
                        dict(disable_verbatim_subframes=True,
                             disable_constant_subframes=True,
                             disable_fixed_subframes=True)]:
            for exhaustive in (False, True):
                opts = dict(oracle_port.PRESETS["8"])
                opts.update(disable, block_size=block_size,
                            exhaustive_model_search=exhaustive)
                pcms = [signals.noise(65536, channels, bps, 11 * channels + bps),
                        np.zeros(65536 * channels, np.int32)]
                check_batch(gpu_engine, pcms, channels, bps, opts)


@pytest.mark.parametrize("porder", [7, 9, 12, 15])
def test_deep_partition_orders(gpu_engine, porder):
    """many tracks per batch (persistent grid, frames sharing output words)"""
    opts = dict(block_size=32768, max_lpc_order=12, min_residual_partition_order=0,
                max_residual_partition_order=porder, mid_side=True,
                adaptive_mid_side=False, exhaustive_model_search=porder % 2 == 1)
    rng = np.random.default_rng(porder)
    pcms = []
    for k, kind in enumerate(["tone", "chirp", "noise", "wasted", "sine", "silence", "tone"]):
        n = int(rng.integers(1000, 3 * 32768))
        pcms.append(signals.make(kind, n, 2, 16, seed=100 * porder + k))
    check_batch(gpu_engine, pcms, 2, 16, opts)


def test_big_and_small_frames_mixed(gpu_engine):
    """4096-sample presets stay on the LDS kernels; one track with a frame
    above 4096 (explicit read sizes) sends the whole batch to flac_big"""
    opts = dict(oracle_port.PRESETS["8"])
    opts["block_size"] = 8192
    pcm = signals.make("tone", 30000, 2, 16, seed=9)
    sizes = [8192, 5000, 8192, 300, 4096, 4220]
    got = gpu_encode_tracks(gpu_engine, [pcm, pcm[:2 * 9000]], 2, 16, 44100, opts,
                            frame_sizes=[sizes, None])
    img, lst = got[0]
    assert [n for _, n in lst] == sizes
    want, wlst = oracle_port.encode(pcm, 2, 16, 44100, frame_sizes=sizes, **opts)
    assert img == want and lst == wlst
    dec, ch, b, r = oracle_port.decode(img)
    assert np.array_equal(dec, pcm)
    want, wlst = oracle_port.encode(pcm[:2 * 9000], 2, 16, 44100, **opts)
    assert got[1][0] == want and got[1][1] == wlst


def test_big_frames_decode_on_gpu(gpu_engine):
    """GPU encode -> GPU FlacDecoder of 65535-sample frames (MD5 verified
    by the decoder at end of stream)"""
    from audiotools import decoders
    opts = dict(oracle_port.PRESETS["8"])
    opts["block_size"] = 65535
    pcms = [signals.make(k, 200000, 2, 16, seed=i) for i, k in
            enumerate(["tone", "noise", "chirp"])]
    got = gpu_encode_tracks(gpu_engine, pcms, 2, 16, 44100, opts)
    for p, (img, _) in zip(pcms, got):
        dec = decoders.FlacDecoder(img)
        parts = []
        while True:
            fl = dec.read(65536)
            if not len(fl):
                break
            parts.append(np.asarray(fl.samples, dtype=np.int32))
        dec.close()
        assert np.array_equal(np.concatenate(parts), p)
