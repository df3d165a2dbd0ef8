"""GPU: BASELINE config 1 on the product path -- the reference's
test/wav-2ch.wav through audiotools.wav.WaveReader (reference
audiotools/wav.py:421-553) -> BufferedPCMReader -> encoders.encode_flac
(GPU) at FLAC-8.  Pinned to the reference encoder's output for that file
(whole file sha256 bf481da9..., frame region a561eba0...)."""
import hashlib
import os

import pytest

import oracle_port

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WAV = os.path.join(HERE, "golden", "wav-2ch.wav")


def test_wav_2ch_flac8_matches_reference(tmp_path):
    import audiotools
    from audiotools import encoders, wav
    fn = str(tmp_path / "wav-2ch.flac")
    reader = wav.WaveReader(WAV)
    offsets = encoders.encode_flac(fn, audiotools.BufferedPCMReader(reader),
                                   **oracle_port.PRESETS["8"])
    data = open(fn, "rb").read()
    assert len(data) == 4204
    assert hashlib.sha256(data).hexdigest() == (
        "bf481da91f617d3ae3b4d6d2cb1f28d6f13146d2c62f90ff0f097099e8d9beb6")
    _, frames = oracle_port.split_flac(data)
    assert hashlib.sha256(frames).hexdigest() == (
        "a561eba098e65ef2f77c4ee434547051edede0b5191c061da8ce482cabfccf34")
    assert offsets == [(0, 20)]


def test_wav_to_flac_round_trip_via_wave_audio(tmp_path):
    """WaveAudio.to_pcm() -> FlacAudio.from_pcm -> FlacDecoder, exact PCM"""
    import numpy as np
    from audiotools import flac, wav
    w = wav.WaveAudio(WAV)
    fn = str(tmp_path / "w.flac")
    a = flac.FlacAudio.from_pcm(fn, w.to_pcm(), "8", total_pcm_frames=w.total_frames())
    r = w.to_pcm()
    want = r.read(1000).samples
    r.close()
    dec = a.to_pcm()
    got = dec.read(4096).samples
    assert np.array_equal(got, want)
    assert len(dec.read(4096)) == 0
