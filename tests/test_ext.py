"""CPU: the compiled CPython extensions (audiotools._encoders_c,
audiotools._decoders_c) import, keep the reference's argument parsing and
error behaviour (src/encoders/flac.c:52-121, src/decoders/flac.c:28-98) and
write the reference's bytes where no GPU call is needed (an empty stream).
The encode/decode paths themselves run in tests/test_gpu_ext.py."""
import os

import numpy as np
import pytest

import audiotools
import oracle_port
from audiotools import _decoders_c, _encoders_c

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_extensions_link_libatgpu():
    import subprocess
    for m in (_encoders_c, _decoders_c):
        out = subprocess.run(["ldd", m.__file__], capture_output=True, text=True).stdout
        assert "libatgpu.so" in out and "not found" not in out


def test_encode_flac_signature_errors(tmp_path):
    r = audiotools.FrameListReader(np.zeros(20, np.int32), 44100, 2, 16)
    with pytest.raises(TypeError):
        _encoders_c.encode_flac(str(tmp_path / "x.flac"), r)          # too few arguments
    with pytest.raises(OSError) as e:
        _encoders_c.encode_flac("/nonexistent-dir/x.flac", r, 4096, 12, 0, 6)
    assert e.value.filename == "/nonexistent-dir/x.flac"


class _NotFrameList(object):
    sample_rate, channels, bits_per_sample, channel_mask = 44100, 2, 16, 3

    def read(self, n):
        return [0, 0]

    def close(self):
        pass


def test_encode_flac_reader_contract(tmp_path):
    with pytest.raises(TypeError):
        _encoders_c.encode_flac(str(tmp_path / "x.flac"), _NotFrameList(), 4096, 12, 0, 6)
    r = audiotools.PCMReaderError(u"boom", 44100, 2, 3, 16)
    with pytest.raises(ValueError):
        _encoders_c.encode_flac(str(tmp_path / "y.flac"), r, 4096, 12, 0, 6)


@pytest.mark.parametrize("padding", [4096, 0, 77])
def test_encode_flac_empty_stream_matches_oracle(tmp_path, padding):
    """no frames: the header alone (host code), byte-identical to the oracle"""
    r = audiotools.FrameListReader(np.zeros(0, np.int32), 44100, 2, 16)
    fn = str(tmp_path / "e.flac")
    opts = dict(oracle_port.PRESETS["8"], padding_size=padding)
    assert _encoders_c.encode_flac(fn, r, **opts) == []
    want, _ = oracle_port.encode(np.zeros(0, np.int32), 2, 16, 44100, **opts)
    assert open(fn, "rb").read() == want


def test_flac_decoder_metadata_errors(tmp_path):
    with pytest.raises(ValueError):
        _decoders_c.FlacDecoder(b"RIFF" + b"\0" * 100)
    with pytest.raises(IOError):
        _decoders_c.FlacDecoder(b"fLaC\x00\x00")
    d = _decoders_c.FlacDecoder(os.path.join(GOLDEN, "tone.flac"))
    assert (d.sample_rate, d.bits_per_sample, d.channels, d.channel_mask) == (44100, 16, 2, 3)
    with pytest.raises(TypeError):
        _decoders_c.FlacDecoder(open(os.path.join(GOLDEN, "tone.flac"), "rb").read()).seek(0)
