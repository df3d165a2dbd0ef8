"""CPU: libatgpu's host-side FLAC metadata reader (atg_flac_read_metadata,
the decoder's restatement of flacdec_read_metadata, src/decoders/flac.c:
568-707) agrees with the oracle on every golden decode case -- same return
code and, when it succeeds, the same STREAMINFO, channel mask, first-frame
offset and SEEKTABLE.  Host code only; no GPU needed."""
import decode_cases
import oracle_port

from audiotools import _atgpu

CASES = decode_cases.load_cases()

FIELDS = ("min_block_size", "max_block_size", "min_frame_size", "max_frame_size",
          "sample_rate", "channels", "bits_per_sample", "channel_mask",
          "total_samples", "frames_offset", "n_seekpoints")


def test_metadata_matches_oracle():
    seen = 0
    for c in CASES:
        data = decode_cases.case_bytes(c)
        rc, si, pts = _atgpu.read_metadata(data)
        orc, info, opts, _ = oracle_port.read_metadata(data)
        assert rc == orc, c["name"]
        if rc:
            continue
        seen += 1
        for f in FIELDS:
            assert getattr(si, f) == info[f], (c["name"], f)
        assert bytes(si.md5) == info["md5"], c["name"]
        assert pts == opts, c["name"]
    assert seen > 500


def test_metadata_errors():
    assert _atgpu.read_metadata(b"")[0] == 2
    assert _atgpu.read_metadata(b"RIFF....")[0] == 1
    data = open(decode_cases.FIX + "/tone1.flac", "rb").read()
    assert _atgpu.read_metadata(data[:20])[0] == 2
