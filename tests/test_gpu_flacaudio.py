"""GPU: FlacAudio.from_pcm (audiotools/flac.py) finishes the GPU encoder's
output the way the reference's flac.py does.  Pin: the reference's own
fixture test/tone.flac (written by the reference's from_pcm: STREAMINFO,
SEEKTABLE, VORBIS_COMMENT, PADDING 4096, frames) is reproduced byte for byte
from its PCM, except the vendor version inside VORBIS_COMMENT ("2.21alpha1"
there, "2.22alpha1" = this build's reference version; same length)."""
import os

import numpy as np
import pytest

import oracle_port
import signals

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_tone_flac_whole_file(tmp_path):
    import audiotools
    from audiotools import flac
    ref = open(os.path.join(HERE, "golden", "tone.flac"), "rb").read()
    pcm, ch, bps, rate = oracle_port.decode(ref)
    assert (ch, bps, rate) == (2, 16, 44100)
    fn = str(tmp_path / "tone.flac")
    out = flac.FlacAudio.from_pcm(fn, audiotools.FrameListReader(pcm, rate, ch, bps, 0x3),
                                  "8", total_pcm_frames=len(pcm) // ch)
    got = open(fn, "rb").read()
    want = ref.replace(b"Python Audio Tools 2.21alpha1", b"Python Audio Tools 2.22alpha1")
    assert got == want
    assert out.total_frames() == len(pcm) // ch


def test_multichannel_mask_tag_and_round_trip(tmp_path):
    import audiotools
    from audiotools import _atgpu, flac
    n = 44100 * 12 + 333
    pcm = signals.make("tone", n, 6, 16, seed=4)
    fn = str(tmp_path / "six.flac")
    a = flac.FlacAudio.from_pcm(fn, audiotools.FrameListReader(pcm, 44100, 6, 16, 0),
                                "5", total_pcm_frames=n)
    data = open(fn, "rb").read()
    blocks, frames_at = flac._blocks(data)
    types = [t for t, _ in blocks]
    assert types == [flac.STREAMINFO, flac.SEEKTABLE, flac.VORBIS_COMMENT, flac.PADDING]
    assert b"WAVEFORMATEXTENSIBLE_CHANNEL_MASK=0x003F" in blocks[2][1]
    # 2 seekpoints (0 s and 10 s) planned in the padding: the file's metadata
    # is exactly the encoder's plus nothing -- padding absorbed the growth
    rc, si, pts = _atgpu.read_metadata(data)
    assert rc == 0 and si.channel_mask == 0x3F and len(pts) == 2
    assert pts[0][:2] == (0, 0)
    dec = a.to_pcm()
    got = []
    while True:
        fl = dec.read(4096)
        if not len(fl):
            break
        got.append(fl.samples)
    assert np.array_equal(np.concatenate(got), pcm)
    assert a.to_pcm().offsets()[0][0] == 0
