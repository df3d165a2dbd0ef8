"""GPU: the drop-in under track2track / trackverify.

track2track's per-file step is `AudioFile.convert(target, FlacAudio, "8")`
(reference audiotools/__init__.py:3760-3774; FlacAudio's override
flac.py:2360-2398) and trackverify's is `AudioFile.verify()`
(__init__.py:3939-3970).  Here both run through the GPU encoder and
decoders:

  * the reference's test/wav-2ch.wav converted to FLAC-8 has the reference
    encoder's frame bytes (sha256 a561eba0...) and verifies;
  * the reference's flac-id3.flac / flac-id3-2.flac (ID3v2-prefixed, one
    with an ID3v1 tail) verify, and their PCM MD5 equals what the reference
    decoder wrote (tests/golden/id3_vectors.json; flac-id3.flac's is also
    the reference's own tracklint known answer 9a0ab096...);
  * truncated and corrupted FLAC files raise InvalidFile; a file removed
    after FlacAudio opened it gives a PCMReaderError and InvalidFile;
  * FLAC -> WAV and ALAC -> FLAC conversions through the same calls.
"""
import hashlib
import json
import os

import pytest

import oracle_port

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "fixtures")
WAV2 = os.path.join(HERE, "golden", "wav-2ch.wav")
ID3 = json.load(open(os.path.join(HERE, "golden", "id3_vectors.json")))


def _pcm_md5(audiofile):
    import audiotools
    h = hashlib.md5()
    r = audiofile.to_pcm()
    audiotools.transfer_framelist_data(r, h.update)
    r.close()
    return h.hexdigest()


def test_wav_2ch_convert_flac8_matches_reference(tmp_path):
    import audiotools
    w = audiotools.WaveAudio(WAV2)
    seen = []
    out = w.convert(str(tmp_path / "w.flac"), audiotools.FlacAudio, "8",
                    progress=lambda cur, tot: seen.append((cur, tot)))
    assert isinstance(out, audiotools.FlacAudio)
    data = open(out.filename, "rb").read()
    _, frames = oracle_port.split_flac(data)
    assert hashlib.sha256(frames).hexdigest() == (
        "a561eba098e65ef2f77c4ee434547051edede0b5191c061da8ce482cabfccf34")
    assert seen[-1] == (20, 20)
    assert out.verify() is True
    prog = []
    assert out.verify(progress=lambda cur, tot: prog.append((cur, tot))) is True
    assert prog[-1] == (20, 20)
    assert out == w and w == out
    assert int(out.channel_mask()) == 0x3


@pytest.mark.parametrize("name", sorted(ID3))
def test_id3_prefixed_flac_verifies_with_reference_pcm(name):
    import audiotools
    v = ID3[name]
    f = audiotools.FlacAudio(os.path.join(FIX, name))
    assert (f.channels(), f.bits_per_sample(), f.total_frames()) == (
        v["channels"], v["bits_per_sample"], v["pcm_frames"])
    assert f.verify() is True
    assert _pcm_md5(f) == v["pcm_md5"]
    assert int(f.channel_mask()) == 0x3


def test_flac_id3_tracklint_known_answer():
    """the reference's own known answer for this fixture's PCM
    (test/test_utils.py:3383-3406)"""
    import audiotools
    f = audiotools.FlacAudio(os.path.join(FIX, "flac-id3.flac"))
    assert _pcm_md5(f) == "9a0ab096c517a627b0ab5a0b959e5f36"


def test_truncated_and_corrupt_flac_raise_invalid_file(tmp_path):
    import audiotools
    w = audiotools.WaveAudio(WAV2)
    good = w.convert(str(tmp_path / "g.flac"), audiotools.FlacAudio, "8")
    data = open(good.filename, "rb").read()
    _, frames = oracle_port.split_flac(data)
    first = len(data) - len(frames)
    fn = str(tmp_path / "t.flac")
    # the file shrinks after FlacAudio read its metadata
    open(fn, "wb").write(data)
    track = audiotools.FlacAudio(fn)
    for cut in (first + 1, first + len(frames) // 2, len(data) - 1):
        open(fn, "wb").write(data[:cut])
        with pytest.raises(audiotools.InvalidFile):
            track.verify()
    # a flipped byte inside the frame: CRC or MD5 failure
    bad = bytearray(data)
    bad[first + len(frames) // 2] ^= 0x55
    open(fn, "wb").write(bytes(bad))
    with pytest.raises(audiotools.InvalidFile):
        audiotools.FlacAudio(fn).verify()
    # a file cut inside its metadata cannot be opened at all
    open(fn, "wb").write(data[:20])
    with pytest.raises(audiotools.InvalidFile):
        audiotools.FlacAudio(fn)


def test_flac_removed_after_open_gives_pcmreadererror(tmp_path):
    import audiotools
    w = audiotools.WaveAudio(WAV2)
    f = w.convert(str(tmp_path / "g.flac"), audiotools.FlacAudio, "8")
    os.unlink(f.filename)
    r = f.to_pcm()
    assert isinstance(r, audiotools.PCMReaderError)
    assert (r.sample_rate, r.channels, r.bits_per_sample, r.channel_mask) == (44100, 2, 16, 3)
    with pytest.raises(audiotools.InvalidFile):
        f.verify()
    with pytest.raises(audiotools.EncodingError):
        f.convert(str(tmp_path / "x.flac"), audiotools.FlacAudio, "8")
    assert not os.path.exists(str(tmp_path / "x.flac"))


@pytest.mark.parametrize("name", ["wav-1ch.wav", "wav-6ch.wav", "wav-8bit.wav"])
def test_wave_fixtures_convert_to_flac_and_back(name, tmp_path):
    """the reference's other WAVE fixtures through WAV -> FLAC -> WAV:
    the FLAC verifies, and the WAVE written from it is the fixture byte for
    byte (FlacAudio.convert -> WaveAudio.from_pcm)"""
    import audiotools
    src = audiotools.WaveAudio(os.path.join(FIX, name))
    f = src.convert(str(tmp_path / "a.flac"), audiotools.FlacAudio, "8")
    assert f.verify() is True
    assert f.total_frames() == src.total_frames()
    assert f == src
    assert int(f.channel_mask()) == int(src.channel_mask())
    back = f.convert(str(tmp_path / "b.wav"), audiotools.WaveAudio)
    assert open(back.filename, "rb").read() == open(src.filename, "rb").read()
    assert back.verify() is True


@pytest.mark.parametrize("name", sorted(ID3))
def test_id3_flac_convert_to_wav(name, tmp_path):
    import audiotools
    f = audiotools.FlacAudio(os.path.join(FIX, name))
    w = f.convert(str(tmp_path / "o.wav"), audiotools.WaveAudio)
    assert w.verify() is True
    data = open(w.filename, "rb").read()
    assert hashlib.md5(data[44:44 + w.total_frames() * 4]).hexdigest() == ID3[name]["pcm_md5"]


def test_alac_convert_to_flac_and_verify(tmp_path):
    """the config-5 chain's source side: ALAC (GPU decode) -> FLAC-8 (GPU
    encode), both files verify and carry the same PCM"""
    import audiotools
    a = audiotools.ALACAudio(os.path.join(FIX, "alac-allframes.m4a"))
    assert a.verify() is True
    f = a.convert(str(tmp_path / "a.flac"), audiotools.FlacAudio, "8")
    assert f.verify() is True
    assert f == a
    assert audiotools.pcm_frame_cmp(a.to_pcm(), f.to_pcm()) is None


def test_invalid_alac_raises_invalid_file(tmp_path):
    import audiotools
    fn = str(tmp_path / "x.m4a")
    open(fn, "wb").write(open(os.path.join(FIX, "alac-allframes.m4a"), "rb").read()[:100])
    with pytest.raises(audiotools.InvalidFile):
        audiotools.ALACAudio(fn)
