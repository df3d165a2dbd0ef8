"""GPU parity of the decoder's frame-end hypothesis (flac_decode.hip
k_dec_spec; atg_decoder_set_frame_hypothesis).

The parse takes a frame's end from the next frame-header candidate whose
bytes carry a zero CRC-16 residue and skips walking the frame's last
subframe; the restore checks the hypothesis on the subframe it walks, and a
batch with a failed check is redone with every subframe walked.  The results
must be the full parse's (the reference's read() loop,
src/decoders/flac.c:174-285) in every mode:

* mode 0 (every subframe walked: the path the golden tests pinned), 1 (the
  default) and 2 (every batch redone) give identical results, PCM, frame
  offsets and block sizes on every golden case of
  tests/golden/flac_decode_vectors.json (the reference's fixtures and their
  seeded corruptions) and on GPU-encoded streams;
* a stream whose first frame is followed by two zero bytes: the hypothesis
  for that frame (the next frame's header, residue still zero) is wrong, the
  restore's check catches it, the batch is redone, and the results are the
  full parse's.
"""
import numpy as np
import pytest

import decode_cases
import oracle_port
import signals

pytestmark = pytest.mark.gpu

CASES = decode_cases.load_cases()


def _batch(datas):
    from audiotools import _atgpu
    tracks, parts, pos = [], [], 0
    for d in datas:
        rc, si, _ = _atgpu.read_metadata(d)
        if rc:
            continue
        body = d[si.frames_offset:]
        pad = (-len(body)) % 4
        tracks.append(_atgpu.dec_track(pos, len(body), si))
        parts.append(body + b"\0" * pad)
        pos += len(body) + pad
    return tracks, b"".join(parts)


def _key(r):
    return (r.status, r.pcm_frames, r.n_frames, bytes(r.md5), r.walk_end, r.walk_frames,
            r.walk_status, r.first_frame, r.pcm_offset)


def _decode_modes(blob, tracks, modes=(0, 1, 2)):
    from audiotools import _atgpu
    out = {}
    for mode in modes:
        dec = _atgpu.Decoder(0)
        dec.set_frame_hypothesis(mode)
        pcm, res, offs, bss = dec.decode(blob, tracks)
        out[mode] = ([_key(r) for r in res], pcm.copy(), offs.copy(), bss.copy(),
                     dec.frame_hypothesis_redos())
        dec.close()
    return out


def _same(a, b):
    assert a[0] == b[0]
    assert np.array_equal(a[1], b[1])
    assert np.array_equal(a[2], b[2])
    assert np.array_equal(a[3], b[3])


def test_modes_agree_on_golden_cases():
    datas = [decode_cases.case_bytes(c) for c in CASES if c["file"] != "1h.flac"]
    tracks, blob = _batch(datas)
    got = _decode_modes(blob, tracks)
    _same(got[0], got[1])
    _same(got[0], got[2])
    assert got[0][4] == 0
    assert got[2][4] == 1  # the self-check mode redid the batch


def test_modes_agree_on_encoded_streams(gpu_engine):
    from audiotools import _atgpu
    datas = []
    for i, (kind, ch, bps, preset) in enumerate([("tone", 2, 16, "8"), ("noise", 2, 16, "8"),
                                                  ("chirp", 1, 16, "5"), ("sine", 6, 16, "8"),
                                                  ("silence", 2, 24, "0"), ("tone", 2, 8, "2")]):
        pcm = signals.make(kind, 4096 * 5 + 333 * i, ch, bps, seed=40 + i)
        opts = _atgpu.make_options(**oracle_port.PRESETS[preset])
        dtype = np.int16 if bps <= 16 else np.int32
        out, res, _, _ = gpu_engine.encode(opts, pcm.astype(dtype), [(0, len(pcm) // ch)], ch,
                                           bps, 44100)
        datas.append(out[res[0].out_offset:res[0].out_offset + res[0].bytes].tobytes())
    tracks, blob = _batch(datas)
    got = _decode_modes(blob, tracks)
    _same(got[0], got[1])
    _same(got[0], got[2])
    assert got[1][4] == 0
    assert all(k[0] == 0 for k in got[1][0])


def test_wrong_hypothesis_is_caught_and_redone(gpu_engine):
    """two zero bytes after the first frame: CRC-16 over the first frame and
    the zeros is still 0, so the hypothesis ends the frame at the next
    header -- two bytes past its true end.  The restore's walk of the last
    subframe ends elsewhere: the batch is redone with the full parse, which
    stops at the junk as the reference's read() does"""
    from audiotools import _atgpu
    opts = _atgpu.make_options(**oracle_port.PRESETS["8"])
    pcm = signals.make("chirp", 4096 * 4, 2, 16, seed=77)
    out, res, _, _ = gpu_engine.encode(opts, pcm.astype(np.int16), [(0, len(pcm) // 2)], 2, 16,
                                       44100)
    img = out[res[0].out_offset:res[0].out_offset + res[0].bytes].tobytes()
    rc, si, _ = _atgpu.read_metadata(img)
    assert rc == 0
    tracks, blob = _batch([img])
    _, _, offs, _ = _atgpu.Decoder(0).decode(blob, tracks)
    cut = si.frames_offset + int(offs[1])  # the second frame's first byte
    bad = img[:cut] + b"\0\0" + img[cut:]
    tracks, blob = _batch([bad])
    got = _decode_modes(blob, tracks, modes=(0, 1))
    _same(got[0], got[1])
    assert got[1][4] == 1  # the hypothesis failed its check: one redo
    assert got[0][0][0][0] != 0  # the full parse stops at the junk


@pytest.mark.parametrize("depth", [3, 6])
def test_redo_inside_a_pipeline(gpu_engine, depth):
    """device batches in flight (rolled MD5 from 4 on), every other batch
    holding the stream whose first frame is followed by junk: the failed
    check redoes that batch inside its decode_wait while the others stay in
    flight; every batch's results and PCM equal the full parse's"""
    import torch
    from audiotools import _atgpu
    opts = _atgpu.make_options(**oracle_port.PRESETS["8"])
    pcm = signals.make("tone", 4096 * 6 + 55, 2, 16, seed=12)
    out, res, _, _ = gpu_engine.encode(opts, pcm.astype(np.int16), [(0, len(pcm) // 2)], 2, 16,
                                       44100)
    img = out[res[0].out_offset:res[0].out_offset + res[0].bytes].tobytes()
    rc, si, _ = _atgpu.read_metadata(img)
    tracks, blob = _batch([img])
    _, _, offs, _ = _atgpu.Decoder(0).decode(blob, tracks)
    cut = si.frames_offset + int(offs[1])
    bad = img[:cut] + b"\0\0" + img[cut:]
    batches = [_batch([img, bad, img]), _batch([img, img])]
    dev = []
    for tr, bl in batches:
        d = torch.frombuffer(bytearray(bl + b"\0" * 64), dtype=torch.uint8).cuda()
        dev.append((d, len(bl), tr))
    torch.cuda.synchronize()
    ref = _atgpu.Decoder(0)
    ref.set_frame_hypothesis(0)
    want = [[_key(r) for r in ref.decode_device(d.data_ptr(), n, tr)[0]] for d, n, tr in dev]
    ref.close()
    dec = _atgpu.Decoder(0)
    dec.set_inflight(depth)
    pending = []
    for i in range(depth + 4):
        if len(pending) == depth:
            j, t = pending.pop(0)
            got, _, _ = dec.decode_wait(t)
            assert [_key(r) for r in got] == want[j % 2], j
        d, n, tr = dev[i % 2]
        pending.append((i, dec.decode_device_async(d.data_ptr(), n, tr)))
    for j, t in pending:
        got, _, _ = dec.decode_wait(t)
        assert [_key(r) for r in got] == want[j % 2], j
    # one redo per batch holding the junk stream
    assert dec.frame_hypothesis_redos() == (depth + 5) // 2
    dec.close()


def test_redo_streak_falls_back_to_full_parse(gpu_engine):
    """batch after batch of input the hypothesis fails on: the decoder redoes
    four in a row, then walks every subframe (mode 0, flac_decode.hip
    kSpecStreak) -- every batch's results equal the full parse's, and only
    four redos are paid"""
    from audiotools import _atgpu
    opts = _atgpu.make_options(**oracle_port.PRESETS["8"])
    pcm = signals.make("tone", 4096 * 6 + 55, 2, 16, seed=13)
    out, res, _, _ = gpu_engine.encode(opts, pcm.astype(np.int16), [(0, len(pcm) // 2)], 2, 16,
                                       44100)
    img = out[res[0].out_offset:res[0].out_offset + res[0].bytes].tobytes()
    rc, si, _ = _atgpu.read_metadata(img)
    tracks, blob = _batch([img])
    _, _, offs, _ = _atgpu.Decoder(0).decode(blob, tracks)
    cut = si.frames_offset + int(offs[1])
    bad = img[:cut] + b"\0\0" + img[cut:]
    tracks, blob = _batch([bad, img])
    ref = _atgpu.Decoder(0)
    ref.set_frame_hypothesis(0)
    want = [_key(r) for r in ref.decode(blob, tracks)[1]]
    ref.close()
    dec = _atgpu.Decoder(0)
    for _ in range(7):
        assert [_key(r) for r in dec.decode(blob, tracks)[1]] == want
    assert dec.frame_hypothesis_redos() == 4
    dec.set_frame_hypothesis(1)  # the caller's setting starts a new streak
    assert [_key(r) for r in dec.decode(blob, tracks)[1]] == want
    assert dec.frame_hypothesis_redos() == 5
    dec.close()
