"""GPU parity: libatgpu's FLAC decoder (flac_decode.hip) vs the reference
decoder's recorded behaviour and vs the CPU oracle decoder.

* every golden case of tests/golden/flac_decode_vectors.json (the
  reference's own FLAC fixtures plus seeded corruptions, recorded with the
  reference decoder by tests/golden/make_decode_golden.py): same status code,
  same number of PCM bytes before it, same PCM MD5 -- one GPU batch per
  fixture (33 streams);
* GPU encode -> GPU decode round trips across presets, channel counts and
  bit depths (bit-exact PCM, STREAMINFO MD5 verified on the GPU), and
  offsets() equal to the encoder's frame list;
* the FlacDecoder interface: one frame per read(), errors raised at the
  frame where the reference raises them.
"""
import hashlib

import numpy as np
import pytest

import decode_cases
import oracle_port
import signals

pytestmark = pytest.mark.gpu

CASES = decode_cases.load_cases()
FILES = sorted(set(c["file"] for c in CASES))


def _batch(datas):
    from audiotools import _atgpu
    tracks, parts, infos, pos = [], [], [], 0
    for d in datas:
        rc, si, _ = _atgpu.read_metadata(d)
        infos.append((rc, si))
        if rc:
            continue
        body = d[si.frames_offset:]
        pad = (-len(body)) % 4
        tracks.append(_atgpu.dec_track(pos, len(body), si))
        parts.append(body + b"\0" * pad)
        pos += len(body) + pad
    return tracks, b"".join(parts), infos


@pytest.mark.parametrize("fname", FILES)
def test_golden_cases_batch(fname):
    from audiotools import _atgpu
    cases = [c for c in CASES if c["file"] == fname]
    datas = [decode_cases.case_bytes(c) for c in cases]
    tracks, blob, infos = _batch(datas)
    _, res, _, _ = _atgpu.decoder().decode(blob, tracks, fetch_pcm=False)
    k = 0
    for c, (rc, si) in zip(cases, infos):
        if rc:
            assert c["code"] == 100, c["name"]
            continue
        r = res[k]
        k += 1
        bb = (si.bits_per_sample + 7) // 8
        assert r.status == c["code"], (c["name"], r.status, c["code"])
        assert r.pcm_frames * si.channels * bb == c["pcm_bytes"], c["name"]
        assert bytes(r.md5).hex() == c["pcm_md5"], c["name"]


def test_golden_pcm_matches_oracle():
    """PCM samples (not only their MD5) of the uncorrupted fixtures"""
    from audiotools import _atgpu
    datas = [decode_cases.case_bytes(c) for c in CASES
             if not c["xor"] and c["cut"] is None and c["file"] != "1h.flac"]
    tracks, blob, infos = _batch(datas)
    pcm, res, offs, bss = _atgpu.decoder().decode(blob, tracks)
    k = 0
    for d, (rc, si) in zip(datas, infos):
        if rc:
            continue
        r = res[k]
        k += 1
        want = oracle_port.decode_frames(d)
        got = pcm[r.pcm_offset * si.channels:(r.pcm_offset + r.pcm_frames) * si.channels]
        assert np.array_equal(got, np.asarray(want["pcm"], dtype=np.int32))
        got_offs = [(int(o), int(b)) for o, b in
                    zip(offs[r.first_frame:r.first_frame + r.n_frames],
                        bss[r.first_frame:r.first_frame + r.n_frames])]
        assert got_offs == [tuple(x) for x in want["offsets"]]


@pytest.mark.parametrize("preset", ["8", "5", "0", "2"])
@pytest.mark.parametrize("channels,bps", [(2, 16), (1, 16), (2, 24), (6, 16), (1, 8), (2, 8)])
def test_encode_decode_round_trip(gpu_engine, preset, channels, bps):
    from audiotools import _atgpu
    opts = dict(oracle_port.PRESETS[preset])
    B = opts["block_size"]
    kinds = ["tone", "noise", "silence", "chirp", "sine", "wasted"]
    pcms = [signals.make(k, B * (1 + i % 3) + 37 * i, channels, bps, seed=i)
            for i, k in enumerate(kinds)]
    o = _atgpu.make_options(**opts)
    tracks, start = [], 0
    for p in pcms:
        tracks.append((start, len(p) // channels))
        start += len(p) // channels
    allpcm = np.concatenate(pcms).astype(np.int16 if bps <= 16 else np.int32)
    out, res, eoffs, efp = gpu_engine.encode(o, allpcm, tracks, channels, bps, 44100)
    images = [out[r.out_offset:r.out_offset + r.bytes].tobytes() for r in res]
    dtracks, blob, infos = _batch(images)
    pcm, dres, offs, bss = _atgpu.decoder().decode(blob, dtracks)
    for i, (p, r, er) in enumerate(zip(pcms, dres, res)):
        si = infos[i][1]
        assert r.status == 0, (i, r.status)
        got = pcm[r.pcm_offset * channels:(r.pcm_offset + r.pcm_frames) * channels]
        assert np.array_equal(got, p.astype(np.int32))
        assert bytes(r.md5) == bytes(si.md5)
        got_offs = [int(x) for x in offs[r.first_frame:r.first_frame + r.n_frames]]
        want_offs = [int(x) for x in eoffs[er.first_frame:er.first_frame + er.n_frames]]
        assert got_offs == want_offs


def test_flacdecoder_interface(tmp_path):
    from audiotools import decoders
    data = open(decode_cases.FIX + "/tone2.flac", "rb").read()
    fn = tmp_path / "t.flac"
    fn.write_bytes(data)
    want = oracle_port.decode_frames(data)
    with open(fn, "rb") as f:
        dec = decoders.FlacDecoder(f)
    frames = []
    while True:
        fl = dec.read(4096)
        if not len(fl):
            break
        frames.append(fl)
    assert len(frames) == len(want["offsets"])
    got = np.concatenate([f.samples for f in frames]).astype(np.int32)
    assert np.array_equal(got, np.asarray(want["pcm"], dtype=np.int32))
    # offsets() walks from the current position (flac.c:380): nothing left
    assert dec.offsets() == []
    with open(fn, "rb") as f:
        assert decoders.FlacDecoder(f).offsets() == [tuple(x) for x in want["offsets"]]
    dec.close()
    with pytest.raises(ValueError):
        dec.read(1)


def test_flacdecoder_raises_at_bad_frame():
    from audiotools import decoders
    bad = [c for c in CASES if c["code"] == 14 and c["file"] == "tone3.flac"][0]
    data = decode_cases.case_bytes(bad)
    dec = decoders.FlacDecoder(data)
    n = 0
    with pytest.raises(ValueError) as e:
        while True:
            fl = dec.read(4096)
            n += fl.frames
            if not len(fl):
                break
    assert "invalid checksum in frame" in str(e.value)
    bb = (dec.bits_per_sample + 7) // 8
    assert n * dec.channels * bb == bad["pcm_bytes"]


def test_truncated_stream_raises_ioerror():
    from audiotools import decoders
    bad = [c for c in CASES if c["code"] == 15][0]
    dec = decoders.FlacDecoder(decode_cases.case_bytes(bad))
    with pytest.raises(IOError):
        while len(dec.read(4096)):
            pass


def test_async_decode_three_in_flight(gpu_engine):
    """atg_flac_decode_device_async: three batches in flight (batch k's
    restore, emit and MD5 on its slot's stream under batch k+1's scan and
    parse) give the synchronous decode's results and PCM; a fourth enqueue
    before a wait is refused"""
    import torch
    from audiotools import _atgpu
    opts = dict(oracle_port.PRESETS["8"])
    pcms = [signals.make(k, 4096 * 5 + 311 * i, 2, 16, seed=40 + i)
            for i, k in enumerate(["tone", "noise", "chirp", "silence", "sine"])]
    o = _atgpu.make_options(**opts)
    tracks, start = [], 0
    for p in pcms:
        tracks.append((start, len(p) // 2))
        start += len(p) // 2
    allpcm = np.concatenate(pcms).astype(np.int16)
    out, res, _, _ = gpu_engine.encode(o, allpcm, tracks, 2, 16, 44100)
    images = [out[r.out_offset:r.out_offset + r.bytes].tobytes() for r in res]
    dtracks, blob, _ = _batch(images)
    d_blob = torch.frombuffer(bytearray(blob + b"\0" * 64), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    dec = _atgpu.Decoder(0)
    want, _, wn = dec.decode_device(d_blob.data_ptr(), len(blob), dtracks)
    want = [(r.status, r.pcm_frames, bytes(r.md5)) for r in want]
    t1 = dec.decode_device_async(d_blob.data_ptr(), len(blob), dtracks)
    t2 = dec.decode_device_async(d_blob.data_ptr(), len(blob), dtracks)
    t3 = dec.decode_device_async(d_blob.data_ptr(), len(blob), dtracks)
    with pytest.raises(_atgpu.ATGError):
        dec.decode_device_async(d_blob.data_ptr(), len(blob), dtracks)
    for t in (t1, t2, t3):
        got, d_pcm, n = dec.decode_wait(t)
        assert [(r.status, r.pcm_frames, bytes(r.md5)) for r in got] == want
        assert n == wn == len(allpcm)
        host = np.empty(n, dtype=np.int32)
        gpu_engine.copy_to_host(host, d_pcm)
        assert np.array_equal(host, allpcm.astype(np.int32))
    with pytest.raises(_atgpu.ATGError):
        dec.decode_wait(t1)
    dec.close()


def test_async_decode_fetch_frame_table(gpu_engine):
    """atg_flac_decode_fetch after an async batch: the frame table lives in
    the batch's slot, so the last waited batch's offsets and block sizes are
    readable while two newer batches are in flight, equal to the host
    decode's; once a newer batch takes that slot, fetch is refused"""
    import ctypes
    import torch
    from audiotools import _atgpu
    opts = dict(oracle_port.PRESETS["5"])
    pcms = [signals.make(k, 4096 * 3 + 129 * i, 2, 16, seed=70 + i)
            for i, k in enumerate(["tone", "noise", "chirp"])]
    o = _atgpu.make_options(**opts)
    tracks, start = [], 0
    for p in pcms:
        tracks.append((start, len(p) // 2))
        start += len(p) // 2
    allpcm = np.concatenate(pcms).astype(np.int16)
    out, res, _, _ = gpu_engine.encode(o, allpcm, tracks, 2, 16, 44100)
    images = [out[r.out_offset:r.out_offset + r.bytes].tobytes() for r in res]
    dtracks, blob, _ = _batch(images)
    dec = _atgpu.Decoder(0)
    _, want, woffs, wbs = dec.decode(blob, dtracks)
    d_blob = torch.frombuffer(bytearray(blob + b"\0" * 64), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    t1 = dec.decode_device_async(d_blob.data_ptr(), len(blob), dtracks)
    t2 = dec.decode_device_async(d_blob.data_ptr(), len(blob), dtracks)
    t3 = dec.decode_device_async(d_blob.data_ptr(), len(blob), dtracks)
    dec.decode_wait(t1)
    nf = len(woffs)
    offs = np.empty(nf, dtype=np.uint64)
    bss = np.empty(nf, dtype=np.uint32)
    lib = dec.lib
    st = lib.atg_flac_decode_fetch(dec.handle, None, 0, offs.ctypes.data_as(ctypes.c_void_p),
                                   bss.ctypes.data_as(ctypes.c_void_p), nf)
    assert st == 0, lib.atg_decoder_last_error()
    assert np.array_equal(offs, woffs) and np.array_equal(bss, wbs)
    t4 = dec.decode_device_async(d_blob.data_ptr(), len(blob), dtracks)  # t1's slot
    st = lib.atg_flac_decode_fetch(dec.handle, None, 0, offs.ctypes.data_as(ctypes.c_void_p),
                                   bss.ctypes.data_as(ctypes.c_void_p), nf)
    assert st != 0
    for t in (t2, t3, t4):
        got, _, _ = dec.decode_wait(t)
        assert [(r.status, r.pcm_frames) for r in got] == [(r.status, r.pcm_frames) for r in want]
    dec.close()



@pytest.mark.parametrize("depth", [4, 8, 16])
def test_rolled_decode_many_in_flight(gpu_engine, depth):
    """atg_decoder_set_inflight(depth >= 4): every batch's MD5 hashes run in
    depth - 2 slices on the decoder's roll stream (md5.hip
    k_bytes_md5_roll).  More batches than slots, alternating between a
    batch of clean round-trip tracks and a batch of the reference's golden
    corrupt cases: every batch's statuses, PCM counts and MD5s equal the
    synchronous depth-3 decode's (the golden cases' also the reference
    decoder's recorded values), the clean PCM equals the source, waits both
    oldest-first and out of order, and a (depth + 1)-th enqueue is refused"""
    import torch
    from audiotools import _atgpu
    opts = _atgpu.make_options(**oracle_port.PRESETS["8"])
    pcms = [signals.make(k, 4096 * 4 + 77 * i, 2, 16, seed=90 + i)
            for i, k in enumerate(["tone", "noise", "chirp", "sine", "silence"])]
    tracks, start = [], 0
    for p in pcms:
        tracks.append((start, len(p) // 2))
        start += len(p) // 2
    allpcm = np.concatenate(pcms).astype(np.int16)
    out, res, _, _ = gpu_engine.encode(opts, allpcm, tracks, 2, 16, 44100)
    clean = _batch([out[r.out_offset:r.out_offset + r.bytes].tobytes() for r in res])
    fname = FILES[len(FILES) // 2]
    cases = [c for c in CASES if c["file"] == fname]
    gold = _batch([decode_cases.case_bytes(c) for c in cases])
    blobs = []
    for dtracks, blob, _ in (clean, gold):
        d = torch.frombuffer(bytearray(blob + b"\0" * 64), dtype=torch.uint8).cuda()
        blobs.append((d, len(blob), dtracks))
    torch.cuda.synchronize()
    dec = _atgpu.Decoder(0)
    want = []
    for d, n, dt in blobs:
        w, _, _ = dec.decode_device(d.data_ptr(), n, dt)
        want.append([(r.status, r.pcm_frames, bytes(r.md5)) for r in w])
    # the golden batch: the reference decoder's recorded values
    k = 0
    for c, (rc, si) in zip(cases, gold[2]):
        if rc:
            continue
        st, nfr, md5 = want[1][k]
        k += 1
        assert st == c["code"] and md5.hex() == c["pcm_md5"], c["name"]
    dec.set_inflight(depth)

    def check(i, got, d_pcm, n):
        assert [(r.status, r.pcm_frames, bytes(r.md5)) for r in got] == want[i % 2], i
        if i % 2 == 0:
            host = np.empty(n, dtype=np.int32)
            gpu_engine.copy_to_host(host, d_pcm)
            assert np.array_equal(host, allpcm.astype(np.int32)), i

    pending = []
    for i in range(depth + 4):
        if len(pending) == depth:
            j, t = pending.pop(0)
            check(j, *dec.decode_wait(t))
        d, n, dt = blobs[i % 2]
        pending.append((i, dec.decode_device_async(d.data_ptr(), n, dt)))
    with pytest.raises(_atgpu.ATGError):
        d, n, dt = blobs[0]
        dec.decode_device_async(d.data_ptr(), n, dt)
    for j, t in reversed(pending):
        check(j, *dec.decode_wait(t))
    dec.set_inflight(3)
    d, n, dt = blobs[0]
    check(0, *dec.decode_wait(dec.decode_device_async(d.data_ptr(), n, dt)))
    for bad in (2, 17):  # the rotation is 3..16 batches
        with pytest.raises(_atgpu.ATGError):
            dec.set_inflight(bad)
    dec.close()
