"""GPU: BASELINE config 5 end to end -- the track2track chain
ALAC (192 kHz / 24-bit / 5.1) decode -> 48 kHz sinc resample -> FLAC-8
(six independent subframes per frame, reference src/encoders/flac.c:653-666)
on short tracks, every stage on the GPU and every stage compared with its
CPU oracle:

* GPU ALAC encode (the chain's input) == oracle/alac_port.c mdat, byte for
  byte (the port is pinned to the reference encoder's vectors);
* GPU ALAC decode == the source PCM (lossless) and == the port's decode;
* GPU resample == oracle/resample_port.c, bit for bit (parity unpinned to
  reference output: the BEST table is absent from the reference tree);
* GPU FLAC-8 image == oracle/flac_port.c's image of the port-resampled PCM.

Once through the host-memory entry points (the Python interface's path) and
once device-resident with the data left in HBM between stages and the FLAC
batches pipelined (bench.py's chain leg)."""
import numpy as np
import pytest

import oracle_port as op

pytestmark = pytest.mark.gpu

CH, BPS, RIN, ROUT = 6, 24, 192000, 48000
FLAC8 = op.PRESETS["8"]


def _source(lengths, seed):
    """tone + noise per channel, |x| < 2^23 (a 24-bit source)"""
    rng = np.random.default_rng(seed)
    out = []
    for k, n in enumerate(lengths):
        t = np.arange(n)[:, None]
        f = 110.0 + 37.0 * k + 55.0 * np.arange(CH)[None, :]
        tone = np.sin(2 * np.pi * t * f / RIN) * (3e6 + 1e5 * k)
        x = tone.astype(np.int64) + rng.integers(-4096, 4096, (n, CH))
        if k == 1:
            x[:, 3] = 0             # a silent LFE: CONSTANT subframes
        if k == 2:
            x = x & ~0xFF           # wasted bits in every channel
        out.append(x.astype(np.int32).reshape(-1))
    return out


LENGTHS = [RIN // 3 + 17, RIN // 4, 4096 * 5 + 1, RIN // 5 + 4095, 9000]


def _oracle_stages(p):
    """the CPU oracles' chain for one track -> (mdat, fs, resampled, flac)"""
    mdat, fs = op.alac_encode(p, CH, BPS)
    rs = op.resample(p, CH, BPS, ROUT / RIN)
    img, _ = op.encode(rs, CH, BPS, ROUT, **FLAC8)
    return mdat, fs, rs, img


def test_chain_host_path_vs_oracles():
    from audiotools import _atgpu, decoders, m4a
    src = _source(LENGTHS, 51)
    want = [_oracle_stages(p) for p in src]
    # 1. ALAC encode
    enc = _atgpu.alac_encoder()
    tracks, pos = [], 0
    for p in src:
        tracks.append((pos, len(p) // CH))
        pos += len(p) // CH
    out, res, fsb = enc.encode(enc.options(), np.concatenate(src), tracks, CH, BPS)
    images = []
    for k, r in enumerate(res):
        assert r.status == 0
        mdat = out[r.out_offset:r.out_offset + r.bytes].tobytes()
        fs = [int(x) for x in fsb[r.first_frameset:r.first_frameset + r.n_framesets]]
        assert mdat == want[k][0] and fs == want[k][1], "ALAC encode track %d" % k
        images.append(m4a.m4a_file(CH, BPS, RIN, 4096, len(src[k]) // CH, mdat, fs,
                                   create_date=3))
    # 2. ALAC decode
    dec = decoders.decode_alac_batch(images)
    for k, (st, info, pcm) in enumerate(dec):
        assert st == 0 and np.array_equal(pcm, src[k]), "ALAC decode track %d" % k
        got = op.alac_decode(images[k])
        assert got["code"] == 0 and np.array_equal(got["pcm"], pcm)
    # 3. resample 192k -> 48k
    rtracks, pos = [], 0
    for p in src:
        rtracks.append((pos, len(p) // CH, RIN, ROUT))
        pos += len(p) // CH
    rs, offs, cnt = _atgpu.resample_host(np.concatenate([d[2] for d in dec]), rtracks, CH, BPS)
    parts = []
    for k in range(len(src)):
        got = rs[int(offs[k]) * CH:(int(offs[k]) + int(cnt[k])) * CH]
        assert np.array_equal(got, want[k][2]), "resample track %d" % k
        parts.append(got)
    # 4. FLAC-8, 6 independent 24-bit subframes per frame
    eng = _atgpu.engine()
    ftracks, pos = [], 0
    for p in parts:
        ftracks.append((pos, len(p) // CH))
        pos += len(p) // CH
    fout, fres, _, _ = eng.encode(_atgpu.make_options(**FLAC8), np.concatenate(parts),
                                  ftracks, CH, BPS, ROUT)
    for k, r in enumerate(fres):
        img = fout[r.out_offset:r.out_offset + r.bytes].tobytes()
        assert img == want[k][3], "FLAC-8 track %d: %d vs %d B" % (k, len(img), len(want[k][3]))


def test_chain_device_resident_pipelined(gpu_engine):
    """bench.py's chain leg on a small batch: ALAC encode_device ->
    decode_device -> resample_device -> encode_device_async, three rounds
    with two FLAC batches in flight"""
    import torch
    from audiotools import _atgpu
    src = _source(LENGTHS, 77)
    want = [_oracle_stages(p) for p in src]
    n_in = [len(p) // CH for p in src]
    d_src = torch.from_numpy(np.concatenate(src)).to("cuda")
    torch.cuda.synchronize()
    aenc = _atgpu.AlacEncoder(0)
    aopts = aenc.options()
    atracks, pos = [], 0
    for n in n_in:
        atracks.append((pos, n))
        pos += n
    n_fs, acap = aenc.bounds(aopts, atracks, CH, BPS)
    alac = torch.zeros(acap, dtype=torch.uint8, device="cuda")
    fsb = np.zeros(max(1, n_fs), dtype=np.uint32)
    torch.cuda.synchronize()
    ares = aenc.encode_device(aopts, d_src.data_ptr(), _atgpu.PCM_S32, atracks, CH, BPS,
                              alac.data_ptr(), acap, fsb)
    aenc.close()
    alac_h = alac.cpu().numpy()
    info = _atgpu.AlacInfo()
    info.max_samples_per_frame, info.bits_per_sample = 4096, BPS
    info.history_multiplier, info.initial_history, info.maximum_k = 40, 10, 14
    info.channels, info.sample_rate = CH, RIN
    dtracks = []
    for k, r in enumerate(ares):
        assert r.status == 0
        mdat = alac_h[r.out_offset:r.out_offset + r.bytes].tobytes()
        assert mdat == want[k][0], "ALAC encode_device track %d" % k
        info.total_frames = n_in[k]
        dtracks.append(_atgpu.alac_dec_track(
            r.out_offset, r.bytes, info, start=8, remaining=n_in[k],
            frameset_bytes=fsb[r.first_frameset:r.first_frameset + r.n_framesets]))
    nbytes = max(int(r.out_offset + r.bytes) for r in ares)
    adec = _atgpu.AlacDecoder(0)
    rtracks, pos = [], 0
    for n in n_in:
        rtracks.append((pos, n, RIN, ROUT))
        pos += n
    n_out = [_atgpu.resample_output_frames(n, CH, RIN, ROUT) for n in n_in]
    ftracks, pos = [], 0
    for n in n_out:
        ftracks.append((pos, n))
        pos += n
    ys = [torch.empty(sum(n_out) * CH, dtype=torch.int32, device="cuda") for _ in range(2)]
    eng = gpu_engine
    fopts = _atgpu.make_options(**FLAC8)
    _, fcap = eng.bounds(fopts, ftracks, CH, BPS)
    flacs = [torch.empty(fcap, dtype=torch.uint8, device="cuda") for _ in range(2)]
    stream = torch.cuda.current_stream().cuda_stream
    pending = []
    done = []
    for step in range(3):
        dres, d_pcm, nsamp = adec.decode_device(alac.data_ptr(), nbytes, dtracks)
        assert nsamp == d_src.numel()
        assert all(r.status == 0 and r.pcm_frames == n for r, n in zip(dres, n_in))
        y = ys[step % 2]
        offs, cnts = _atgpu.resample_device(d_pcm, y.data_ptr(), y.numel(), rtracks, CH, BPS,
                                            stream)
        assert [int(c) for c in cnts] == n_out
        assert [int(o) for o in offs] == [f[0] for f in ftracks]
        torch.cuda.synchronize()
        t = eng.encode_device_async(fopts, y.data_ptr(), _atgpu.PCM_S32, ftracks, CH, BPS, ROUT,
                                    flacs[step % 2].data_ptr(), fcap)
        if pending:
            done.append((pending[0][0], eng.wait(pending.pop(0)[1])))
        pending.append((step, t))
        # the decoded PCM is the source
        got = torch.empty_like(d_src)
        eng.copy_device(got.data_ptr(), d_pcm, d_src.numel() * 4)
        assert torch.equal(got, d_src)
    done.append((pending[0][0], eng.wait(pending.pop(0)[1])))
    adec.close()
    assert [s for s, _ in done] == [0, 1, 2]
    for step, fres in done[-2:]:
        yh = ys[step % 2].cpu().numpy()
        fh = flacs[step % 2].cpu().numpy()
        for k in range(len(src)):
            got = yh[ftracks[k][0] * CH:(ftracks[k][0] + n_out[k]) * CH]
            assert np.array_equal(got, want[k][2]), "resample_device track %d" % k
            r = fres[k]
            img = fh[r.out_offset:r.out_offset + r.bytes].tobytes()
            assert img == want[k][3], "FLAC-8 step %d track %d" % (step, k)
