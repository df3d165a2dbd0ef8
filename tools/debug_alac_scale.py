"""Debug aid: GPU ALAC encode -> GPU ALAC decode at config-5 scale
(64 x 10 s of 192 kHz / 24-bit / 6 ch), reporting which tracks do not
round-trip and whether the CPU port decodes their images to the source."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-audio-tools_amd"), os.path.join(ROOT, "tests")]


def main():
    import torch
    from audiotools import _atgpu
    import oracle_port
    n_tracks = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    secs = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ch, rin, bps = 6, 192000, 24
    n_in = secs * rin
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    if len(sys.argv) > 3 and sys.argv[3] == "noise":
        src = torch.randint(-(1 << 22), 1 << 22, (n_tracks * n_in * ch,), dtype=torch.int32,
                            device=dev, generator=g)
    else:  # bench.py chain_leg's signal
        t = torch.arange(n_in, device=dev, dtype=torch.float64)
        src = torch.empty((n_tracks, n_in, ch), dtype=torch.int32, device=dev)
        for k in range(n_tracks):
            f = (110.0 + 37.0 * k + 55.0 * torch.arange(ch, device=dev, dtype=torch.float64))
            tone = torch.sin(2 * np.pi * t[:, None] * f[None, :] / rin) * (3e6 + 1e5 * (k % 40))
            noise = torch.randint(-4096, 4096, (n_in, ch), device=dev, generator=g,
                                  dtype=torch.int32)
            src[k] = tone.to(torch.int32) + noise
        del t
        src = src.reshape(-1)
    torch.cuda.synchronize()
    aenc = _atgpu.AlacEncoder(0)
    aopts = aenc.options()
    atracks = [(k * n_in, n_in) for k in range(n_tracks)]
    n_fs, acap = aenc.bounds(aopts, atracks, ch, bps)
    alac = torch.zeros(acap, dtype=torch.uint8, device=dev)
    fsb = np.zeros(max(1, n_fs), dtype=np.uint32)
    ares = aenc.encode_device(aopts, src.data_ptr(), _atgpu.PCM_S32, atracks, ch, bps,
                              alac.data_ptr(), acap, fsb)
    print("encoded", n_fs, "framesets, cap", acap, "last out end",
          max(r.out_offset + r.bytes for r in ares), flush=True)
    info = _atgpu.AlacInfo()
    info.max_samples_per_frame, info.bits_per_sample = 4096, bps
    info.history_multiplier, info.initial_history, info.maximum_k = 40, 10, 14
    info.channels, info.sample_rate, info.total_frames = ch, rin, n_in
    dtracks = [_atgpu.alac_dec_track(r.out_offset, r.bytes, info, start=8, remaining=n_in,
                                     frameset_bytes=fsb[r.first_frameset:r.first_frameset +
                                                        r.n_framesets]) for r in ares]
    adec = _atgpu.AlacDecoder(0)
    nbytes = max(int(r.out_offset + r.bytes) for r in ares)
    dres, d_pcm, nsamp = adec.decode_device(alac.data_ptr(), nbytes, dtracks)
    eng = _atgpu.Engine(0)
    got = torch.empty_like(src)
    eng.copy_device(got.data_ptr(), d_pcm, src.numel() * 4)
    per = n_in * ch
    bad = [t for t in range(n_tracks)
           if not torch.equal(got[t * per:(t + 1) * per], src[t * per:(t + 1) * per])]
    print("status", sorted({int(r.status) for r in dres}), "bad tracks", bad, flush=True)
    if bad:
        t = bad[0]
        gh = got[t * per:(t + 1) * per].cpu().numpy()
        sh = src[t * per:(t + 1) * per].cpu().numpy()
        diff = np.flatnonzero(gh != sh)
        print("track", t, "first diff sample", diff[0], "frame", diff[0] // ch, "count", len(diff),
              "offset of track pcm bytes", t * per * 4, flush=True)
        r = ares[t]
        img = alac[r.out_offset:r.out_offset + r.bytes].cpu().numpy().tobytes()
        pinfo = oracle_port.AlacInfo()
        for f in ("max_samples_per_frame", "bits_per_sample", "history_multiplier",
                  "initial_history", "maximum_k", "channels", "sample_rate", "total_frames"):
            setattr(pinfo, f, getattr(info, f))
        d = oracle_port.alac_decode(img, info=pinfo, start=8, remaining=n_in)
        print("port decode of the GPU image: code", d["code"], "equal to source",
              np.array_equal(d["pcm"], sh), "equal to GPU decode", np.array_equal(d["pcm"], gh),
              flush=True)
        want, wfs = oracle_port.alac_encode(sh, ch, bps)
        print("port encode of the source equals the GPU image:", want == img,
              "sizes equal:", list(wfs) == [int(x) for x in
                                             fsb[r.first_frameset:r.first_frameset +
                                                 r.n_framesets]], flush=True)


if __name__ == "__main__":
    main()
