#!/usr/bin/env python3
"""Isolated FLAC-8 encode of a config-5-shaped batch (64 tracks, 10 s,
48 kHz, 5.1, 24-bit in int32 containers) and of a 16-bit stereo batch with
the same bytes per track, synchronously, one batch at a time: the MD5
kernel time per 64-byte block without other work on the GPU (development
tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from audiotools import _atgpu
    dev = torch.device("cuda", 0)
    eng = _atgpu.Engine(0)
    opts = _atgpu.make_options(**bench.FLAC8)
    for name, ch, bps, fmt, frames in (("s32_24bit_6ch", 6, 24, _atgpu.PCM_S32, 480000),
                                       ("s16_2ch", 2, 16, _atgpu.PCM_S16, 480000 * 9 // 2)):
        n = 64
        g = torch.Generator(device=dev)
        g.manual_seed(3)
        lim = 1 << (bps - 2)
        dt = torch.int32 if fmt == _atgpu.PCM_S32 else torch.int16
        pcm = torch.randint(-lim, lim, (n * frames * ch,), device=dev, generator=g,
                            dtype=torch.int32).to(dt)
        tracks = [(k * frames, frames) for k in range(n)]
        _, cap = eng.bounds(opts, tracks, ch, bps)
        out = torch.empty(cap, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        for rep in range(3):
            eng.encode_device(opts, pcm.data_ptr(), fmt, tracks, ch, bps, 48000, out.data_ptr(), cap)
            kt = eng.kernel_times()
        nbytes = frames * ch * (bps // 8)
        blocks = nbytes // 64
        md5 = kt.get("track_md5", 0.0)
        print("%s: %d tracks x %.2f MB, track_md5 %.2f ms = %.3f us per block; %s"
              % (name, n, nbytes / 1e6, md5, md5 * 1e3 / blocks,
                 {k: round(v, 3) for k, v in kt.items()}), flush=True)
        del pcm, out


if __name__ == "__main__":
    main()
