"""Resampler kernel timing at BASELINE config-3 scale (1024 stereo 24-bit
tracks x 262144 frames, 44.1k -> 48k) or config-5's resample (192k 5.1 ->
48k), with a spot check of a few tracks against oracle/resample_port.c.
A development tool (bench.py's resample leg is the judged measurement).

usage: python tools/bench_resample.py [--config 3|5] [--tracks N] [--steps K]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-audio-tools_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--tracks", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--check", type=int, default=8)
    a = ap.parse_args()
    import torch
    from audiotools import _atgpu
    import oracle_port
    if a.config == 3:
        ch, rin, rout = 2, 44100, 48000
    else:
        ch, rin, rout = 6, 192000, 48000
    dev = torch.device("cuda", 0)
    n = a.frames
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    x = torch.randint(-(1 << 23), 1 << 23, (a.tracks * n * ch,), dtype=torch.int32, device=dev,
                      generator=g)
    tracks = [(t * n, n, rin, rout) for t in range(a.tracks)]
    n_out = _atgpu.resample_output_frames(n, ch, rin, rout)
    total = n_out * a.tracks
    y = torch.empty(total * ch, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(2):
        _atgpu.resample_device(x.data_ptr(), y.data_ptr(), total * ch, tracks, ch, 24, stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ks = []
    for _ in range(a.steps):
        _atgpu.resample_device(x.data_ptr(), y.data_ptr(), total * ch, tracks, ch, 24, stream)
        ks.append(_atgpu.resample_kernel_times())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    filt = sorted(k["rs_filter"] for k in ks)
    print("config %d: %d tracks x %d frames, %d ch: step %.3f ms, rs_filter median %.3f ms "
          "(min %.3f), %.3g output frames/s" % (a.config, a.tracks, n, ch, dt * 1e3,
                                               filt[len(filt) // 2], filt[0], total / dt),
          flush=True)
    xh = x[:a.check * n * ch].cpu().numpy()
    yh = y[:a.check * n_out * ch].cpu().numpy()
    ok = 0
    for t in range(a.check):
        want = oracle_port.resample(xh[t * n * ch:(t + 1) * n * ch], ch, 24, rout / rin)
        ok += int(np.array_equal(want, yh[t * n_out * ch:(t + 1) * n_out * ch]))
    print("checked %d/%d tracks bit-exact vs oracle" % (ok, a.check), flush=True)
    return 0 if ok == a.check else 1


if __name__ == "__main__":
    sys.exit(main())
