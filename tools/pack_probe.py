"""Frame-pack probe: a config-5-shaped FLAC-8 batch (64 tracks x 10 s of
48 kHz 6-channel 24-bit PCM: per channel two sines + noise, as the chain's
resampled output), encoded synchronously on the GPU, the engine's own
kernel times averaged over the batches after the first.  The library comes
from ATGPU_LIB (an A/B build) or the product; the images' digest lets two
builds be compared byte for byte.  One JSON line.

    python tools/pack_probe.py [--batches 6] [--channels 6] [--bits 24]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from audiotools import _atgpu  # noqa: E402


def synth(tracks, ns, ch, bits, rate, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(0x9ACC)
    n = torch.arange(ns, dtype=torch.float64, device=dev)
    full = float((1 << (bits - 1)) - 1)
    out = torch.empty((tracks, ns, ch), dtype=torch.int32, device=dev)
    for t in range(tracks):
        r = np.random.RandomState(0x5EED + t)
        for c in range(ch):
            f1, f2 = r.uniform(60, 3000), r.uniform(3000, 16000)
            a1, a2 = r.uniform(0.05, 0.5), r.uniform(0.0, 0.2)
            x = (a1 * torch.sin(2 * np.pi * f1 * n / rate) +
                 a2 * torch.sin(2 * np.pi * f2 * n / rate)) * full
            x = x + torch.randn(ns, generator=g, device=dev, dtype=torch.float64) * 256.0
            out[t, :, c] = torch.round(x).clamp_(-full - 1, full).to(torch.int32)
    return out.reshape(-1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--tracks", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--channels", type=int, default=6)
    ap.add_argument("--bits", type=int, default=24)
    ap.add_argument("--rate", type=int, default=48000)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("ATGPU_LIB", "product")))
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = _atgpu.Engine(0)
    opts = _atgpu.make_options(**bench.FLAC8)
    ns = int(a.seconds * a.rate)
    pcm = synth(a.tracks, ns, a.channels, a.bits, a.rate, dev)
    tracks = [(i * ns, ns) for i in range(a.tracks)]
    _, cap = eng.bounds(opts, tracks, a.channels, a.bits)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    kt, n, digest = {}, 0, None
    for k in range(a.batches):
        res = eng.encode_device(opts, pcm.data_ptr(), _atgpu.PCM_S32, _atgpu.TrackTable(tracks),
                                a.channels, a.bits, a.rate, out.data_ptr(), cap)
        torch.cuda.synchronize()
        if k:
            for key, v in eng.kernel_times().items():
                kt[key] = kt.get(key, 0.0) + v
            n += 1
        else:
            nb = max(r.out_offset + r.bytes for r in res)
            digest = hashlib.sha256(out[:nb].cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"tag": a.tag, "kernel_ms": {k: round(v / max(1, n), 4) for k, v in kt.items()},
                      "bytes": int(nb), "sha256_16": digest, "channels": a.channels,
                      "bits": a.bits, "tracks": a.tracks}), flush=True)
    eng.close()
    _atgpu.close_all()


if __name__ == "__main__":
    main()
