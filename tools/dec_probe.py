"""Decoder probe: config-2 batch (bench.synth_batch, FLAC-8 encode on the
GPU), then the GPU decoder two ways -- synchronous batches (kernel times
without the pipeline's concurrency) and the pipelined step the bench leg
times -- with every track's PCM compared against the source.  The library
comes from ATGPU_LIB (an exp/ build) or the product.  One JSON line.

    python tools/dec_probe.py [--steps 20] [--tag name]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from audiotools import _atgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--tracks", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("ATGPU_LIB", "product")))
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = _atgpu.Engine(0)
    opts = _atgpu.make_options(**bench.FLAC8)
    ns = a.frames * bench.BLOCK
    pcm = bench.synth_batch(torch, list(range(a.tracks)), ns, dev)
    tracks = [(i * ns, ns) for i in range(a.tracks)]
    _, cap = eng.bounds(opts, tracks, 2, 16)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    res = eng.encode_device(opts, pcm.data_ptr(), _atgpu.PCM_S16, _atgpu.TrackTable(tracks), 2, 16,
                            44100, out.data_ptr(), cap)
    torch.cuda.synchronize()
    dtr = []
    for r in res:
        si = _atgpu.StreamInfo()
        si.total_samples = ns
        si.sample_rate, si.channels, si.bits_per_sample = 44100, 2, 16
        si.max_block_size = bench.BLOCK
        si.md5[:] = bytes(r.md5)
        dtr.append(_atgpu.dec_track(r.out_offset + bench.HEADER_BYTES,
                                    r.bytes - bench.HEADER_BYTES, si))
    nbytes = max(r.out_offset + r.bytes for r in res)
    comp = sum(int(r.bytes) - bench.HEADER_BYTES for r in res)
    dec = _atgpu.Decoder(0)
    # synchronous: one batch at a time
    kt, n = {}, 0
    for k in range(5):
        dres, d_pcm, nsamp = dec.decode_device(out.data_ptr(), nbytes, dtr)
        if k:
            for key, v in dec.kernel_times().items():
                kt[key] = kt.get(key, 0.0) + v
            n += 1
    kt = {k: round(v / n, 4) for k, v in kt.items()}
    ok = all(r.status == 0 and r.pcm_frames == ns for r in dres)
    got = np.empty(int(nsamp), dtype=np.int32)
    eng.copy_to_host(got, d_pcm)
    src = pcm.cpu().numpy().astype(np.int32)
    same = bool(np.array_equal(got, src))
    # pipelined
    if a.steps == 0:
        print(json.dumps({"tag": a.tag, "sync_kernel_ms": kt, "ok": ok, "pcm_same": same}))
        return
    pend = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if len(pend) == a.inflight:
            dec.decode_wait(pend.pop(0))
        pend.append(dec.decode_device_async(out.data_ptr(), nbytes, dtr))
    bad = {}
    while pend:
        last = dec.decode_wait(pend.pop(0))
        for i, r in enumerate(last[0]):
            if r.status != 0 or r.pcm_frames != ns:
                bad.setdefault(int(r.status), []).append(i)
    dt = time.perf_counter() - t0
    ok2 = not bad
    same2 = False
    if last[2] == pcm.numel():
        got2 = np.empty(int(last[2]), dtype=np.int32)
        eng.copy_to_host(got2, last[1])
        same2 = bool(np.array_equal(got2, src))
    print(json.dumps({"tag": a.tag, "sync_kernel_ms": kt, "ok": ok, "pcm_same": same,
                      "pipelined_ms_per_step": round(dt / a.steps * 1e3, 3), "pipelined_ok": ok2, "pipelined_bad": {k: v[:8] for k, v in bad.items()},
                      "pipelined_last_pcm_same": same2,
                      "compressed_bytes": comp, "tracks": a.tracks}), flush=True)


if __name__ == "__main__":
    main()
