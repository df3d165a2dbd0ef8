"""Host-to-host FLAC-8 pipeline (atg_flac_encode_host) on config 2, for a
rocprofv3 kernel + memory-copy trace: pinned PCM / output, 256 MB chunks.
    rocprofv3 --kernel-trace --memory-copy-trace --stats -- python3 tools/host_timeline.py
Prints the wall time per batch (development tool)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from audiotools import _atgpu
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    pinned = (sys.argv[2] if len(sys.argv) > 2 else "pinned") == "pinned"
    chunk_mb = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    inflight = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    dev = torch.device("cuda", 0)
    n_samples = 64 * 4096
    pcm = bench.synth_batch(torch, list(range(1024)), n_samples, dev).cpu().numpy()
    eng = _atgpu.Engine(0)
    opts = _atgpu.make_options(**bench.FLAC8)
    tracks = [(i * n_samples, n_samples) for i in range(1024)]
    nb = eng.bounds(opts, tracks, 2, 16)[1]
    if pinned:
        p = _atgpu.pinned_empty(pcm.shape, np.int16)
        p[:] = pcm
        pcm = p
    out = _atgpu.pinned_empty(nb, np.uint8) if pinned else None
    eng.set_host_chunk_bytes(chunk_mb << 20)
    eng.encode(opts, pcm, tracks, 2, 16, 44100, out=out)
    for _ in range(steps):
        t0 = time.perf_counter()
        eng.encode(opts, pcm, tracks, 2, 16, 44100, out=out)
        dt = time.perf_counter() - t0
        print("batch %.2f ms  %.3f M frames/s (%s, sync)"
              % (dt * 1e3, 65536 / dt / 1e6, "pinned" if pinned else "pageable"), flush=True)
    # batches queued back to back (atg_flac_encode_host_async), `inflight`
    # jobs in flight
    outs = [out] + [_atgpu.pinned_empty(nb, np.uint8) if pinned else None
                    for _ in range(inflight - 1)]
    t0 = time.perf_counter()
    pend = []
    for k in range(steps):
        pend.append(eng.encode_async(opts, pcm, tracks, 2, 16, 44100, out=outs[k % inflight]))
        if len(pend) >= inflight:
            pend.pop(0).wait()
    while pend:
        pend.pop(0).wait()
    dt = (time.perf_counter() - t0) / steps
    print("batch %.2f ms  %.3f M frames/s (%s, queued, chunk %d MB, %d in flight, HW queues %s)"
          % (dt * 1e3, 65536 / dt / 1e6, "pinned" if pinned else "pageable", chunk_mb, inflight,
             os.environ.get("GPU_MAX_HW_QUEUES", "default")), flush=True)


if __name__ == "__main__":
    main()
