#!/usr/bin/env python3
"""K2 dynamic event counts for the instruction ledger (DESIGN 4a'').

Run with ATGPU_LIB pointing at a build with -DATG_K2F_COUNT=1
(tools/build_exp.sh k2l_cnt flac_search16.hip -DATG_K2F_COUNT=1): encodes
one config-2 batch (bench.py's generator, 1024 tracks x 64 frames) and
prints the counters k_frame_search_ms recorded, one JSON object."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "python-audio-tools_amd"))

NAMES = (["frames", "active_candidates", "fixed_jobs", "lpc_jobs"] +
         ["jobs_order_%d" % o for o in range(13)] +
         ["fold_jobs", "split_jobs", "wide_jobs", "pruned_jobs", "fast32_searches",
          "wide_searches", "side_lr_jobs", "side_packed_jobs", "slow_units"])


def main():
    import torch
    import bench
    from audiotools import _atgpu
    dev = torch.device("cuda", 0)
    eng = _atgpu.Engine(0)
    lib = _atgpu.load_library()
    lib.atg_k2_counters.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_int]
    lib.atg_k2_counters.restype = ctypes.c_int
    opts = _atgpu.make_options(**bench.FLAC8)
    n_tracks, frames = 1024, 64
    n_samples = frames * bench.BLOCK
    pcm = bench.synth_batch(torch, list(range(n_tracks)), n_samples, dev)
    tracks = [(i * n_samples, n_samples) for i in range(n_tracks)]
    _, cap = eng.bounds(opts, tracks, 2, 16)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    table = _atgpu.TrackTable(tracks)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 64)()
    lib.atg_k2_counters(buf, 64, 1)
    eng.wait(eng.encode_device_async(opts, pcm.data_ptr(), _atgpu.PCM_S16, table, 2, 16, 44100,
                                     out.data_ptr(), cap))
    n = lib.atg_k2_counters(buf, 64, 1)
    if n != len(NAMES):
        raise SystemExit("counter count %d, expected %d" % (n, len(NAMES)))
    print(json.dumps({k: int(buf[i]) for i, k in enumerate(NAMES)}))
    eng.close()


if __name__ == "__main__":
    main()
