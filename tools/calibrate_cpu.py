#!/usr/bin/env python3
"""Cross-calibrate the CPU port (oracle/flac_port.c) against the reference
encoder itself (oracle/_ref/flacenc, built from /root/reference/src) on the
same cores and the same synthetic config-2 tracks (the two
must agree within +-20 %).  Runs in the build container (where the
reference build exists); writes profiles/<round>_cpu_calibration.json.

  python3 tools/calibrate_cpu.py [round] [tracks] [frames]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r02"
    tracks = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    import torch
    n = frames * bench.BLOCK
    pcm = bench.synth_batch(torch, list(range(tracks)), n, torch.device("cpu")).numpy()
    cores = os.cpu_count() or 1
    out = {"cpu_model": bench.cpu_model(), "host_cpus": cores, "tracks": tracks,
           "frames_per_track": frames, "runs": []}
    for threads in (1, cores):
        t0 = time.perf_counter()
        ref = bench.ref_encode_sample(pcm, tracks, n, threads)
        if ref is None:
            sys.exit("oracle/_ref/flacenc missing: make -C oracle ref")
        ref_imgs, ref_dt = ref
        port_imgs, port_dt = bench.port_encode_all(pcm, tracks, n, threads)
        same = all(a == b for a, b in zip(ref_imgs, port_imgs))
        fr = tracks * frames
        out["runs"].append({"threads": threads,
                            "reference_frames_per_s": round(fr / ref_dt, 2),
                            "port_frames_per_s": round(fr / port_dt, 2),
                            "port_over_reference": round(ref_dt / port_dt, 3),
                            "identical_bytes": same,
                            "wall_s": round(time.perf_counter() - t0, 2)})
    r1 = out["runs"][0]
    out["summary"] = {"port_over_reference_1_thread": r1["port_over_reference"],
                      "port_over_reference_all_cores": out["runs"][1]["port_over_reference"],
                      "within_20pct": all(0.8 <= r["port_over_reference"] <= 1.2
                                          for r in out["runs"]),
                      "where": "build container (%s, %d cores); the reference build is "
                               "compiled from /root/reference/src" % (out["cpu_model"], cores)}
    fn = os.path.join(ROOT, "profiles", "%s_cpu_calibration.json" % rnd)
    json.dump(out, open(fn, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
