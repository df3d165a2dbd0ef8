"""Where the drop-in calculate_replay_gain's time goes on the config-4 album
(1024 titles x 10 s, 44.1 kHz 16-bit stereo, host int32 PCM): the title
reads (read(4096) FrameLists), then album_scan's phases."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from audiotools import replaygain  # noqa: E402

n_tracks, n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 441000
rng = np.random.default_rng(5)
x = rng.integers(-3000, 3000, n_tracks * n * 2, dtype=np.int32)
mem = [bench._MemTrack(x[k * n * 2:(k + 1) * n * 2], 2, 16, 44100) for k in range(n_tracks)]
replaygain.album_scan([replaygain._read_title(mem[0].to_pcm(), 44100)], 44100)  # warm
t0 = time.perf_counter()
titles = [replaygain._read_title(m.to_pcm(), 44100) for m in mem]
t1 = time.perf_counter()
gains, hist, peak = replaygain.album_scan(titles, 44100)
t2 = time.perf_counter()
print(json.dumps({"tracks": n_tracks, "read_s": round(t1 - t0, 3), "album_scan_s": round(t2 - t1, 3),
                  "phases": getattr(replaygain, "_last_phases", None)}))
