"""Debug: GPU decode of the fixture files vs the oracle frame loop; prints
the first mismatching sample per file (frame index, channel, values)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "python-audio-tools_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
import decode_cases  # noqa: E402
import oracle_port  # noqa: E402
from audiotools import _atgpu  # noqa: E402

files = sorted(set(c["file"] for c in decode_cases.load_cases()))
dec = _atgpu.Decoder(0)
for fn in files:
    d = open(os.path.join(decode_cases.FIX, fn), "rb").read()
    rc, si, _ = _atgpu.read_metadata(d)
    if rc:
        continue
    body = d[si.frames_offset:]
    body += b"\0" * ((-len(body)) % 4)
    tr = [_atgpu.dec_track(0, len(d) - si.frames_offset, si)]
    pcm, res, _, _ = dec.decode(body, tr)
    want = oracle_port.decode_frames(d)
    r = res[0]
    got = pcm[r.pcm_offset * si.channels:(r.pcm_offset + r.pcm_frames) * si.channels]
    w = want["pcm"]
    n = min(len(got), len(w))
    bad = np.nonzero(got[:n] != w[:n])[0]
    info = "status %d frames %d/%d ch %d bps %d" % (r.status, r.pcm_frames, want["pcm_frames"],
                                                  si.channels, si.bits_per_sample)
    if len(bad):
        i = bad[0]
        fr = i // si.channels
        print(fn, info, "first bad sample", i, "frame-sample", fr, "ch", i % si.channels,
              "got", got[i], "want", w[i], "nbad", len(bad), "block", si.max_block_size, flush=True)
    else:
        print(fn, info, "ok", flush=True)
