"""Exit-time teardown with work still in flight.

A child process opens an engine and a decoder, runs host-memory jobs from
pinned and pageable buffers, pipelines device batches at depth 12 (rolled
MD5) and decode batches at depth 8, leaves two encode batches, two decode
batches and (on the process-wide default engine) a host job unwaited, closes
nothing and exits.  glibc's heap checks
are on (MALLOC_CHECK_=3, MALLOC_PERTURB_), so a host write through a freed
pointer during the run or the teardown aborts the child.  Passing = exit
status 0 and nothing on stderr (the image's libdrm `amdgpu.ids` notice
aside).  The host-instrumented (AddressSanitizer) replay of the same
sequence is tools/teardown_probe.cpp.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, sys
import numpy as np
sys.path.insert(0, %(pkg)r)
sys.path.insert(0, %(tests)r)
from audiotools import _atgpu
import signals

FLAC8 = dict(block_size=4096, max_lpc_order=12, min_residual_partition_order=0,
             max_residual_partition_order=6,
             mid_side=True, exhaustive_model_search=True)
lib = _atgpu.load_library()
eng = _atgpu.Engine(0)
opts = _atgpu.make_options(**FLAC8)
pcms = [signals.make("tone" if t %% 3 else "noise", 4096 * 6 + 77 * t, 2, 16, seed=t)
        for t in range(48)]
tracks, pos = [], 0
for p in pcms:
    tracks.append((pos, len(p) // 2))
    pos += len(p) // 2
pcm = np.concatenate(pcms).astype(np.int16)
nf, nb = eng.bounds(opts, tracks, 2, 16)

# host jobs: pinned in / out, then pageable
pin = _atgpu.pinned_empty(pcm.shape, np.int16)
pin[:] = pcm
pout = _atgpu.pinned_empty(nb)
out, res, _, _ = eng.encode_async(opts, pin, tracks, 2, 16, 44100, out=pout).wait()
out2, res2, _, _ = eng.encode(opts, pcm, tracks, 2, 16, 44100)
assert all(out[a.out_offset:a.out_offset + a.bytes].tobytes() ==
           out2[b.out_offset:b.out_offset + b.bytes].tobytes() for a, b in zip(res, res2))
eng.encode_async(opts, pcm, tracks, 2, 16, 44100).wait()

# device batches at depth 12 (rolled MD5), the last two never waited
def dalloc(n):
    p = ctypes.c_void_p()
    assert lib.atg_device_alloc(eng.handle, n, ctypes.byref(p)) == 0
    return p.value
d_pcm = dalloc(pcm.nbytes)
assert lib.atg_copy_to_device(eng.handle, ctypes.c_void_p(d_pcm),
                              pcm.ctypes.data_as(ctypes.c_void_p), pcm.nbytes) == 0
eng.set_inflight(12)
outs = [dalloc(nb) for _ in range(12)]
table = _atgpu.TrackTable(tracks)
pend = []
for k in range(30):
    pend.append(eng.encode_device_async(opts, d_pcm, _atgpu.PCM_S16, table, 2, 16, 44100,
                                        outs[k %% 12], nb))
    if len(pend) >= 12:
        r = eng.wait(pend.pop(0))
while len(pend) > 2:
    r = eng.wait(pend.pop(0))

# decode the batch images at depth 8, two batches never waited
img = np.empty(nb, dtype=np.uint8)
eng.copy_to_host(img, outs[0])
dec = _atgpu.Decoder(0)
dec.set_inflight(8)
dtr = []
for t in r:  # the device images' layout (the host jobs pack theirs)
    rc, si, _ = _atgpu.read_metadata(img[t.out_offset:t.out_offset + t.bytes].tobytes())
    assert rc == 0
    dtr.append(_atgpu.dec_track(t.out_offset + si.frames_offset, t.bytes - si.frames_offset, si))
dp = []
for k in range(12):
    dp.append(dec.decode_device_async(outs[0], nb, dtr))
    if len(dp) >= 8:
        dres = dec.decode_wait(dp.pop(0))[0]
        assert all(x.status == 0 for x in dres)
while len(dp) > 2:
    dec.decode_wait(dp.pop(0))
# the process-wide default engine, a pageable host job left in flight on it
dangling = _atgpu.engine().encode_async(opts, pcm, tracks, 2, 16, 44100)
print("child done", flush=True)
# exit with everything open
"""


@pytest.mark.gpu
def test_exit_with_work_in_flight():
    env = dict(os.environ)
    env.update(MALLOC_CHECK_="3", MALLOC_PERTURB_="165")
    script = CHILD % {"pkg": os.path.join(ROOT, "python-audio-tools_amd"),
                      "tests": os.path.join(ROOT, "tests")}
    p = subprocess.run([sys.executable, "-c", script], env=env, capture_output=True,
                       text=True, timeout=240)
    err = "\n".join(l for l in p.stderr.splitlines() if "amdgpu.ids" not in l)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], err[-4000:])
    assert "child done" in p.stdout
    assert err.strip() == "", err[-4000:]
