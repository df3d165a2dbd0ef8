"""GPU: the encoder service (atgpu-encoderd, csrc/encoderd.cpp; client
csrc/service.hip).  Fresh processes -- as track2track's conversion processes
are (reference audiotools/__init__.py:5494-5521) -- call encode_flac; the
first starts the service, every process's segments are encoded there (the
processes never open the GPU themselves), concurrent processes' segments
share GPU batches, and every file equals the port's encode of its PCM.
Each test uses its own socket name (ATG_ENCODER_SOCKET), so a service left
idle by another test or run is never reused."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import oracle_port
import signals

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CHILD = r"""
import json, os, sys
sys.path.insert(0, %(pkg)r)
sys.path.insert(0, %(tests)r)
import numpy as np
import audiotools
from audiotools import encoders
import signals
spec = json.loads(sys.argv[1])
x = signals.make(spec["kind"], spec["n"], spec["ch"], spec["bps"], seed=spec["seed"])
r = audiotools.FrameListReader(x, 44100, spec["ch"], spec["bps"])
if spec.get("sizes"):
    class R(object):
        def __init__(self):
            self.sample_rate, self.channels = 44100, spec["ch"]
            self.bits_per_sample, self.channel_mask = spec["bps"], 0
            self.sizes = list(spec["sizes"])
        def read(self, n):
            return r.read(self.sizes.pop(0) if self.sizes else n)
        def close(self):
            pass
    reader = R()
else:
    reader = r
offs = encoders.encode_flac(spec["out"], reader, **spec["opts"])
kfd = any("/dev/kfd" in ln for ln in open("/proc/self/maps"))
print(json.dumps({"offsets": offs, "gpu_opened": kfd}))
""" % {"pkg": os.path.join(ROOT, "python-audio-tools_amd"), "tests": HERE}


def _run(specs, sock):
    env = dict(os.environ, ATG_ENCODER_SOCKET=sock)
    env.pop("ATG_ENCODER_SERVICE", None)
    procs = [subprocess.Popen([sys.executable, "-c", CHILD, json.dumps(s)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for s in specs]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    return outs


def _check(spec, got):
    x = signals.make(spec["kind"], spec["n"], spec["ch"], spec["bps"], seed=spec["seed"])
    fs = None
    if spec.get("sizes"):
        fs = spec["sizes"]
    want, wl = oracle_port.encode(x, spec["ch"], spec["bps"], 44100, frame_sizes=fs,
                                  **spec["opts"])
    assert open(spec["out"], "rb").read() == want, spec
    assert [tuple(o) for o in got["offsets"]] == wl
    assert not got["gpu_opened"], "the client process opened the GPU itself"


def test_service_concurrent_processes(tmp_path):
    """8 processes at once (track2track -j 8): the first starts the service,
    all are served by it, files byte-equal to the port"""
    sock = "atgpu-test-%d-%d" % (os.getpid(), int(time.time() * 1e3) % 100000)
    opts = dict(oracle_port.PRESETS["8"])
    specs = [dict(kind=["tone", "noise", "chirp", "sine"][k % 4], n=4096 * 9 + 37 * k, ch=2,
                  bps=16, seed=k, opts=opts, out=str(tmp_path / ("t%d.flac" % k)))
             for k in range(8)]
    for spec, got in zip(specs, _run(specs, sock)):
        _check(spec, got)


def test_service_mixed_formats_and_sizes(tmp_path):
    """concurrent requests of different formats / presets / explicit frame
    sizes (grouped per format in the service), and a stream longer than one
    256-frame segment"""
    sock = "atgpu-test-mix-%d" % os.getpid()
    specs = [
        dict(kind="tone", n=4096 * 300 + 5, ch=2, bps=16, seed=1,
             opts=dict(oracle_port.PRESETS["8"])),
        dict(kind="chirp", n=20000, ch=6, bps=24, seed=2, opts=dict(oracle_port.PRESETS["8"])),
        dict(kind="noise", n=9000, ch=1, bps=8, seed=3, opts=dict(oracle_port.PRESETS["5"])),
        dict(kind="tone", n=15000, ch=2, bps=16, seed=4, opts=dict(oracle_port.PRESETS["8"]),
             sizes=[4096, 1000, 7, 4096]),
        dict(kind="sine", n=3000, ch=2, bps=24, seed=5, opts=dict(oracle_port.PRESETS["0"])),
    ]
    for k, s in enumerate(specs):
        s["out"] = str(tmp_path / ("m%d.flac" % k))
    for spec, got in zip(specs, _run(specs, sock)):
        _check(spec, got)


def test_service_refuses_bad_options(tmp_path):
    """invalid options raise the local path's exception (ValueError) in a
    process served by the service"""
    sock = "atgpu-test-err-%d" % os.getpid()
    env = dict(os.environ, ATG_ENCODER_SOCKET=sock)
    code = CHILD.replace('offs = encoders.encode_flac(spec["out"], reader, **spec["opts"])',
                         'try:\n    encoders.encode_flac(spec["out"], reader, **spec["opts"])\n'
                         'except ValueError as e:\n    print(json.dumps({"error": str(e)}))\n'
                         '    sys.exit(0)\nsys.exit(3)')
    spec = dict(kind="tone", n=5000, ch=2, bps=16, seed=1, out=str(tmp_path / "e.flac"),
                opts=dict(block_size=4096, max_lpc_order=40, min_residual_partition_order=0,
                          max_residual_partition_order=6))
    p = subprocess.run([sys.executable, "-c", code, json.dumps(spec)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "error" in json.loads(p.stdout.strip().splitlines()[-1])
