"""Device choice for the drop-in entry points (csrc/devices.hip), on CPU:
no HIP call is made, so the node-wide round robin, the environment overrides
and the visible-device count are exercised here with a mocked device count
(ATG_DEVICE_COUNT / HIP_VISIBLE_DEVICES) and a private counter file
(ATG_RR_FILE).  Reference: track2track forks one process per track
(audiotools/__init__.py:5263-5529); here those processes spread over the
node's GPUs."""
import collections
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-audio-tools_amd")

PICK = ("import sys; sys.path.insert(0, %r); from audiotools import _atgpu; "
        "print(_atgpu.default_device(), _atgpu.visible_devices())" % PKG)


def _env(tmp_path, **kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("ATG_DEVICE", "LOCAL_RANK", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                        "ROCR_VISIBLE_DEVICES", "ATG_DEVICE_COUNT")}
    env["ATG_RR_FILE"] = str(tmp_path / "rr")
    env.update({k: str(v) for k, v in kw.items()})
    return env


def _pick(env):
    out = subprocess.run([sys.executable, "-c", PICK], env=env, capture_output=True, text=True,
                         check=True).stdout.split()
    return int(out[0]), int(out[1])


def test_round_robin_over_visible_devices(tmp_path):
    env = _env(tmp_path, ATG_DEVICE_COUNT=4)
    picks = [_pick(env) for _ in range(8)]
    assert all(n == 4 for _, n in picks)
    assert collections.Counter(d for d, _ in picks) == {0: 2, 1: 2, 2: 2, 3: 2}
    assert [d for d, _ in picks] == [0, 1, 2, 3, 0, 1, 2, 3]


def test_parallel_processes_share_the_counter(tmp_path):
    env = _env(tmp_path, HIP_VISIBLE_DEVICES="0,1,2,3,4,5,6,7")
    procs = [subprocess.Popen([sys.executable, "-c", PICK], env=env, stdout=subprocess.PIPE,
                              text=True) for _ in range(16)]
    got = [int(p.communicate()[0].split()[0]) for p in procs]
    assert collections.Counter(got) == {d: 2 for d in range(8)}


def test_overrides_and_counts(tmp_path):
    assert _pick(_env(tmp_path, ATG_DEVICE_COUNT=8, ATG_DEVICE=5))[0] == 5
    assert _pick(_env(tmp_path, ATG_DEVICE_COUNT=8, LOCAL_RANK=3))[0] == 3
    assert _pick(_env(tmp_path, ATG_DEVICE_COUNT=8, ATG_DEVICE=1, LOCAL_RANK=3))[0] == 1
    assert _pick(_env(tmp_path, HIP_VISIBLE_DEVICES="2,5,7"))[1] == 3
    assert _pick(_env(tmp_path, ROCR_VISIBLE_DEVICES="0,1"))[1] == 2
    assert _pick(_env(tmp_path, HIP_VISIBLE_DEVICES="3"))[0] == 0  # one device: always 0


def test_fork_picks_again(tmp_path):
    code = ("import os, sys; sys.path.insert(0, %r); from audiotools import _atgpu\n"
            "a = _atgpu.default_device(); b = _atgpu.default_device()\n"
            "r, w = os.pipe()\n"
            "pid = os.fork()\n"
            "if pid == 0:\n"
            "    os.write(w, str(_atgpu.default_device()).encode()); os._exit(0)\n"
            "os.waitpid(pid, 0); print(a, b, os.read(r, 16).decode())\n" % PKG)
    env = _env(tmp_path, ATG_DEVICE_COUNT=4)
    a, b, c = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                             text=True, check=True).stdout.split()
    assert (a, b, c) == ("0", "0", "1")  # decided once per process, again after fork
