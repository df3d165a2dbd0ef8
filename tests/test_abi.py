"""CPU: the C-ABI library libatgpu.so loads, exports every function that
include/atgpu.h declares, and its host-side logic (planning, option
validation, batch bounds) works without a GPU.  No kernel is launched."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from audiotools import _atgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "atgpu.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    return sorted(set(re.findall(r"\b(atg_[a-z0-9_]+)\s*\(", text)))


def test_header_and_binding_agree():
    decl = declared_functions()
    assert decl, "no functions parsed from include/atgpu.h"
    assert sorted(_atgpu.EXPORTS) == decl


def test_library_exports_every_declared_symbol():
    lib = _atgpu.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", _atgpu.LIB_PATH],
                        capture_output=True, text=True, check=True).stdout
    exported = set(l.split()[-1] for l in nm.splitlines() if l.strip())
    for name in declared_functions():
        assert name in exported, name


def test_abi_version_matches_header():
    lib = _atgpu.load_library()
    m = re.search(r"#define\s+ATG_ABI_VERSION\s+(\d+)", open(HEADER).read())
    assert lib.atg_abi_version() == int(m.group(1))


def gpu_visible():
    return os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "x") != ""


@pytest.mark.skipif(gpu_visible(), reason="a GPU is visible: covered by -m gpu tests")
def test_engine_create_fails_loudly_without_gpu():
    with pytest.raises(_atgpu.ATGError) as e:
        _atgpu.Engine(0)
    assert e.value.status == _atgpu.ATG_ERR_DEVICE


def flac8(**kw):
    d = dict(block_size=4096, max_lpc_order=12, min_residual_partition_order=0,
             max_residual_partition_order=6, mid_side=True, exhaustive_model_search=True)
    d.update(kw)
    return _atgpu.make_options(**d)


def bounds(opts, tracks, ch=2, bps=16):
    lib = _atgpu.load_library()
    arr, n, _keep = _atgpu._track_array(tracks)
    nf, nb = ctypes.c_uint64(), ctypes.c_uint64()
    st = lib.atg_flac_batch_bounds(ctypes.byref(opts), arr, n, ch, bps,
                                   ctypes.byref(nf), ctypes.byref(nb))
    return st, nf.value, nb.value


def test_batch_bounds_frame_count_and_capacity():
    import oracle_port
    import signals
    tracks = [(0, 4096 * 3 + 5), (20000, 100), (30000, 0), (40000, 4096)]
    st, nf, nb = bounds(flac8(), tracks)
    assert st == _atgpu.ATG_OK
    assert nf == 4 + 1 + 0 + 1
    # the worst case covers what the oracle writes for white noise
    worst = 0
    for _, n in tracks:
        pcm = signals.noise(n, 2, 16, n + 1)
        worst += len(oracle_port.encode(pcm, 2, 16, 44100, **oracle_port.PRESETS["8"])[0])
    assert nb >= worst


def test_explicit_frame_sizes_checked():
    sizes = np.array([4096, 1000, 5], dtype=np.uint32)
    st, nf, _ = bounds(flac8(), [(0, 5101, sizes)])
    assert st == _atgpu.ATG_OK and nf == 3
    st, _, _ = bounds(flac8(), [(0, 5000, sizes)])
    assert st == _atgpu.ATG_ERR_INVALID


@pytest.mark.parametrize("kw,ch,bps,status", [
    (dict(block_size=65536), 2, 16, _atgpu.ATG_ERR_UNSUPPORTED),
    (dict(max_residual_partition_order=16), 2, 16, _atgpu.ATG_ERR_INVALID),
    (dict(block_size=0), 2, 16, _atgpu.ATG_ERR_INVALID),
    (dict(max_lpc_order=33), 2, 16, _atgpu.ATG_ERR_INVALID),
    (dict(), 9, 16, _atgpu.ATG_ERR_INVALID),
    (dict(), 2, 32, _atgpu.ATG_ERR_UNSUPPORTED),
])
def test_option_validation(kw, ch, bps, status):
    st, _, _ = bounds(flac8(**kw), [(0, 10000)], ch, bps)
    assert st == status
    assert _atgpu.load_library().atg_last_error()


@pytest.mark.parametrize("kw", [dict(block_size=8192), dict(block_size=65535),
                                dict(max_residual_partition_order=15)])
def test_large_frame_options_accepted(kw):
    """block sizes up to 65535 and partition orders up to 15 take the
    large-frame path (flac_big.hip), as the reference encoder accepts them"""
    st, nf, nb = bounds(flac8(**kw), [(0, 100000)])
    assert st == _atgpu.ATG_OK and nf >= 2 and nb > 0


def test_null_arguments_rejected():
    lib = _atgpu.load_library()
    assert lib.atg_engine_create(0, None) == _atgpu.ATG_ERR_INVALID
    lib.atg_engine_destroy(None)  # no-op
    assert lib.atg_engine_kernel_times(None, None, None, 0) == 0


@pytest.mark.parametrize("ch,bps,rate,n,pad", [(2, 16, 44100, 30000, 4096), (6, 24, 48000, 9001, 0),
                                               (1, 8, 8000, 0, 100), (2, 16, 700000, 5, 4096)])
def test_host_stream_header_matches_port(ch, bps, rate, n, pad):
    """atg_flac_stream_header (host code, no GPU): the streaming encoder's
    header equals the whole-stream header the oracle writes -- STREAMINFO
    fields and MD5 as given, VORBIS_COMMENT vendor, PADDING"""
    import hashlib
    import oracle_port
    import signals
    from audiotools.encoders import pcm_le_bytes
    x = signals.make("tone", n, ch, bps, seed=n) if n else np.zeros(0, np.int32)
    opts = dict(oracle_port.PRESETS["8"], padding_size=pad)
    img, lst = oracle_port.encode(x, ch, bps, rate, **opts)
    blocks, frames = oracle_port.split_flac(img)
    hdr_len = len(img) - len(frames)
    sizes = []
    for k, (off, _) in enumerate(lst):
        end = lst[k + 1][0] if k + 1 < len(lst) else len(frames)
        sizes.append(end - off)
    md5 = hashlib.md5(pcm_le_bytes(x, bps)).digest()
    got = _atgpu.stream_header(_atgpu.make_options(**opts), ch, bps, rate, n,
                               min(sizes) if sizes else 0xFFFFFF, max(sizes) if sizes else 0,
                               md5)
    assert got == img[:hdr_len]
