"""CPU: the encoder service's client (csrc/service.hip) against fake
services -- host code only, no kernel runs.

The service name is an abstract Unix socket, which has no permissions, so
the client must not trust whoever answers on it:
  * a reply whose frame count differs from the request (the old client
    copied 4 * n_frames bytes into a 256-entry buffer), whose frame sizes do
    not add up, whose byte count exceeds the segment's bound, or whose error
    text is oversized is refused with ATG_ERR_DEVICE (the caller then uses
    an engine of its own) and nothing is written past the caller's buffers;
  * a service that never answers is given up after the deadline
    (ATG_SERVICE_TIMEOUT_MS), not waited on forever;
  * a well-formed reply is accepted.
The peer-uid check (SO_PEERCRED) cannot be exercised here without a second
user; its code path is the same getsockopt the daemon uses on accept.
"""
import ctypes
import os
import socket
import struct
import threading
import time

import numpy as np
import pytest

from audiotools import _atgpu

REQ_HDR = 104   # atg_svc_request (service.h): 2 u32, options (12 u32), 4 u32, 4 u64
ATG_OK, ATG_ERR_DEVICE = 0, -3


def _lib():
    lib = _atgpu.load_library()
    lib.atg_service_connect.argtypes = [ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_void_p)]
    lib.atg_service_connect.restype = ctypes.c_int
    lib.atg_service_close.argtypes = [ctypes.c_void_p]
    lib.atg_service_last_error.restype = ctypes.c_char_p
    u64, u32p = ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)
    lib.atg_service_encode_frames.argtypes = [
        ctypes.c_void_p, ctypes.POINTER(_atgpu.FlacOptions), ctypes.c_void_p, ctypes.c_int,
        u64, u32p, u64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u64,
        ctypes.c_void_p, u64, ctypes.POINTER(u64), u32p]
    lib.atg_service_encode_frames.restype = ctypes.c_int
    return lib


class FakeService(object):
    """one connection: read the request, then send `reply(request)`"""

    def __init__(self, name, reply):
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.bind("\0" + name)
        self.sock.listen(4)
        self.reply = reply
        self.t = threading.Thread(target=self.run, daemon=True)
        self.t.start()

    def run(self):
        c, _ = self.sock.accept()
        buf = b""
        while len(buf) < REQ_HDR:
            buf += c.recv(65536)
        n_sizes, pcm_bytes = struct.unpack_from("<Q", buf, 88)[0], struct.unpack_from("<Q", buf, 96)[0]
        need = REQ_HDR + 4 * n_sizes + pcm_bytes
        while len(buf) < need:
            buf += c.recv(65536)
        out = self.reply(buf)
        if out is not None:
            try:
                c.sendall(out)
            except OSError:   # the client hung up on a refused reply
                pass
        time.sleep(1.0)
        c.close()

    def close(self):
        self.sock.close()


def _encode(lib, name, n_frames_pcm=4096 * 3, frame_bytes_cap=256, out_cap=1 << 20,
            timeout_ms=None):
    os.environ["ATG_ENCODER_SOCKET"] = name
    if timeout_ms is not None:
        os.environ["ATG_SERVICE_TIMEOUT_MS"] = str(timeout_ms)
    try:
        svc = ctypes.c_void_p()
        assert lib.atg_service_connect(0, 0, ctypes.byref(svc)) == ATG_OK
        opts = _atgpu.make_options(4096, 12, 0, 6, mid_side=1, exhaustive_model_search=1)
        pcm = np.zeros(n_frames_pcm * 2, dtype=np.int16)
        # guard words past the frame_bytes buffer catch any overflow
        fb = np.full(frame_bytes_cap + 64, 0xA5A5A5A5, dtype=np.uint32)
        out = np.zeros(out_cap, dtype=np.uint8)
        nb = ctypes.c_uint64(0)
        t0 = time.time()
        st = lib.atg_service_encode_frames(
            svc, ctypes.byref(opts), pcm.ctypes.data, _atgpu.PCM_S16, n_frames_pcm, None, 0,
            2, 16, 44100, 0, out.ctypes.data, out_cap, ctypes.byref(nb),
            fb.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        dt = time.time() - t0
        err = lib.atg_service_last_error().decode()
        lib.atg_service_close(svc)
        assert (fb[frame_bytes_cap:] == 0xA5A5A5A5).all(), "frame_bytes overflowed"
        return st, err, dt, fb, nb.value, out
    finally:
        os.environ.pop("ATG_ENCODER_SOCKET", None)
        os.environ.pop("ATG_SERVICE_TIMEOUT_MS", None)


def _resp(status, msg=b"", n_frames=0, sizes=(), body=b"", out_bytes=None):
    ob = len(body) if out_bytes is None else out_bytes
    return (struct.pack("<iIQQ", status, len(msg), ob, n_frames) + msg +
            struct.pack("<%dI" % len(sizes), *sizes) + body)


def _name(tag):
    return "atg-test-fake-%d-%s-%d" % (os.getpid(), tag, time.monotonic_ns())


def test_reply_with_oversized_frame_count_is_refused():
    lib = _lib()
    name = _name("nf")
    # 100000 "frame sizes" for a 3-frame segment: the old client copied
    # 400 KB into a 256-entry buffer
    fake = FakeService(name, lambda req: _resp(0, n_frames=100000, sizes=[1] * 100000,
                                               body=b"\0" * 100000))
    st, err, _, _, _, _ = _encode(lib, name)
    fake.close()
    assert st == ATG_ERR_DEVICE and "frame count" in err


def test_reply_with_wrong_sizes_or_bound_is_refused():
    lib = _lib()
    cases = [(_resp(0, n_frames=3, sizes=[10, 10, 10], body=b"\0" * 31), "add up"),
             (_resp(0, n_frames=3, sizes=[1 << 30, 1 << 30, 1 << 30], body=b"",
                    out_bytes=3 << 30), "bound"),
             (struct.pack("<iIQQ", -1, 1 << 30, 0, 0), "malformed"),
             (_resp(-1, msg=b"x", n_frames=5), "malformed")]
    for reply, what in cases:
        name = _name("sz")
        fake = FakeService(name, lambda req, r=reply: r)
        st, err, _, _, _, _ = _encode(lib, name)
        fake.close()
        assert st == ATG_ERR_DEVICE and what in err, (what, err)


def test_silent_service_times_out():
    lib = _lib()
    name = _name("to")
    fake = FakeService(name, lambda req: None)
    st, err, dt, _, _, _ = _encode(lib, name, timeout_ms=300)
    fake.close()
    assert st == ATG_ERR_DEVICE and "timed out" in err
    assert dt < 5.0


def test_error_reply_reaches_the_caller():
    lib = _lib()
    name = _name("err")
    fake = FakeService(name, lambda req: _resp(-2, msg=b"unsupported thing"))
    st, err, _, _, _, _ = _encode(lib, name)
    fake.close()
    assert st == -2 and err == "unsupported thing"


def test_well_formed_reply_is_accepted():
    lib = _lib()
    name = _name("ok")
    body = bytes(range(30))
    fake = FakeService(name, lambda req: _resp(0, n_frames=3, sizes=[10, 12, 8], body=body))
    st, err, _, fb, nb, out = _encode(lib, name)
    fake.close()
    assert st == ATG_OK, err
    assert nb == 30 and bytes(out[:30]) == body and list(fb[:3]) == [10, 12, 8]
