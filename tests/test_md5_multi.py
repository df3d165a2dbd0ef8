"""CPU: the host MD5 the engine's host-hash mode runs (md5_cpu.h
hash_bytes_multi: one core hashes 16 tracks side by side in AVX-512 lanes)
equals its scalar path on random stream counts (1-16) and lengths (equal
and unequal, 0-5000 bytes), and RFC 1321's MD5("abc").  Built with g++ from
tools/md5_multi_check.cpp; the vector path is exercised only where the CPU
has AVX-512 (the check still compares the scalar path with itself elsewhere)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_multi_stream_md5_matches_scalar(tmp_path):
    exe = str(tmp_path / "md5_multi_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tools", "md5_multi_check.cpp")], check=True)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    first = p.stdout.splitlines()[0].split()
    assert first[0] == "cases" and int(first[1]) > 2000 and first[3] == "0"
    assert first[5] == "90015098"  # MD5("abc") = 90015098 3cd24fb0 ...
