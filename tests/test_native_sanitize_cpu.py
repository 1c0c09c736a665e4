"""Host-code sanitizer run: the native crc32c used by the TF-V2-bundle checkpoint
codec, built with AddressSanitizer + UndefinedBehaviorSanitizer (host only -- GPU sanitizers are
not available on the MI355X pool) and checked against a bitwise reference on every length and
misalignment."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_crc32c_asan_ubsan(tmp_path):
    exe = str(tmp_path / "crc32c_san")
    src = os.path.join(HERE, "native", "crc32c_sanitize_main.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", src, "-o", exe], check=True, capture_output=True, timeout=120)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout
