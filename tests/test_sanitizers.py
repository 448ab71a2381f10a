"""ASan/UBSan build of the host-side store + socket code."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_store_under_asan(tmp_path):
    exe = tmp_path / "store_selftest"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           f"-I{REPO}/csrc", f"{REPO}/csrc/selftest/store_selftest.cpp", f"{REPO}/csrc/store/tcp_store.cpp",
           "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
