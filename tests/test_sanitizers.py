"""ASan/UBSan builds of the host-side native code:

* the TCP store + socket layer (csrc/selftest/store_selftest.cpp);
* the host communicator's ring collectives and the Reducer's threaded
  hook / launch / finalize / rebuild logic, driven by world_size=2 forked ranks
  doing real libtorch autograd backward passes (csrc/selftest/reducer_selftest.cpp:
  synced averages, no_sync accumulation, find_unused_parameters,
  gradient_as_bucket_view).

The sanitizer runtime is linked statically into the test executables, so
nothing is preloaded.
"""
import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize=vptr", "-fno-omit-frame-pointer"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_store_under_asan(tmp_path):
    exe = tmp_path / "store_selftest"
    cmd = ["g++", "-std=c++17", "-O1", "-g", *SAN, "-static-libasan", f"-I{REPO}/csrc",
           f"{REPO}/csrc/selftest/store_selftest.cpp", f"{REPO}/csrc/store/tcp_store.cpp", "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True)
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_reducer_and_host_comm_under_asan(tmp_path):
    import torch

    tdir = os.path.dirname(torch.__file__)
    lib = os.path.join(tdir, "lib")
    if not glob.glob(os.path.join(lib, "libc10_hip.so")):
        pytest.skip("ROCm torch libraries not present")
    inc = [f"-I{REPO}/csrc", f"-I{tdir}/include", f"-I{tdir}/include/torch/csrc/api/include",
           f"-I{sys.base_prefix}/include/python{sys.version_info.major}.{sys.version_info.minor}", "-I/opt/rocm/include"]
    flags = ["-O1", "-g", "-fPIC", "-std=c++17", *SAN, "-Wno-deprecated-declarations", "-D__HIP_PLATFORM_AMD__=1",
             "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1", *inc]
    srcs = ["selftest/reducer_selftest", "selftest/kern_stubs", "reducer/reducer", "comm/host_comm",
            "comm/communicator", "store/tcp_store", "trace/trace", "ops"]

    def compile_one(s):
        obj = tmp_path / (s.replace("/", "_") + ".o")
        r = subprocess.run(["g++", *flags, "-c", f"{REPO}/csrc/{s}.cpp", "-o", str(obj)], capture_output=True,
                           text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        return str(obj)

    with ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    exe = tmp_path / "reducer_selftest"
    r = subprocess.run(["g++", *SAN, "-static-libasan", *objs, f"-L{lib}", f"-Wl,-rpath,{lib}", "-ltorch",
                        "-ltorch_cpu", "-lc10", "-lc10_hip", "-ltorch_hip", "-lamdhip64", "-lpthread", "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe), "2"], capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-5000:]
    assert r.stdout.strip().endswith("OK"), r.stdout
    assert r.stdout.count(" ok") == 4
