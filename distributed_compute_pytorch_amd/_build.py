"""Native build driver: compiles csrc/ into the in-tree extension ``_C``.

No hipify, no CUDA: ``.hip`` sources go through ``hipcc --offload-arch=gfx950``,
``.cpp`` sources (torch/pybind glue, store, communicators, reducer) through the
host C++ compiler with the same flags torch's ROCm extensions use, and the
objects are linked against torch's bundled ``libamdhip64`` / ``librccl`` so a
single HIP runtime and a single RCCL live in the process.

The resulting ``distributed_compute_pytorch_amd/_C*.so`` is git-ignored but
travels to the GPU box with the repo snapshot.

Usage: ``python -m distributed_compute_pytorch_amd._build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import re
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
EXT_NAME = "_C"


def _torch_paths():
    import torch

    root = Path(torch.__file__).resolve().parent
    return root / "include", root / "lib"


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG_DIR / f"{EXT_NAME}{suffix}"


def _flags():
    inc, _ = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    defs = [
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-DHIPBLAS_V2",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-D_GLIBCXX_USE_CXX11_ABI=1",
    ]
    incs = [
        f"-I{CSRC}",
        f"-I{inc}",
        f"-I{inc / 'torch' / 'csrc' / 'api' / 'include'}",
        f"-I{py_inc}",
        f"-I{ROCM / 'include'}",
    ]
    common = ["-O3", "-fPIC", "-std=c++17", "-Wno-unused-parameter", "-Wno-deprecated-declarations"]
    cxx = ["g++"] + common + defs + incs + ["-fvisibility=hidden"]
    hip = (
        # VGPR-form MFMA: accumulators in the unified VGPR file instead of
        # AGPRs — the attention kernels' softmax / rescale no longer pays a
        # v_accvgpr read + write per element (fwd VALU -26 %, dK/dV 332 → 199
        # registers: two waves per SIMD instead of one; NOTES §22)
        [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-mllvm",
         "-amdgpu-mfma-vgpr-form"]
        + common
        + defs
        + incs
        + [
            "-D__HIP_NO_HALF_OPERATORS__=1",
            "-D__HIP_NO_HALF_CONVERSIONS__=1",
            "-fno-gpu-rdc",
        ]
    )
    return cxx, hip


# per-source extra compile flags (relative to csrc/)
_FILE_FLAGS = {
    # the attention kernels feed MFMA outputs to fmaxf: under IEEE NaN
    # handling hipcc quiets each operand first (one v_max x, x per score —
    # 33 of the forward's ~500 VALU instructions per key block, in a
    # VALU-bound loop); nothing in the file depends on NaN semantics
    "kernels/attention.hip": ["-fno-honor-nans"],
    # the LM-head GEMM's softmax-partials epilogue (EPI 7): 9 quieting v_max
    # per row of 8 logits per lane otherwise (the bf16 unpacks and DPP moves
    # are not known canonical); the file tests ±inf, never NaN
    "kernels/gemm_pp.hip": ["-fno-honor-nans"],
}


def _file_flags(src: Path) -> list:
    return _FILE_FLAGS.get(str(src.relative_to(CSRC)), [])


def _link_cmd(objs, out):
    _, lib = _torch_paths()
    return (
        ["g++", "-shared", "-o", str(out)]
        + [str(o) for o in objs]
        + [
            f"-L{lib}",
            "-ltorch",
            "-ltorch_cpu",
            "-ltorch_python",
            "-lc10",
            "-lc10_hip",
            "-ltorch_hip",
            f"{lib / 'libamdhip64.so'}",
            f"{lib / 'librccl.so'}",
            f"-Wl,-rpath,{lib}",
            "-Wl,--no-as-needed",
            "-ldl",
        ]
    )


def _sources():
    srcs = sorted(CSRC.rglob("*.cpp")) + sorted(CSRC.rglob("*.hip"))
    # standalone sanitizer / self-test programs are not part of the extension
    return [s for s in srcs if "selftest" not in s.parts]


def _header_digest():
    h = hashlib.sha1()
    for p in sorted(list(CSRC.rglob("*.h")) + list(CSRC.rglob("*.cuh")) + list(CSRC.rglob("*.inc"))):
        h.update(p.read_bytes())
    return h.hexdigest()


DIGEST_SYMBOL = "dcp_source_digest"


def source_digest() -> str:
    """Content digest of everything the extension is built from: every source
    and header (relative path + bytes) and the compile / link flags with the
    checkout's location masked out (the GPU box runs the same tree from a
    different path). Embedded into ``_C`` at link time (``DIGEST_SYMBOL``) and
    checked by ``_ext.load()`` before the extension is imported, so a stale
    binary is rebuilt or refused instead of tested silently."""
    h = hashlib.sha1()
    files = _sources() + sorted(list(CSRC.rglob("*.h")) + list(CSRC.rglob("*.cuh")) + list(CSRC.rglob("*.inc")))
    for p in sorted(files):
        h.update(str(p.relative_to(CSRC)).encode() + b"\0")
        h.update(p.read_bytes())
    cxx, hip = _flags()
    h.update(" ".join(cxx + hip).replace(str(CSRC), "<csrc>").encode())
    h.update(repr(sorted(_FILE_FLAGS.items())).encode())
    return h.hexdigest()


DIGEST_MARKER = b"DCP_SRC_DIGEST:"


def embedded_digest(so: Path) -> str | None:
    """The source digest linked into ``so`` (None if it carries none).

    Read from the file's bytes (the digest object stores ``DIGEST_MARKER``
    followed by the 40 hex digits), never by loading the library: a dlopen of
    a stale ``_C`` here would stay mapped, and the import after a rebuild at
    the same path would get that old mapping back from the dynamic loader."""
    import mmap

    try:
        with open(so, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
            i = m.find(DIGEST_MARKER)
            if i < 0:
                return None
            d = m[i + len(DIGEST_MARKER):i + len(DIGEST_MARKER) + 40]
    except (OSError, ValueError):
        return None
    try:
        d = d.decode("ascii")
    except UnicodeDecodeError:
        return None
    return d if re.fullmatch(r"[0-9a-f]{40}", d) else None


def _digest_obj(cxx, digest: str) -> Path:
    src = BUILD / f"digestm.{digest[:16]}.cpp"
    obj = BUILD / f"digestm.{digest[:16]}.o"
    if not obj.exists():
        marker = DIGEST_MARKER.decode()
        src.write_text(f'extern "C" __attribute__((visibility("default"), used)) const char '
                       f'{DIGEST_SYMBOL}[{len(marker) + 41}] = "{marker}{digest}";\n')
        r = subprocess.run(cxx + ["-c", str(src), "-o", str(obj)], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj


def _obj_for(src: Path, cmd, hdr):
    rel = src.relative_to(CSRC)
    key = hashlib.sha1((" ".join(cmd) + hdr).encode() + src.read_bytes()).hexdigest()[:16]
    return BUILD / (str(rel).replace("/", "__") + f".{key}.o")


def build(jobs: int | None = None, force: bool = False, verbose: bool = False) -> Path:
    """Compile every native source for gfx950 and link ``_C``. Returns the .so path."""
    BUILD.mkdir(parents=True, exist_ok=True)
    cxx, hip = _flags()
    hdr = _header_digest()
    tasks = []
    objs = []
    for src in _sources():
        cmd = (hip if src.suffix == ".hip" else cxx) + _file_flags(src)
        obj = _obj_for(src, cmd, hdr)
        objs.append(obj)
        if force or not obj.exists():
            tasks.append((src, cmd, obj))

    def compile_one(t):
        src, cmd, obj = t
        full = cmd + (["-x", "hip"] if src.suffix == ".hip" else []) + ["-c", str(src), "-o", str(obj) + ".tmp"]
        if verbose:
            print(" ".join(full), flush=True)
        r = subprocess.run(full, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
        os.replace(str(obj) + ".tmp", obj)
        return src

    if tasks:
        n = jobs or min(8, os.cpu_count() or 4)
        with ThreadPoolExecutor(max_workers=n) as ex:
            for src in ex.map(compile_one, tasks):
                print(f"[dcp build] compiled {src.relative_to(REPO)}", flush=True)
    objs.append(_digest_obj(cxx, source_digest()))
    out = ext_path()
    newest_obj = max(o.stat().st_mtime for o in objs)
    if force or tasks or not out.exists() or out.stat().st_mtime < newest_obj:
        tmp = out.with_suffix(".tmp.so")
        r = subprocess.run(_link_cmd(objs, tmp), capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out)
        print(f"[dcp build] linked {out.relative_to(REPO)}", flush=True)
    # drop stale objects
    keep = {o.name for o in objs}
    for o in BUILD.glob("*.o"):
        if o.name not in keep:
            o.unlink()
    for c in BUILD.glob("digest*.cpp"):
        if c.with_suffix(".o").name not in keep:
            c.unlink()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--clean", action="store_true")
    a = ap.parse_args(argv)
    if a.clean:
        shutil.rmtree(BUILD, ignore_errors=True)
    build(a.jobs, a.force, a.verbose)


if __name__ == "__main__":
    main(sys.argv[1:])
