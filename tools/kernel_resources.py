"""Per-kernel resources of one HIP source (device-only gfx950 build on the CPU):
VGPR / AGPR / SGPR counts, scratch (private segment) bytes, static LDS.

    python tools/kernel_resources.py csrc/kernels/gemm.hip [NAME_REGEX]
"""
import os
import re
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    src = sys.argv[1]  # a .hip source, or an already built device code object (.co)
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    with tempfile.TemporaryDirectory() as d:
        co = src if src.endswith(".co") else os.path.join(d, "k.co")
        if co != src:
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--offload-device-only", "--no-gpu-bundle-output", "-O3", "-std=c++17",
                        "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form", f"-I{R}/csrc", "-I/opt/rocm/include", src, "-o", co],
                           check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                               check=True).stdout
    for blk in re.split(r"\n  - \.agpr_count:", notes)[1:]:
        def g(k):
            m = re.search(r"\." + k + r":\s+(\S+)", blk)
            return m.group(1) if m else "?"
        agpr = blk.split("\n", 1)[0].strip()
        name = g("name")
        if not pat.search(name):
            continue
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        print(f"vgpr={g('vgpr_count'):>4} agpr={agpr:>4} sgpr={g('sgpr_count'):>4} "
              f"scratch={g('private_segment_fixed_size'):>5} lds={g('group_segment_fixed_size'):>6}  {dem[:160]}")


if __name__ == "__main__":
    main()
