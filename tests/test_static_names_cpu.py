"""Static check: no undefined names anywhere in the package, tools, tests or
examples (tools/check_names.py). GPU-only branches are never executed by the
CPU suite, so a leftover call to a removed helper would otherwise surface only
on the GPU box."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_undefined_names():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_names.py")], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
