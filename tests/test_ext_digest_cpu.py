"""The in-tree extension carries the digest of the sources it was built from,
and the loader refuses / rebuilds a binary whose digest does not match csrc/
(a stale .so would otherwise be tested silently on the GPU box)."""
import pytest

from distributed_compute_pytorch_amd import _build, _ext


def test_built_extension_matches_sources():
    so = _build.ext_path()
    assert so.exists()
    assert _build.embedded_digest(so) == _build.source_digest()
    assert _ext._stale() is None


def test_digest_ignores_checkout_location(monkeypatch):
    # the compile flags embed the checkout's csrc path; the digest masks it out
    monkeypatch.setattr(_build, "_flags", lambda: (["g++", f"-I{_build.CSRC}"], ["hipcc"]))
    here = _build.source_digest()
    monkeypatch.setattr(_build, "_flags", lambda: (["g++", "-I<csrc>"], ["hipcc"]))
    assert _build.source_digest() == here
    monkeypatch.setattr(_build, "_flags", lambda: (["g++", "-I<csrc>", "-O2"], ["hipcc"]))
    assert _build.source_digest() != here


def test_stale_binary_is_detected(monkeypatch):
    monkeypatch.setattr(_build, "source_digest", lambda: "0" * 40)
    why = _ext._stale()
    assert why is not None and "other sources" in why


def test_no_autobuild_refuses_stale(monkeypatch):
    monkeypatch.setattr(_build, "source_digest", lambda: "0" * 40)
    monkeypatch.setattr(_ext, "_C", None)
    monkeypatch.setenv("DCP_NO_AUTOBUILD", "1")
    with pytest.raises(ImportError, match="stale"):
        _ext.load()


def test_digest_read_does_not_map_the_library():
    """embedded_digest reads the file's bytes: the library must not get mapped
    (a dlopen of a stale _C would survive the rebuild in this process)."""
    import subprocess
    import sys

    code = (
        # _build.py on its own: importing the package would load _C itself
        "import importlib.util, sys\n"
        f"spec = importlib.util.spec_from_file_location('dcp_build', {str(_build.__file__)!r})\n"
        "_build = importlib.util.module_from_spec(spec); sys.modules['dcp_build'] = _build\n"
        "spec.loader.exec_module(_build)\n"
        "so = _build.ext_path()\n"
        "d = _build.embedded_digest(so)\n"
        "assert d is not None and len(d) == 40, d\n"
        "maps = open('/proc/self/maps').read()\n"
        "assert so.name not in maps, 'digest read mapped the extension'\n"
        "print('ok')\n"
    )
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       cwd=str(_build.REPO), timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr


def test_rebuild_after_load_refuses_in_place(monkeypatch):
    """A process that has _C mapped cannot swap it for a rebuilt one: load()
    must ask for a restart instead of importing the old mapping again."""
    import sys

    assert "distributed_compute_pytorch_amd._C" in sys.modules  # imported by the package
    monkeypatch.setattr(_build, "source_digest", lambda: "0" * 40)
    monkeypatch.setattr(_ext, "_C", None)
    monkeypatch.delenv("DCP_NO_AUTOBUILD", raising=False)
    monkeypatch.setattr(_build, "build", lambda *a, **k: pytest.fail("must not rebuild in place"))
    with pytest.raises(ImportError, match="restart"):
        _ext.load()
