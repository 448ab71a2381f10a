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
