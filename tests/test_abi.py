"""The C-ABI library builds for gfx950, loads, and exports every entry point include/hbam.h
declares (no compute calls: this runs without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT


def _declared():
    txt = open(os.path.join(ROOT, "include", "hbam.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"\b(hbam_[a-z_0-9]+)\s*\(", txt))
    return sorted(names)


def test_header_declares_expected_entry_points():
    from hadoop_bam import _lib
    assert set(_declared()) == set(_lib.EXPORTS)


def test_library_exports_every_symbol():
    from hadoop_bam import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__  # noqa: F401
        __import__("__graft_entry__").build()
    L = C.CDLL(_lib.LIB_PATH)
    for name in _declared():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], stdout=subprocess.PIPE,
                         text=True).stdout
    exported = set(re.findall(r" T (hbam_\w+)", out))
    assert set(_declared()) <= exported


def test_library_contains_gfx950_code_object():
    from hadoop_bam import _lib
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list",
                          "--type=o", "--input=" + _lib.LIB_PATH],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True).stdout
    if "gfx950" not in out:
        # fall back to scanning the embedded fat binary
        data = open(_lib.LIB_PATH, "rb").read()
        assert b"gfx950" in data


def test_no_device_context_without_gpu():
    """Without a GPU the product path fails loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from hadoop_bam import _lib
    with pytest.raises(_lib.HbamUnavailable):
        _lib.Context(0)
