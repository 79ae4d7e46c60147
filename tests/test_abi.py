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


def test_struct_layouts_match_the_header():
    """hbam_columns / hbam_sorted_run as compiled C (gcc on include/hbam.h) have the sizes and
    field offsets the ctypes binding and the Java shim's COLUMNS layout assume."""
    import tempfile
    from hadoop_bam import _lib
    src = r'''
#include <stddef.h>
#include <stdio.h>
#include "hbam.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(hbam_columns), offsetof(hbam_columns, voffset),
         offsetof(hbam_columns, ubuf_len), offsetof(hbam_columns, aux), sizeof(hbam_sorted_run),
         sizeof(hbam_timing), sizeof(hbam_bcf_header), sizeof(hbam_bcf_columns),
         offsetof(hbam_bcf_columns, data_len), offsetof(hbam_bcf_columns, n_fmt_sample));
  return 0;
}'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "l")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, c], check=True)
        got = [int(x) for x in subprocess.run([exe], stdout=subprocess.PIPE, text=True).stdout.split()]
    assert got[0] == C.sizeof(_lib.Columns) == 240
    assert got[1] == _lib.Columns.voffset.offset and got[2] == _lib.Columns.ubuf_len.offset
    assert got[3] == _lib.Columns.aux.offset
    assert got[4] == C.sizeof(_lib.SortedRunC) and got[5] == C.sizeof(_lib.Timing)
    assert got[6] == C.sizeof(_lib.BcfHeaderC) == 32 and got[7] == C.sizeof(_lib.BcfColumnsC)
    assert got[8] == _lib.BcfColumnsC.data_len.offset and got[9] == _lib.BcfColumnsC.n_fmt_sample.offset
    # the Java shim: 4 header fields, then 27 pointer-sized slots in the header's order
    java = open(os.path.join(ROOT, "java", "src", "main", "java", "org", "seqdoop", "hadoop_bam",
                             "hip", "Hbam.java")).read()

    def layout(name):
        body = java[java.index("StructLayout %s = MemoryLayout.structLayout(" % name):]
        return re.findall(r'withName\("(\w+)"\)', body[:body.index(");")])
    names = layout("COLUMNS")
    assert names == [f[0] for f in _lib.Columns._fields_]
    assert len(names) - 4 == 27
    assert layout("BCF_COLUMNS") == [f[0] for f in _lib.BcfColumnsC._fields_]
    assert layout("BCF_HEADER") == [f[0] for f in _lib.BcfHeaderC._fields_]


_C2J = {"void": None}


def _ctype_letter(t):
    t = t.strip()
    if "*" in t:
        return "A"
    t = t.replace("const", "").strip()
    if t == "hbam_read_fn":  # a function pointer (the Java shim's upcall stub)
        return "A"
    if t in ("int", "int32_t", "uint32_t"):
        return "I"
    if t in ("int64_t", "uint64_t", "size_t"):
        return "J"
    if t == "void":
        return None
    raise AssertionError("unmapped C type %r" % t)


def _prototypes():
    txt = open(os.path.join(ROOT, "include", "hbam.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w ]*?\**)\s*\b(hbam_\w+)\s*\(([^)]*)\)\s*;", txt):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ps = [p for p in (x.strip() for x in params.split(",")) if p and p != "void"]
        # a parameter's type: everything but its name
        types = [re.sub(r"\b\w+$", "", p) if not p.endswith("*") else p for p in ps]
        out[name] = (_ctype_letter(ret), [_ctype_letter(t) for t in types])
    return out


def test_java_downcalls_match_the_header():
    """Every downcall the Java shim binds (Hbam.java fn(name, FunctionDescriptor...)) has the
    header's return type and parameter list (A = pointer, I = 32-bit, J = 64-bit)."""
    protos = _prototypes()
    java = open(os.path.join(ROOT, "java", "src", "main", "java", "org", "seqdoop", "hadoop_bam",
                             "hip", "Hbam.java")).read()
    binds = re.findall(r'fn\("(hbam_\w+)",\s*FunctionDescriptor\.(of|ofVoid)\(([^)]*)\)\)', java)
    assert len(binds) >= 20
    for name, kind, args in binds:
        assert name in protos, name
        letters = [a.strip() for a in args.split(",") if a.strip()]
        ret = None if kind == "ofVoid" else letters.pop(0)
        assert (ret, letters) == protos[name], (name, (ret, letters), protos[name])
