"""ctypes wrapper of the synthetic BAM generator (tools/gen_bam.cpp -> libhbamgen.so).

Test/bench tooling: deterministic seeded 150 bp paired-end BAMs.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class Params(C.Structure):
    _fields_ = [("n_records", C.c_uint64), ("target_bytes", C.c_uint64), ("seed", C.c_uint64),
                ("sorted", C.c_int32), ("qual_model", C.c_int32), ("block_payload", C.c_int32),
                ("straddle", C.c_int32), ("level", C.c_int32), ("threads", C.c_int32),
                ("segment_records", C.c_int32), ("empty_block_every", C.c_int32),
                ("long_read_every", C.c_int32), ("odd_every", C.c_int32),
                ("unplaced_permille", C.c_int32), ("mate_unmapped_permille", C.c_int32),
                ("write_terminator", C.c_int32), ("n_ref", C.c_int32)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libhbamgen.so")
        src = os.path.join(_HERE, "gen_bam.cpp")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", path, src,
                            "-lz", "-lpthread"], check=True)
        L = C.CDLL(path)
        L.hbamgen_default_params.argtypes = [C.POINTER(Params)]
        L.hbamgen_generate_mem.argtypes = [C.POINTER(Params), C.POINTER(C.POINTER(C.c_uint8)),
                                           C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.hbamgen_generate_mem.restype = C.c_int
        L.hbamgen_generate_file.argtypes = [C.POINTER(Params), C.c_char_p,
                                            C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.hbamgen_free.argtypes = [C.POINTER(C.c_uint8)]
        L.hbamgen_generate_range.argtypes = [C.POINTER(Params), C.c_uint64, C.c_uint64, C.c_uint64,
                                             C.c_int32, C.POINTER(C.POINTER(C.c_uint8)),
                                             C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.hbamgen_generate_range.restype = C.c_int
        _LIB = L
    return _LIB


def params(**kw):
    p = Params()
    lib().hbamgen_default_params(C.byref(p))
    names = {
        "records": "n_records", "target_bytes": "target_bytes", "seed": "seed",
        "sorted": "sorted", "uniform_qual": "qual_model", "payload": "block_payload",
        "straddle": "straddle", "level": "level", "threads": "threads",
        "segment": "segment_records", "empty_every": "empty_block_every",
        "long_every": "long_read_every", "odd_every": "odd_every",
        "unplaced_permille": "unplaced_permille", "mate_unmapped_permille": "mate_unmapped_permille",
        "terminator": "write_terminator", "n_ref": "n_ref",
    }
    for k, v in kw.items():
        setattr(p, names[k], int(v))
    if "target_bytes" in kw and "records" not in kw:
        p.n_records = 0
    return p


def generate(**kw):
    """Return the BAM file bytes as a numpy uint8 array (and record count via .n_records)."""
    p = params(**kw)
    out = C.POINTER(C.c_uint8)()
    n = C.c_uint64(0)
    nrec = C.c_uint64(0)
    rc = lib().hbamgen_generate_mem(C.byref(p), C.byref(out), C.byref(n), C.byref(nrec))
    if rc:
        raise MemoryError("hbamgen_generate_mem failed")
    a = np.ctypeslib.as_array(out, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint8)
    lib().hbamgen_free(out)
    return GenBam(a, nrec.value)


def generate_file(path, **kw):
    p = params(**kw)
    n = C.c_uint64(0)
    nrec = C.c_uint64(0)
    rc = lib().hbamgen_generate_file(C.byref(p), path.encode(), C.byref(n), C.byref(nrec))
    if rc:
        raise OSError("hbamgen_generate_file failed")
    return n.value, nrec.value


class GenBam(np.ndarray):
    """uint8 array with the generated record count attached."""

    def __new__(cls, a, n_records):
        obj = np.asarray(a).view(cls)
        obj.n_records = n_records
        return obj

    def __array_finalize__(self, obj):
        self.n_records = getattr(obj, "n_records", 0)


def generate_range(n_seg_total, seg_first, seg_count, header=False, tail=False, **kw):
    """Bytes of segments [seg_first, seg_first+seg_count) of ONE file of n_seg_total main
    segments (+ the header blocks / the unplaced tail and terminator): consecutive ranges
    concatenate to that file, so ranks can each hold their byte range of it."""
    p = params(**kw)
    out = C.POINTER(C.c_uint8)()
    n = C.c_uint64(0)
    nrec = C.c_uint64(0)
    rc = lib().hbamgen_generate_range(C.byref(p), n_seg_total, seg_first, seg_count,
                                      (1 if header else 0) | (2 if tail else 0), C.byref(out),
                                      C.byref(n), C.byref(nrec))
    if rc:
        raise ValueError("hbamgen_generate_range failed (empty_every must be 0)")
    a = np.ctypeslib.as_array(out, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint8)
    lib().hbamgen_free(out)
    return GenBam(a, nrec.value)
