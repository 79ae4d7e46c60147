"""Diagnose a guess that differs from the oracle: the window fixture's guess on the device
(profiling build: per-candidate trace of guess 0), the oracle's, and the device inflate of
every block of the window against zlib."""
import ctypes as C
import os
import struct
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
os.environ["HBAM_LIB"] = os.path.join(ROOT, "hadoop-bam_amd", "libhbam_prof.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from hadoop_bam import _lib  # noqa: E402

ctx = _lib.Context(0)
L = _lib.load()
L.hbam_prof_attach_trace.argtypes = [C.c_void_p, C.c_uint]


def show_trace(tr):
    t = tr.cpu().numpy().astype(np.uint64)
    k = int(t[0])
    for j in range(min(k, 12)):
        a, b = int(t[1 + 2 * j]), int(t[2 + 2 * j])
        print("   cand cp0 %d up0 %d rc %d b %d any %d memo %d" % (a >> 32, a & 0xffffffff,
              C.c_int32(b >> 32).value, (b >> 8) & 0xff, b & 1, (b >> 1) & 1))
    if k > 12:
        print("   ... %d candidates" % k)
    q = t[8193:]
    for j in range(min(int(q[0]), 40)):
        pos, ci, sc, cp = (int(x) for x in q[1 + 4 * j:5 + 4 * j])
        print("   cache pos %d clen %d isize %d st %d crc %08x want %08x pad %d" % (
            pos, ci >> 32, ci & 0xffffffff, C.c_int32(sc >> 32).value, sc & 0xffffffff, cp >> 32, cp & 1))


if len(sys.argv) > 1 and sys.argv[1] == "--batch":
    # the config #3 batch (tools/bench_guess.py) with guess(es) sys.argv[2:] traced
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import genbam
    g = genbam.generate(target_bytes=int(10e9), seed=3, threads=int(os.environ.get("OMP_NUM_THREADS", 16)))
    data = np.asarray(g)
    n = len(data)
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    d[:n].copy_(torch.from_numpy(data))
    d[n:].zero_()
    h = ctx.parse_header(d[:n])
    rng = np.random.default_rng(3)
    beg = np.sort(rng.integers(0, n - 1, 10000)).astype(np.int64)
    end = np.minimum(beg + (128 << 20), n).astype(np.int64)
    for idx in (int(x) for x in sys.argv[2:]):
        want = oracle.guess_bam_record_start(data, int(beg[idx]), int(end[idx]), h["n_ref"])
        for lo, hi in ((0, 10000), (idx, idx + 1)):
            tr = torch.zeros(1 + 2 * 4096 + 1 + 4 * 512, dtype=torch.int64, device="cuda")
            assert L.hbam_prof_attach_trace(C.c_void_p(tr.data_ptr()), idx - lo) == 0
            rc, out, err = ctx.guess_batch(d[:n], beg[lo:hi], end[lo:hi], h["n_ref"])
            L.hbam_prof_attach_trace(C.c_void_p(0), 0)
            o = int(out[idx - lo])
            print("guess %d beg %d batch [%d,%d): device %d %d err %d | oracle %d %d %d" % (
                idx, beg[idx], lo, hi, (o >> 16) - beg[idx], o & 0xffff, int(err[idx - lo]),
                (want[0] >> 16) - beg[idx], want[0] & 0xffff, want[1]), flush=True)
            show_trace(tr)
    sys.exit(0)

for name in sys.argv[1:]:
    w = np.fromfile(os.path.join(ROOT, "tests", "golden", name), np.uint8)
    n_ref = 25
    want = oracle.guess_bam_record_start(w, 0, len(w), n_ref)
    tr = torch.zeros(1 + 2 * 4096 + 1 + 4 * 512, dtype=torch.int64, device="cuda")
    assert L.hbam_prof_attach_trace(C.c_void_p(tr.data_ptr()), 0) == 0
    rc, out, err = ctx.guess_batch(w, np.array([0], np.int64), np.array([len(w)], np.int64), n_ref)
    L.hbam_prof_attach_trace(C.c_void_p(0), 0)
    print(name, "device", int(out[0]) >> 16, int(out[0]) & 0xffff, int(err[0]),
          "oracle", want[0] >> 16, want[0] & 0xffff, want[1], flush=True)
    show_trace(tr)
    # blocks of the window from the first magic on: device inflate vs zlib
    bw = w.tobytes()
    p = bw.find(b"\x1f\x8b\x08\x04")
    co, cl, isz, crc = [], [], [], []
    while p + 18 <= len(bw) and bw[p:p + 4] == b"\x1f\x8b\x08\x04":
        bs = struct.unpack("<H", bw[p + 16:p + 18])[0] + 1
        if p + bs > len(bw):
            break
        c_, i_ = struct.unpack("<II", bw[p + bs - 8:p + bs])
        co.append(p); cl.append(bs); isz.append(i_); crc.append(c_)
        p += bs
    blocks = {"coff": np.array(co, np.uint64), "clen": np.array(cl, np.uint32),
              "isize": np.array(isz, np.uint32), "crc": np.array(crc, np.uint32)}
    rc, u, off, st = ctx.inflate(w, blocks, check_crc=True)
    for j in range(len(co)):
        ref = zlib.decompressobj(-15).decompress(bw[co[j] + 18:co[j] + cl[j] - 8])
        got = u[int(off[j]):int(off[j + 1])].tobytes()
        print("   block %d isize %d st %d same %s" % (co[j], isz[j], int(st[j]), got == ref))
