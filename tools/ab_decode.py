"""A/B timing of the whole split decode (hbam_decode_split on a device-resident shard, the
bench.py step) across library builds: per-stage times of each rep, and a digest of every
output column and pool so the builds can be checked against each other.
usage: ab_decode.py --size 5e9 --libs libhbam.so libhbam_x.so --reps 3"""
import argparse
import ctypes as C
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import genbam  # noqa: E402
from hadoop_bam import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=float, default=5e9)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--seed", type=int, default=2)
ap.add_argument("--libs", nargs="+", default=["libhbam.so"])
ap.add_argument("--digest", type=int, default=1)
ap.add_argument("--addr", type=int, default=1, help="print the output buffers' device addresses")
a = ap.parse_args()
g = genbam.generate(target_bytes=int(a.size), seed=a.seed, threads=16)
data = np.asarray(g)
d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
d[:len(data)].copy_(torch.from_numpy(data))
d[len(data):].zero_()
torch.cuda.synchronize()
print("comp_bytes %d" % len(data), flush=True)
digests = {}
for lib in a.libs:
    _lib._LIB = None
    L = _lib.load(os.path.join(ROOT, "hadoop-bam_amd", lib))
    ctx = _lib.Context(0)
    h = ctx.parse_header(data[:1 << 20])
    v0, v1 = h["first_voffset"], (len(data) << 16) | 0xffff
    for r in range(a.reps):
        rc, cols = ctx.decode_split_device(d[:len(data)], v0, v1, h["n_ref"])
        t = ctx.timing()
        if r == 0 and a.addr:  # where the pools kernel's buffers landed (placement A/B)
            ad = {k: C.cast(getattr(cols, k), C.c_void_p).value or 0
                  for k in ("ubuf", "rec_off", "names", "cigars", "seq", "qual", "aux", "name_off", "seq_off")}
            print("%-18s addr %s" % (lib, " ".join("%s=%x(%%2M=%x)" % (k, v, v % (2 << 20)) for k, v in ad.items())),
                  flush=True)
        print("%-18s rep %d rc %d n %d total %.3f ms  scan %.3f huffman %.3f resolve %.3f walk %.3f "
              "decode %.3f pools %.3f" % (lib, r, rc, cols.n_records, t["total_ms"], t["scan_ms"],
                                          t["huffman_ms"], t["resolve_ms"], t["walk_ms"], t["decode_ms"],
                                          t["pools_ms"]), flush=True)
    if a.digest:
        hc = _lib.Columns()
        assert ctx.L.hbam_columns_to_host(ctx.h, C.byref(cols), C.byref(hc)) == 0, ctx.last_error()
        out = _lib.host_columns_to_numpy(hc)
        ctx.L.hbam_free_host_columns(C.byref(hc))
        dg = {k: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest()[:16]
              for k, v in out.items() if isinstance(v, np.ndarray)}
        digests[lib] = dg
        del out
    ctx.close()
if len(digests) > 1:
    ref = digests[a.libs[0]]
    for lib, dg in digests.items():
        diff = sorted(k for k in ref if dg.get(k) != ref[k])
        print("%-18s columns/pools differing from %s: %s" % (lib, a.libs[0], diff or "none"))
