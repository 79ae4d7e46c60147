"""Build-dependence check of the Huffman pass: inflate one generated BAM with several library
builds (CRC32 checked on the device) and, for the profiling builds (HBAM_PROF), record the
decoder's exit state of the first bad blocks (output position, stream bits consumed, bit-buffer
state, iteration count) and save those blocks' compressed bytes, so the failing symbol can be
located on the CPU (tools/diag_inflate_cpu.py).

usage: diag_inflate_build.py --size 5e8 --libs libhbam.so libhbam_pp.so ... --out gpurun_out/diag
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import genbam  # noqa: E402
from hadoop_bam import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=float, default=5e8)
ap.add_argument("--seed", type=int, default=3)
ap.add_argument("--libs", nargs="+", default=["libhbam.so"])
ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "diag"))
ap.add_argument("--keep", type=int, default=6, help="bad blocks saved per library")
ap.add_argument("--variants", nargs="+", default=["att:0"],
                help="att|noatt:FIRST - attach the profile buffer or not; inflate blocks FIRST.. only")
a = ap.parse_args()
os.makedirs(a.out, exist_ok=True)
torch.cuda.init()
data = np.asarray(genbam.generate(target_bytes=int(a.size), seed=a.seed, threads=16))
d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
d[:len(data)].copy_(torch.from_numpy(data))
d[len(data):].zero_()
torch.cuda.synchronize()
summary = {}
for lib, var in [(x, v) for x in a.libs for v in a.variants]:
    attach, first = var.split(":")[0] == "att", int(var.split(":")[1])
    _lib._LIB = None
    L = _lib.load(os.path.join(ROOT, "hadoop-bam_amd", lib))
    ctx = _lib.Context(0)
    rc, blocks = ctx.scan_blocks(d[:len(data)])
    assert rc == 0, rc
    blocks = {k: v[first:] for k, v in blocks.items()}
    n = len(blocks["coff"])
    prof = None
    if attach and hasattr(L, "hbam_prof_attach"):
        prof = torch.zeros(32 * n, dtype=torch.int64, device="cuda")
        L.hbam_prof_attach.argtypes = [C.c_void_p]
        assert L.hbam_prof_attach(C.c_void_p(prof.data_ptr())) == 0
    arr = (_lib.Block * n)()
    for i in range(n):
        arr[i].coff = int(blocks["coff"][i]); arr[i].clen = int(blocks["clen"][i])
        arr[i].isize = int(blocks["isize"][i]); arr[i].crc = int(blocks["crc"][i])
    off = np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.int32)
    rc = L.hbam_inflate(ctx.h, C.c_void_p(d.data_ptr()), 1, len(data), arr, n, 1, None, 0,
                        off.ctypes.data, st.ctypes.data)
    torch.cuda.synchronize()
    bad = np.nonzero(st != 0)[0]
    rec = {"variant": var, "first_block": first, "rc": int(rc), "blocks": n, "bad": int(len(bad)), "status_hist": {}, "first": []}
    for s in np.unique(st[bad]):
        rec["status_hist"][int(s)] = int(np.sum(st[bad] == s))
    if prof is not None:
        P = prof.view(n, 32).cpu().numpy()
        if hasattr(L, "hbam_prof_attach"):
            L.hbam_prof_attach(C.c_void_p(0))
    for b in bad[:a.keep]:
        b = int(b)
        e = {"block": b + first, "launch_index": b, "status": int(st[b]), "coff": int(blocks["coff"][b]), "clen": int(blocks["clen"][b]),
             "isize": int(blocks["isize"][b])}
        if prof is not None:
            e.update(produced=int(P[b, 11]), iters=int(P[b, 24]), consumed=int(P[b, 25]),
                     bc=int(P[b, 26]) & 0xff, nv=(int(P[b, 26]) >> 8) & 0xff, rd=(int(P[b, 26]) >> 16) & 0xff,
                     it=int(P[b, 27]))
        c0 = int(blocks["coff"][b])
        raw = bytes(data[c0:c0 + int(blocks["clen"][b])])
        with open(os.path.join(a.out, "%s_blk%d.bgzf" % (lib, b + first)), "wb") as f:
            f.write(raw)
        rec["first"].append(e)
    summary[lib + " " + var] = rec
    print(lib, var, json.dumps(rec), flush=True)
    ctx.close()
with open(os.path.join(a.out, "summary.json"), "w") as f:
    json.dump(summary, f, indent=1)
