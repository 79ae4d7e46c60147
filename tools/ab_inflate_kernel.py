"""A/B timing of the batched inflate kernels alone (hbam_inflate on a device-resident file,
no output download, no parity check): prints the Huffman / LZ77 phase times of each rep.
Used with variant libraries (HBAM_LIB=...) built with -D switches; see tools/ab_libs.sh."""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import genbam  # noqa: E402
from hadoop_bam import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=float, default=2e9)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--seed", type=int, default=2)
ap.add_argument("--libs", nargs="+", default=["libhbam.so"])
ap.add_argument("--orders", nargs="+", default=["file"],
                help="block order handed to hbam_inflate: file, clen (descending), shuffle")
ap.add_argument("--slices", nargs="+", type=int, default=[0], help="HBAM_INFLATE_SLICES values (0: library default)")
a = ap.parse_args()
g = genbam.generate(target_bytes=int(a.size), seed=a.seed, threads=16)
data = np.asarray(g)
d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
d[:len(data)].copy_(torch.from_numpy(data))
d[len(data):].zero_()
torch.cuda.synchronize()
for lib, sl, order in [(x, y, z) for x in a.libs for y in a.slices for z in a.orders]:
    if sl:
        os.environ["HBAM_INFLATE_SLICES"] = str(sl)
    else:
        os.environ.pop("HBAM_INFLATE_SLICES", None)
    _lib._LIB = None
    L = _lib.load(os.path.join(ROOT, "hadoop-bam_amd", lib))
    ctx = _lib.Context(0)
    rc, blocks = ctx.scan_blocks(d[:len(data)])
    assert rc == 0, rc
    n = len(blocks["coff"])
    perm = np.arange(n)
    if order == "clen":
        perm = np.argsort(-blocks["clen"].astype(np.int64), kind="stable")
    elif order == "shuffle":
        perm = np.random.default_rng(1).permutation(n)
    blocks = {k: v[perm] for k, v in blocks.items()}
    arr = (_lib.Block * n)()
    for i in range(n):
        arr[i].coff = int(blocks["coff"][i]); arr[i].clen = int(blocks["clen"][i])
        arr[i].isize = int(blocks["isize"][i]); arr[i].crc = int(blocks["crc"][i])
    off = np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.int32)
    for r in range(a.reps):
        rc = L.hbam_inflate(ctx.h, C.c_void_p(d.data_ptr()), 1, len(data), arr, n, 0, None, 0,
                            off.ctypes.data, st.ctypes.data)
        t = ctx.timing()
        print("%-18s order %-7s slices %d rep %d rc %d blocks %d U %.3f GB huffman %.3f ms resolve %.3f ms bad %d"
              % (lib, order, sl, r, rc, n, off[-1] / 1e9, t["huffman_ms"], t["resolve_ms"], int(np.sum(st != 0))),
              flush=True)
    ctx.close()
