"""Whole-file inflate check with CRC32 on the device: every BGZF block of several generated BAMs
(seeds, quality models, compression levels) is inflated by the batched two-phase inflate and its
output checked against the block's CRC32 footer (hbam_inflate with check_crc = 1).  A wrong byte
anywhere shows up as a CRC mismatch.  Prints one line per file; exit status 1 on any bad block."""
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
ap.add_argument("--size", type=float, default=1e9)
a = ap.parse_args()
torch.cuda.init()
ctx = _lib.Context(0)
cases = [dict(seed=s) for s in (3, 4, 5, 6)] + [dict(seed=7, uniform_qual=1), dict(seed=8, level=1),
                                                  dict(seed=9, level=9), dict(seed=10, level=6, uniform_qual=1)]
bad_total = 0
for kw in cases:
    data = np.asarray(genbam.generate(target_bytes=int(a.size), threads=16, **kw))
    d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
    d[:len(data)].copy_(torch.from_numpy(data))
    d[len(data):].zero_()
    torch.cuda.synchronize()
    rc, blocks = ctx.scan_blocks(d[:len(data)])
    assert rc == 0, rc
    n = len(blocks["coff"])
    arr = (_lib.Block * n)()
    for i in range(n):
        arr[i].coff = int(blocks["coff"][i]); arr[i].clen = int(blocks["clen"][i])
        arr[i].isize = int(blocks["isize"][i]); arr[i].crc = int(blocks["crc"][i])
    off = np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.int32)
    rc = ctx.L.hbam_inflate(ctx.h, C.c_void_p(d.data_ptr()), 1, len(data), arr, n, 1, None, 0,
                            off.ctypes.data, st.ctypes.data)
    bad = int(np.sum(st != 0))
    bad_total += bad
    print("case %-40s blocks %7d U %.3f GB rc %d crc/status mismatches %d"
          % (kw, n, off[-1] / 1e9, rc, bad), flush=True)
sys.exit(1 if bad_total else 0)
