"""Profiling driver: one synthetic BAM, one hbam_decode_split (device-resident).  Run under
rocprofv3 --kernel-trace / --pmc to get per-kernel numbers (see profiles/README)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import genbam  # noqa: E402
from hadoop_bam import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=float, default=256e6)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--seed", type=int, default=2)
a = ap.parse_args()
g = genbam.generate(target_bytes=int(a.size), seed=a.seed, threads=16)
data = np.asarray(g)
d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
d[:len(data)].copy_(torch.from_numpy(data))
d[len(data):].zero_()
torch.cuda.synchronize()
ctx = _lib.Context(0)
h = ctx.parse_header(d[:len(data)])
for _ in range(a.reps):
    rc, cols = ctx.decode_split_device(d[:len(data)], h["first_voffset"], (len(data) << 16) | 0xffff,
                                       h["n_ref"])
    assert rc == 0 and cols.status == 0 and cols.n_records == g.n_records
    print({k: round(v, 3) if isinstance(v, float) else v for k, v in ctx.timing().items()}, flush=True)
