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
ap.add_argument("--prof", action="store_true",
                help="use libhbam_prof.so (built with -DHBAM_PROF) and print per-block cycle stats")
ap.add_argument("--prof-lib", default="libhbam_prof.so", help="--prof: the profiling build to load")
a = ap.parse_args()
if a.prof:
    os.environ["HBAM_LIB"] = os.path.join(ROOT, "hadoop-bam_amd", a.prof_lib)
    os.environ["HBAM_INFLATE_SLICES"] = "1"  # per-block prof slots are indexed per launch
    os.environ["HBAM_WAVE_MAX_BLOCKS"] = "0"  # the stamps are in the lane-per-block Huffman pass
g = genbam.generate(target_bytes=int(a.size), seed=a.seed, threads=16)
data = np.asarray(g)
d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
d[:len(data)].copy_(torch.from_numpy(data))
d[len(data):].zero_()
torch.cuda.synchronize()
ctx = _lib.Context(0)
if a.prof:
    import ctypes as C
    L = _lib.load()
    L.hbam_prof_attach.argtypes = [C.c_void_p]
    pbuf = torch.zeros((len(data) // 8000 + 4096) * 32, dtype=torch.int64, device="cuda")
    assert L.hbam_prof_attach(C.c_void_p(pbuf.data_ptr())) == 0
h = ctx.parse_header(d[:len(data)])
for _ in range(a.reps):
    rc, cols = ctx.decode_split_device(d[:len(data)], h["first_voffset"], (len(data) << 16) | 0xffff,
                                       h["n_ref"])
    if not (rc == 0 and cols.status == 0 and cols.n_records == g.n_records):
        raise SystemExit("decode failed: rc %d status %d records %d of %d: %s" % (
            rc, cols.status, cols.n_records, g.n_records, ctx.last_error()))
    print({k: round(v, 3) if isinstance(v, float) else v for k, v in ctx.timing().items()}, flush=True)

if a.prof:
    nb = ctx.timing()["n_blocks"]
    P = pbuf.view(-1, 32)[:nb].cpu().numpy().astype(np.float64)

    def stats(name, col):
        v = P[:, col]
        print("  %-10s mean %10.0f  p50 %10.0f  p99 %10.0f  max %10.0f" %
              (name, v.mean(), np.percentile(v, 50), np.percentile(v, 99), v.max()))

    for lab, s0, s1, cyc in (("tokens", 8, 9, 10), ("resolve", 0, 1, 2)):
        st, en = P[:, s0], P[:, s1]
        ok = en > 0
        span = (en[ok].max() - st[ok].min()) / 100.0  # s_memrealtime = 100 MHz -> us
        busy = ((en - st)[ok]).sum() / 100.0
        print("%s: span %.1f us, sum of block durations %.1f us, mean concurrency %.1f blocks"
              % (lab, span, busy, busy / max(span, 1e-9)))
        stats("cycles", cyc)
        stats("dur_us", None) if False else None
        d = (en - st)[ok] / 100.0
        print("  dur_us     mean %10.2f  p50 %10.2f  p99 %10.2f  max %10.2f"
              % (d.mean(), np.percentile(d, 50), np.percentile(d, 99), d.max()))
    for nm, c in (("stage", 3), ("desc", 4), ("batches", 5), ("  of which pre", 12), ("writeback", 13),
                  ("n_batch", 6), ("n_match", 7)):
        stats(nm, c)
    print("  cycles/batch %.1f, matches/batch %.2f" % (P[:, 5].sum() / max(P[:, 6].sum(), 1),
                                                     P[:, 7].sum() / max(P[:, 6].sum(), 1)))
    stats("tok_out", 11)
