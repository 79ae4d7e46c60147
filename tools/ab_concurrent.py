"""Measurement only (not the product path): does decoding a shard as K FileVirtualSplits on K
contexts (K HIP streams, one host thread each) beat one context decoding the whole shard?  The
Huffman pass holds all of a CU's LDS and registers, so overlap can only come from one split's
later stages (record walk, fixed fields, pools: HBM-bound) running beside another split's inflate.
Both forms decode the same records (the splits are addProbabilisticSplits' of K equal byte
ranges); the record counts are compared.
usage: ab_concurrent.py --size 5e9 --k 2 --reps 3"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import genbam  # noqa: E402
from hadoop_bam import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=float, default=5e9)
ap.add_argument("--k", type=int, default=2)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
data = np.asarray(genbam.generate(target_bytes=int(a.size), seed=2, threads=16))
d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
d[:len(data)].copy_(torch.from_numpy(data))
d[len(data):].zero_()
torch.cuda.synchronize()
whole = _lib.Context(0)
h = whole.parse_header(data[:1 << 20])
n_ref = h["n_ref"]
v_all = (h["first_voffset"], (len(data) << 16) | 0xffff)
b = np.array([len(data) * i // a.k for i in range(a.k)], np.uint64)
e = np.array([len(data) * (i + 1) // a.k for i in range(a.k)], np.uint64)
n, vs, ve = whole.probabilistic_splits(d[:len(data)], b, e)
ctxs = [_lib.Context(0) for _ in range(a.k)]
print("comp_bytes %d splits %s" % (len(data), list(zip([int(x) for x in vs], [int(x) for x in ve]))), flush=True)


def one():
    torch.cuda.synchronize()
    t = time.time()
    rc, cols = whole.decode_split_device(d[:len(data)], v_all[0], v_all[1], n_ref)
    torch.cuda.synchronize()
    assert rc == 0 and cols.status == 0
    return time.time() - t, int(cols.n_records)


def many():
    res = [None] * a.k

    def run(i):
        rc, cols = ctxs[i].decode_split_device(d[:len(data)], int(vs[i]), int(ve[i]), n_ref)
        assert rc == 0 and cols.status == 0
        res[i] = int(cols.n_records)
    torch.cuda.synchronize()
    t = time.time()
    th = [threading.Thread(target=run, args=(i,)) for i in range(a.k)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    return time.time() - t, sum(res)


one()
many()
for r in range(a.reps):
    t1, n1 = one()
    tk, nk = many()
    print("rep %d  one context %.2f ms (%d records)   %d contexts concurrently %.2f ms (%d records)"
          % (r, t1 * 1e3, n1, a.k, tk * 1e3, nk), flush=True)
