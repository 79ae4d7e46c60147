"""Time the device guesser on a few guesses (diagnostic)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import oracle
from hadoop_bam import _lib
data = np.fromfile(os.path.join(ROOT, "tests", "golden", "small_pe.bam"), dtype=np.uint8)
h = oracle.read_header(data)
ctx = _lib.Context(0)
rng = np.random.default_rng(3)
for k in (1, 4, 16, 64):
    beg = np.sort(rng.integers(0, len(data), k)).astype(np.int64)
    end = np.minimum(beg + 300000, len(data)).astype(np.int64)
    t = time.time()
    rc, out, err = ctx.guess_batch(data, beg, end, h["n_ref"])
    dt = time.time() - t
    ok = all((int(out[i]), int(err[i])) == oracle.guess_bam_record_start(data, int(beg[i]), int(end[i]), h["n_ref"]) for i in range(k))
    print("k=%d rc=%d %.3fs parity=%s" % (k, rc, dt, ok), flush=True)
