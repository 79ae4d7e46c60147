"""Config #3 measurement: BAMSplitGuesser.guessNextBAMRecordStart (BAMSplitGuesser.java:109-212)
at K random split offsets over a synthetic BAM resident in HBM, all guesses in one batched
device call (hbam_guess_batch).  Each guess gets the window Hadoop's split sizing gives it:
[off, off + split) with split = 128 MiB (BAMInputFormat feeds the next split's start).
A seeded sample of the guesses is checked against the CPU oracle.  Prints one JSON line.

The file is --size compressed bytes (default 10 GB: one box call cannot print while the
generator runs, so 50 GB is not generated here); a guess reads at most two 64 KiB windows plus
the blocks it inflates, so its cost does not depend on the file size."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=10e9)
    ap.add_argument("--guesses", type=int, default=10000)
    ap.add_argument("--check", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    import genbam
    import oracle
    from hadoop_bam import _lib
    t = time.time()
    g = genbam.generate(target_bytes=int(a.size), seed=3, threads=int(os.environ.get("OMP_NUM_THREADS", 16)))
    data = np.asarray(g)
    print("generated %.2f GB in %.1fs" % (len(data) / 1e9, time.time() - t), file=sys.stderr, flush=True)
    d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
    d[:len(data)].copy_(torch.from_numpy(data))
    d[len(data):].zero_()
    torch.cuda.synchronize()
    ctx = _lib.Context(0)
    h = ctx.parse_header(d[:len(data)])
    rng = np.random.default_rng(3)  # config #3 offsets
    beg = np.sort(rng.integers(0, len(data) - 1, a.guesses)).astype(np.int64)
    end = np.minimum(beg + (128 << 20), len(data)).astype(np.int64)
    t = time.time()
    rc, out, err = ctx.guess_batch(d[:len(data)], beg, end, h["n_ref"])  # warmup
    assert rc == 0, ctx.last_error()
    print("warmup %.3fs" % (time.time() - t), file=sys.stderr, flush=True)
    times = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t = time.time()
        rc, out, err = ctx.guess_batch(d[:len(data)], beg, end, h["n_ref"])
        torch.cuda.synchronize()
        times.append(time.time() - t)
        assert rc == 0, ctx.last_error()
        print("rep %.3fs" % times[-1], file=sys.stderr, flush=True)
    idx = rng.choice(a.guesses, min(a.check, a.guesses), replace=False)
    t = time.time()
    want = oracle.guess_bam_record_start(data, int(beg[idx[0]]), int(end[idx[0]]), h["n_ref"])
    cpu_s = time.time() - t  # one host core, one guess
    import threading
    res = {}

    def chk(ii):
        for i in ii:
            res[int(i)] = tuple(map(int, oracle.guess_bam_record_start(data, int(beg[i]), int(end[i]),
                                                                        h["n_ref"])))
    nt = int(os.environ.get("OMP_NUM_THREADS", 16))
    ths = [threading.Thread(target=chk, args=(idx[j::nt],)) for j in range(nt)]
    t = time.time()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    cpu_s = (time.time() - t) * nt / len(idx)
    bad = sum((int(out[i]), int(err[i])) != res[int(i)] for i in idx)
    best = min(times)
    print(json.dumps({
        "metric": "BAMSplitGuesser guesses/s (config#3, one MI355X)",
        "value": round(a.guesses / best, 1), "unit": "guesses/s", "guesses": a.guesses,
        "seconds": round(best, 4), "all_reps_s": [round(x, 4) for x in times],
        "file_bytes": len(data), "window": "[off, off+128 MiB)",
        "parity_sample": int(len(idx)), "parity_mismatches": int(bad),
        "cpu_oracle_s_per_guess": round(cpu_s, 5),
        "cpu_oracle_guesses_per_s_1core": round(1.0 / cpu_s, 1)}), flush=True)
    if bad:
        sys.exit(1)


if __name__ == "__main__":
    main()
