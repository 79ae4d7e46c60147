"""Config #3 measurement: BAMSplitGuesser.guessNextBAMRecordStart (BAMSplitGuesser.java:109-212)
at K random split offsets (numpy default_rng(3), uniform in [0, C)) over a synthetic BAM of
--size compressed bytes (config #3: 50 GB), all guesses in one device call.  Each guess gets the
window Hadoop's split sizing gives it: [off, off + 128 MiB) (BAMInputFormat feeds the next
split's start), and reads at most 262,139 bytes of it (:114-125).

Default mode (windowed, what a getSplits client does): the file is generated in chunks of
segments (tools/gen_bam.cpp, seed 3) on the host, each guess's window is cut out of the chunks,
and only the windows go to the device (hbam_guess_windows) — the file is never staged.
--resident: the whole file in HBM and hbam_guess_batch (config #3 as r01/r02 measured it).

A seeded sample of the guesses is checked against the CPU oracle run on the same windows (the
guesser reads nothing else; the oracle's window-relative answer is rebased).  One JSON line."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402

MAX_BYTES_READ = 3 * 0xffff + 0xfffe


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_chunks(size, threads, chunk_bytes):
    """The seed-3 file as consecutive chunks of whole generator segments (concatenating to ONE file)."""
    import genbam
    probe = genbam.generate_range(1, 0, 1, seed=3, threads=threads)
    m = max(1, int(round(size / len(probe))))
    per = max(1, int(round(chunk_bytes / len(probe))))
    chunks, nrec = [], 0
    t = time.time()
    for s0 in range(0, m, per):
        c = genbam.generate_range(m, s0, min(per, m - s0), header=(s0 == 0), tail=(s0 + per >= m),
                                  seed=3, threads=threads)
        nrec += int(c.n_records)
        chunks.append(np.asarray(c))
        log("generated segments %d..%d of %d (%.2f GB so far, %.0fs)"
            % (s0, min(s0 + per, m), m, sum(len(x) for x in chunks) / 1e9, time.time() - t))
    return chunks, nrec


def cut(chunks, starts, off, n):
    """bytes [off, off+n) of the file held as chunks"""
    out = np.empty(n, np.uint8)
    k = int(np.searchsorted(starts, off, side="right")) - 1
    got = 0
    while got < n:
        c = chunks[k]
        a = off + got - int(starts[k])
        take = min(n - got, len(c) - a)
        out[got:got + take] = c[a:a + take]
        got += take
        k += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=50e9)
    ap.add_argument("--guesses", type=int, default=10000)
    ap.add_argument("--check", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunk", type=float, default=2.5e9)
    ap.add_argument("--resident", action="store_true")
    a = ap.parse_args()
    import torch
    import oracle
    from hadoop_bam import _lib
    threads = int(os.environ.get("OMP_NUM_THREADS", 16))
    chunks, nrec = gen_chunks(a.size, threads, a.chunk)
    starts = np.cumsum([0] + [len(c) for c in chunks[:-1]]).astype(np.int64)
    flen = int(starts[-1] + len(chunks[-1]))
    ctx = _lib.Context(0)
    head = cut(chunks, starts, 0, min(flen, 1 << 20))
    h = ctx.parse_header(head)
    assert isinstance(h, dict), h
    rng = np.random.default_rng(3)  # config #3 offsets
    beg = np.sort(rng.integers(0, flen - 1, a.guesses)).astype(np.int64)
    end = np.minimum(beg + (128 << 20), flen).astype(np.int64)
    wl = np.array([ctx.guess_window_len(flen, int(b), int(e)) for b, e in zip(beg, end)], np.int64)
    woff = np.zeros(a.guesses + 1, np.uint64)
    woff[1:] = np.cumsum(wl)
    t = time.time()
    windows = np.concatenate([cut(chunks, starts, int(b), int(n)) for b, n in zip(beg, wl)])
    log("gathered %d windows, %.2f GB, in %.1fs" % (a.guesses, len(windows) / 1e9, time.time() - t))
    if a.resident:
        data = np.concatenate(chunks)
        dsrc = torch.empty(flen + 64, dtype=torch.uint8, device="cuda")
        dsrc[:flen].copy_(torch.from_numpy(data))
        del data
        run = lambda: ctx.guess_batch(dsrc[:flen], beg, end, h["n_ref"])  # noqa: E731
        what = "whole file resident in HBM, hbam_guess_batch"
    else:
        dwin = torch.from_numpy(windows).cuda()  # the windows alone in HBM
        run = lambda: ctx.guess_windows(dwin, woff, flen, beg, end, h["n_ref"])  # noqa: E731
        what = "windows only (%.2f GB of a %.2f GB file) in HBM, hbam_guess_windows" % (len(windows) / 1e9, flen / 1e9)
    torch.cuda.synchronize()
    t = time.time()
    rc, out, err = run()  # warmup
    assert rc == 0, ctx.last_error()
    log("warmup %.3fs" % (time.time() - t))
    times = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t = time.time()
        rc, out, err = run()
        torch.cuda.synchronize()
        times.append(time.time() - t)
        assert rc == 0, ctx.last_error()
        log("rep %.3fs" % times[-1])
    # host-window path of the ABI (host windows staged by the library) must agree as well
    rc2, out2, err2 = ctx.guess_windows(windows, woff, flen, beg, end, h["n_ref"])
    assert rc2 == 0
    host_same = bool(np.array_equal(out2, out) and np.array_equal(err2, err))
    idx = np.sort(rng.choice(a.guesses, min(a.check, a.guesses), replace=False))
    res = {}

    def chk(ii):
        for i in ii:
            w = windows[int(woff[i]):int(woff[i + 1])]
            # the guesser over its window alone: beg 0, end = min(end-beg, ...) of the window
            e_rel = int(end[i] - beg[i])
            g, e = oracle.guess_bam_record_start(np.ascontiguousarray(w) if len(w) else np.zeros(1, np.uint8),
                                                 0, e_rel, h["n_ref"]) if len(w) else (e_rel, 0)
            g = int(end[i]) if g == e_rel else (int(beg[i]) << 16) + int(g)
            res[int(i)] = (g, int(e))
    ths = [threading.Thread(target=chk, args=(idx[j::threads],)) for j in range(threads)]
    t = time.time()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    cpu_s = (time.time() - t) * threads / len(idx)
    bad = sum((int(out[i]), int(err[i])) != res[int(i)] for i in idx)
    best = min(times)
    print(json.dumps({
        "metric": "BAMSplitGuesser guesses/s (config#3, one MI355X)",
        "value": round(a.guesses / best, 1), "unit": "guesses/s", "guesses": a.guesses,
        "seconds": round(best, 4), "all_reps_s": [round(x, 4) for x in times],
        "file_bytes": flen, "records": nrec, "window": "[off, off+128 MiB), reads <= 262139 B",
        "mode": what, "window_bytes": int(len(windows)),
        "window_gb_s": round(len(windows) / best / 1e9, 2),
        "host_windows_same": host_same,
        "parity_sample": int(len(idx)), "parity_mismatches": int(bad),
        "cpu_oracle_s_per_guess": round(cpu_s, 5),
        "cpu_oracle_guesses_per_s_1core": round(1.0 / cpu_s, 1)}), flush=True)
    if bad or not host_same:
        sys.exit(1)


if __name__ == "__main__":
    main()
