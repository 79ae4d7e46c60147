"""Config #4 on one GPU: a BAM shard in host memory read as one FileVirtualSplit through the
streamed reader (hbam_split_open/next: windows of --window compressed bytes, the next window
copied H2D on a second stream while the current one decodes).  The rate is PCIe-inclusive
(host bytes in, device columns out); it is the rate a map task reading a host-resident file
sees, never bench.py's device-resident `value`.  Parity (--parity, outside the timed runs): the
windows' records equal one device-resident decode of the same split — every voffset and key, and
for the 64 records on each side of every window cut (where the EMORE continuation resumes)
every fixed column and the record bytes.  Prints one JSON line per window size."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=20e9)
    ap.add_argument("--window", type=float, nargs="+", default=[4e9],
                    help="window sizes (compressed bytes); one JSON line each")
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--parity", type=int, default=1, help="check the windows against a resident decode")
    a = ap.parse_args()
    import torch
    import genbam
    from hadoop_bam import _lib
    t = time.time()
    g = genbam.generate(target_bytes=int(a.size), seed=a.seed, threads=int(os.environ.get("OMP_NUM_THREADS", 16)))
    n = len(g)
    host = np.empty(n + 64, np.uint8)
    host[:n] = np.asarray(g)
    host[n:] = 0
    nrec = int(g.n_records)
    del g
    print("generated %.2f GB (%d records) in %.1fs" % (n / 1e9, nrec, time.time() - t), file=sys.stderr, flush=True)
    ctx = _lib.Context(0)
    # page-locked for libhbam's own HIP runtime (torch's pin_memory belongs to another runtime in
    # this process, so its buffers are pageable to the library and every window copy blocked)
    t = time.time()
    assert ctx.L.hbam_host_register(ctx.h, C.c_void_p(host.ctypes.data), host.size) == 0, ctx.last_error()
    print("registered %.2f GB in %.1fs" % (host.size / 1e9, time.time() - t), file=sys.stderr, flush=True)
    h = ctx.parse_header(host[:n])
    v0, v1 = h["first_voffset"], (n << 16) | 0xffff
    rc, blocks = ctx.scan_blocks(host[:n])
    assert rc == 0
    U = int(np.sum(blocks["isize"].astype(np.uint64)))  # the file's inflated bytes
    lines = [one_window_size(a, ctx, host, n, nrec, h, v0, v1, U, int(win)) for win in a.window]
    if a.parity:
        ctx.close()  # its window-sized work buffers; the check decodes the whole file resident
        par = stream_parity(host, n, h, v0, v1, int(a.window[-1]))
        lines[-1]["parity"] = par
    for ln in lines:
        print(json.dumps(ln), flush=True)
    if not all(ln["record_count_matches_generator"] for ln in lines) or \
            (a.parity and lines[-1]["parity"]["mismatches"] != 0):
        sys.exit(1)


def _vp(p):
    return C.cast(p, C.c_void_p).value


def stream_parity(host, n, h, v0, v1, win):
    """The streamed read of [v0, v1) in windows of `win` against one resident decode of the same
    bytes: every voffset / key, and every fixed column + record bytes of the 64 records on each
    side of each window cut."""
    import torch
    from hadoop_bam import _lib
    t = time.time()
    cs = _lib.Context(0)
    vo, ky, sl = [], [], []
    base = 0
    for d in cs.split_stream(host[:n], v0, v1, h["n_ref"], window_bytes=win, host=False):
        m = int(d.n_records)
        vo.append(cs.download(_vp(d.voffset), 8 * m, np.uint64).copy())
        ky.append(cs.download(_vp(d.key), 8 * m, np.int64).copy())
        sl.append((base, cs.columns_slice(d, 0, min(64, m))))
        sl.append((base + max(0, m - 64), cs.columns_slice(d, max(0, m - 64), m)))
        base += m
    cs.close()
    svo, sky = np.concatenate(vo), np.concatenate(ky)
    del vo, ky
    cr = _lib.Context(0)
    dev = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    dev[n:].zero_()
    dev[:n].copy_(torch.from_numpy(host[:n]))
    rc, d = cr.decode_split_device(dev[:n], v0, v1, h["n_ref"])
    assert rc == 0 and int(d.status) == 0, (rc, cr.last_error())
    R = int(d.n_records)
    mism = 0 if R == base else 1
    rvo = cr.download(_vp(d.voffset), 8 * R, np.uint64)
    rky = cr.download(_vp(d.key), 8 * R, np.int64)
    mism += 0 if (R == base and np.array_equal(rvo, svo) and np.array_equal(rky, sky)) else 1
    checked, bad = 0, 0
    for start, got in sl:
        ref = cr.columns_slice(d, start, start + got["n"])
        same = all(np.array_equal(got[k], ref[k]) for k, _ in _lib.FIXED if k != "rec_off")
        same = same and got["records"] == ref["records"]
        checked += got["n"]
        bad += 0 if same else 1
    cr.close()
    return {"records": base, "resident_records": R, "windows": len(sl) // 2,
            "boundary_records_checked": checked, "boundary_slices_bad": bad,
            "mismatches": mism + bad, "seconds": round(time.time() - t, 1),
            "what": "every voffset and key of the streamed windows == one resident decode of the file; "
                    "the 64 records on each side of every window cut: every fixed column and the "
                    "record bytes"}


def one_window_size(a, ctx, host, n, nrec, h, v0, v1, U, win):
    import torch
    reps = []
    for r in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.time()
        recs, ub, wins = 0, 0, 0
        marks = []
        for d in ctx.split_stream(host[:n], v0, v1, h["n_ref"], window_bytes=win, host=False):
            recs += int(d.n_records)
            wins += 1
            if int(d.status) != 0:
                raise RuntimeError("window status %d" % d.status)
            t = ctx.timing()
            ub += int(t["ubuf_bytes"])  # per window, overlap re-reads included
            marks.append((round(time.time() - t0, 4), round(t["total_ms"], 2)))
        dt = time.time() - t0
        st = ctx.last_stream_stats
        reps.append((dt, recs, ub, wins, st, marks))
        print("window %.1f GB rep %d: %.3fs %d records %d windows h2d %.1f GB in %.1f ms; per window "
              "(host s at return, decode ms): %s" % (win / 1e9, r, dt, recs, wins, st["h2d_bytes"] / 1e9,
                                                     st["h2d_ms"], marks), file=sys.stderr, flush=True)
    dt, recs, ub, wins, st, marks = min(reps, key=lambda x: x[0])
    ok = recs == nrec
    return ({
        "metric": "streamed split decode, PCIe-inclusive (config#4 shape, one MI355X)",
        "value": round(U / dt / 1e9, 3), "unit": "GB/s uncompressed", "uncompressed_bytes": U,
        "inflated_incl_window_overlap": ub, "records_per_s": round(recs / dt, 1),
        "compressed_gb_s": round(n / dt / 1e9, 3), "seconds": round(dt, 4), "all_reps_s": [round(x[0], 4) for x in reps],
        "file_bytes": n, "window_bytes": win, "windows": wins, "records": recs,
        "per_window_host_s_and_decode_ms": marks,
        "h2d": {"bytes": st["h2d_bytes"], "ms": round(st["h2d_ms"], 2),
                "gb_s": round(st["h2d_bytes"] / max(st["h2d_ms"], 1e-9) / 1e6, 2)},
        "host_buffer": "page-locked for libhbam (hbam_host_register)", "record_count_matches_generator": ok})


if __name__ == "__main__":
    main()
