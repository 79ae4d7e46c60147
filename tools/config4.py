"""`bench.py --config4`: BASELINE config #4 — ONE 200 GB synthetic BAM decoded by N GPUs, each rank
its byte range of the file (200/N GB compressed) resident in HBM (strong scaling: the total is fixed).

The file is built so that 200 GB can exist without 200 GB of generator time: the BAM header's BGZF
blocks, then copies of one generated body (whole generator segments: every copy starts and ends on
a BGZF block and a record boundary), then the EOF block.  Copies are dealt to ranks in contiguous
runs; rank r's Hadoop FileSplit is its byte range and its FileVirtualSplit
[guess(start), end << 16 | 0xffff] (BAMInputFormat.java:181-190), as in the headline.

A rank's share can exceed what one hbam_decode_split may hold in HBM beside it (at N = 1: 200 GB
resident + the decode's buffers, ~6.5x the window), so a step decodes the share in windows of W
compressed bytes: each call stops at the last record that completes inside its window
(HBAM_EMORE) and the next window starts at that record's voffset (include/hbam.h, windows).
At N = 8 (25 GB per GPU) one window covers the share.

Parity (outside the timed region): the record count over all ranks equals the copies' records
(+ the records of boundary blocks read by both neighbours, as the reference reads them); a second,
checked pass maps every record of every window to its body-relative virtual offset and compares
voffset, key and block_size with one resident decode of the body, which is itself compared with the
oracle on random 32 MiB FileSplits (bench.parity_at_size).
"""
import ctypes as C
import time

import numpy as np

EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _dev_copy(ctx, ptr, n, elem, dev):
    """n elements of library device memory at ptr -> a torch tensor (hbam_permute, identity)."""
    import torch
    ident = torch.arange(max(n, 1), dtype=torch.int32, device=dev)
    out = torch.empty(max(n, 1), dtype=torch.int64 if elem == 8 else torch.int32, device=dev)
    torch.cuda.synchronize()
    # (hbam_permute returns once its stream is done)
    assert ctx.L.hbam_permute(ctx.h, C.c_void_p(ptr), elem, C.c_void_p(ident.data_ptr()), n,
                              C.c_void_p(out.data_ptr())) == 0, ctx.last_error()
    return out[:n]


def _vp(p):
    return C.cast(p, C.c_void_p).value


def build(rank, world, total, body_target, seed, threads, dev, cdev, dist, log):
    import torch
    import genbam
    from hadoop_bam import parallel
    t = time.time()
    hdr = np.asarray(genbam.generate_range(1, 0, 0, header=True, seed=seed, threads=threads))
    probe = genbam.generate_range(1, 0, 1, seed=seed, threads=threads)
    mb = max(1, int(round(body_target / len(probe))))
    body = genbam.generate_range(mb, 0, mb, seed=seed, threads=threads)
    n_body = int(body.n_records)
    body = np.asarray(body)
    B = len(body)
    copies = max(world, int(round((total - len(hdr)) / B)))
    lo, hi = parallel.owner_ranges(copies, world)[rank]
    off = 0 if rank == 0 else len(hdr) + lo * B
    own_len = (len(hdr) if rank == 0 else 0) + (hi - lo) * B + (len(EOF_BLOCK) if rank == world - 1 else 0)
    file_len = len(hdr) + copies * B + len(EOF_BLOCK)
    tail = min(B, 4 << 20) if rank < world - 1 else 0  # the next rank's first bytes (records running past)
    n = own_len + tail
    d = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    d[n:].zero_()
    hb = torch.from_numpy(body)
    p = 0
    if rank == 0:
        d[:len(hdr)].copy_(torch.from_numpy(hdr))
        p = len(hdr)
    for _ in range(hi - lo):
        d[p:p + B].copy_(hb)
        p += B
    if rank == world - 1:
        d[p:p + len(EOF_BLOCK)].copy_(torch.frombuffer(bytearray(EOF_BLOCK), dtype=torch.uint8))
        p += len(EOF_BLOCK)
    if tail:
        d[p:p + tail].copy_(hb[:tail])
        p += tail
    assert p == n
    torch.cuda.synchronize()
    log("config4 rank %d: copies [%d, %d) of %d x %.2f GB body (%d records each), bytes [%d, %d) of a "
        "%.1f GB file, built in %.1fs" % (rank, lo, hi, copies, B / 1e9, n_body, off, off + own_len,
                                          file_len / 1e9, time.time() - t))
    return dict(hdr_len=len(hdr), body=body, B=B, n_body=n_body, copies=copies, lo=lo, hi=hi, off=off,
                own_len=own_len, file_len=file_len, d=d, n=n)


def windowed_decode(ctx, f, v_start, v_end, W, n_ref, on_window=None):
    """The share decoded in windows of W compressed bytes; returns (records, uncompressed bytes,
    windows, summed stage times)."""
    d, off, n = f["d"], f["off"], f["n"]
    v = v_start
    recs, ub, nwin = 0, 0, 0
    st = {}
    while True:
        a = (v >> 16) - off
        b = min(n, a + W)
        rc, cols = ctx.decode_split_device(d[a:b], v, v_end, n_ref, comp_base=off + a, file_len=f["file_len"])
        if rc:
            raise RuntimeError("config4 window at %d: rc %d: %s" % (a, rc, ctx.last_error()))
        t = ctx.timing()
        for k, x in t.items():
            if isinstance(x, float):
                st[k] = st.get(k, 0.0) + x
        m = int(cols.n_records)
        if on_window is not None:
            on_window(cols, m)
        recs += m
        ub += int(t["ubuf_bytes"])
        nwin += 1
        if cols.status == -12:  # HBAM_EMORE: resume at voffset[m]
            nv = int(ctx.download(_vp(cols.voffset) + 8 * m, 8, np.uint64)[0])
            if nv <= v and m == 0:
                raise RuntimeError("config4: window of %d bytes holds no whole record" % W)
            v = nv
            continue
        if cols.status != 0:
            raise RuntimeError("config4: split status %d" % cols.status)
        return recs, ub, nwin, st


def run(ctx, dist, rank, world, args, dev, cdev, threads, n_ref, log, metric, parity_fn):
    import torch
    f = build(rank, world, args.c4_total, min(args.c4_body, args.c4_total / world), args.seed, threads, dev,
              cdev, dist, log)
    d = f["d"]
    rc, g, err = ctx.guess_batch(d[:f["n"]], np.array([0], np.int64), np.array([f["own_len"]], np.int64), n_ref)
    if rc or err[0] or int(g[0]) == f["own_len"]:
        raise RuntimeError("config4: no record start in rank %d's split" % rank)
    off = f["off"]
    v_start, v_end = (off << 16) + int(g[0]), ((off + f["own_len"]) << 16) | 0xffff
    free = torch.cuda.mem_get_info(dev)[0]
    W = int(min(f["n"], args.c4_window or 1e15, max(1 << 30, free * 0.8 / 6.5)))
    log("config4 rank %d: %.1f GB free beside the share -> windows of %.2f GB" % (rank, free / 1e9, W / 1e9))
    for _ in range(args.warmup):
        windowed_decode(ctx, f, v_start, v_end, W, n_ref)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        recs, ub, nwin, st = windowed_decode(ctx, f, v_start, v_end, W, n_ref)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.time() - t0
    # records of the block starting exactly at this rank's first byte are read by the previous split too
    overlap = 0
    if rank > 0:
        first = {}

        def grab(cols, m):
            if not first:
                k = min(m, 4096)
                first["v"] = _dev_copy(ctx, _vp(cols.voffset), k, 8, dev).cpu().numpy()
        windowed_decode(ctx, f, v_start, min(v_end, ((off + (4 << 20)) << 16) | 0xffff), W, n_ref, grab)
        overlap = int(((first["v"] >> 16) == off).sum()) if first else 0

    # ---- checked pass: every record vs the body's resident decode
    body = f["body"]
    hoff = f["hdr_len"]
    # the body alone, as its own file window (copy 0 sits at file offset hoff on rank 0's layout; here
    # decoded from a device copy of the body with comp_base 0 as a headerless stream)
    db = torch.empty(len(body) + 64, dtype=torch.uint8, device=dev)
    db[len(body):].zero_()
    db[:len(body)].copy_(torch.from_numpy(body))
    torch.cuda.synchronize()
    rc, rcols = ctx.decode_split_device(db[:len(body)], 0, (len(body) << 16) | 0xffff, n_ref)
    assert rc == 0 and rcols.status == 0, (rc, ctx.last_error())
    nb = int(rcols.n_records)
    ref_v = _dev_copy(ctx, _vp(rcols.voffset), nb, 8, dev)
    ref_k = _dev_copy(ctx, _vp(rcols.key), nb, 8, dev)
    ref_bs = _dev_copy(ctx, _vp(rcols.block_size), nb, 4, dev)
    B = f["B"]
    bad = [0, 0]  # records checked, mismatches

    def check(cols, m):
        if not m:
            return
        v = _dev_copy(ctx, _vp(cols.voffset), m, 8, dev)
        k = _dev_copy(ctx, _vp(cols.key), m, 8, dev)
        bs = _dev_copy(ctx, _vp(cols.block_size), m, 4, dev)
        co = (v >> 16) - hoff  # compressed offset from the first copy
        rel = ((co % B) << 16) | (v & 0xffff)
        j = torch.searchsorted(ref_v, rel).clamp(max=nb - 1)
        ok = (ref_v[j] == rel) & (ref_k[j] == k) & (ref_bs[j] == bs)
        bad[0] += m
        bad[1] += int((~ok).sum())
    windowed_decode(ctx, f, v_start, v_end, W, n_ref, check)
    body_parity = None
    if rank == 0 and args.parity_splits > 0:
        body_parity = parity_fn(ctx, body, db[:len(body)], args.parity_splits, args.seed + 17, threads)
    del db, ref_v, ref_k, ref_bs
    tot = torch.tensor([el, float(ub), float(recs), float(f["own_len"]), float(overlap), float(bad[0]),
                        float(bad[1]), float((f["hi"] - f["lo"]) * f["n_body"]), float(nwin)],
                       dtype=torch.float64, device=cdev)
    if dist:
        mx, sm = tot.clone(), tot.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    else:
        mx = sm = tot
    if rank != 0:
        return None
    result_body = body
    el = float(mx[0])
    per = el / args.steps
    ub_all, rec_all, comp_all = float(sm[1]), float(sm[2]), float(sm[3])
    count_ok = int(rec_all - float(sm[4])) == int(sm[7])
    mism = (0 if count_ok else 1) + int(sm[6]) + (body_parity["mismatches"] if body_parity else 0)
    return {
        "metric": metric, "value": round(ub_all / per / 1e9, 3), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(per * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (tools/gen_bam.cpp body, zlib level 5, repeated: tools/config4.py)",
        "config": {"workload": "config#4: ONE %.0f GB synthetic BAM sharded by byte range over %d GPU(s), "
                               "%.1f GB compressed per GPU resident in HBM, decoded in windows of %.2f GB "
                               "(%d per step on rank 0)" % (f["file_len"] / 1e9, world, f["own_len"] / 1e9,
                                                            W / 1e9, nwin),
                   "file_bytes": f["file_len"], "windows_per_step_rank0": nwin, "compressed_bytes_all_gpus": int(comp_all),
                   "uncompressed_bytes_all_gpus": int(ub_all), "records_all_gpus": int(rec_all),
                   "parallelism": "shard%d" % world},
        "records_per_s": round(rec_all / per, 1),
        "stages_ms_rank0_per_step": {k: round(x, 3) for k, x in st.items()},
        "roofline": {"bound": "hbm", "kernel": "Huffman pass (per window)",
                     "achieved": round((f["own_len"] + ub) / (st["huffman_ms"] / 1e3) / 1e9, 2),
                     "peak": 8000.0, "unit": "GB/s",
                     "frac": round((f["own_len"] + ub) / (st["huffman_ms"] / 1e3) / 1e9 / 8000.0, 4),
                     "traffic": None},
        "parity": {"record_count_matches": count_ok, "records_checked_vs_body_decode": int(sm[5]),
                   "record_mismatches": int(sm[6]), "body_vs_oracle": body_parity, "mismatches": mism,
                   "what": "every record of every window: body-relative voffset, key and block_size == one "
                           "resident decode of the body; the body decode vs the oracle on random 32 MiB "
                           "FileSplits; total records == copies x body records (+ boundary-block records "
                           "read twice)"},
        "_body": result_body,
    }
