"""Benchmark of the MI355X BAM read path (BASELINE.json metric).

Workload (BASELINE.json configs[1], "config #2"): a synthetic ~10 GB coordinate-sorted 150 bp
paired-end BAM per GPU (tools/gen_bam.cpp, zlib level 5, htsjdk-style packing), read exactly as
BAMRecordReader reads a FileVirtualSplit: BGZF scan, inflate, record-boundary walk, fixed-field
+ key decode, columnar pools.  A "step" = one hbam_decode_split over the rank's split with the
compressed bytes resident in HBM.

N GPUs (torch.distributed, one rank per GPU, config #4's shape): the N ranks shard ONE file of
N x ~10 GB by byte range.  Rank r holds file bytes [off_r, off_r + S_r) (its Hadoop FileSplit)
plus the next rank's first segment; its FileVirtualSplit is [guess(off_r), (off_r+S_r)<<16 |
0xffff] exactly as BAMInputFormat.addProbabilisticSplits builds it, and it decodes that split
as a window of the file (comp_base = off_r).  Nothing crosses ranks in the timed region except
the barrier; scaling is weak (per-GPU bytes fixed).  Records of a BGZF block that starts exactly
at a split boundary are read by both neighbouring splits, as in the reference; the record count
check subtracts them.

Prints ONE JSON line (rank 0).  roofline = the dominant kernel (the Huffman pass: k_inflate_tokens
at this size, k_inflate_wave for calls of up to HBAM_WAVE_MAX_BLOCKS blocks) with HIP events on
the context's stream, plus per-stage and whole-pipeline fractions; cpu_baseline = the
oracle's C restatement on a bounded sample on the host cores; parity = random FileVirtualSplits
of the benchmarked file re-read by the oracle outside the timed region.
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools"),
                os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

METRIC = "uncompressed BAM GB/s + records/s decoded (whole node, 1/2/4/8 MI355X)"
HBM_PEAK_GBS = 8000.0
# the library's Huffman pass: k_inflate_wave for calls of up to HBAM_WAVE_MAX_BLOCKS blocks
# (hbam_capi.hip), k_inflate_tokens above (a 10 GB shard: ~390k blocks)
WAVE_MAX_BLOCKS = int(os.environ.get("HBAM_WAVE_MAX_BLOCKS", "90000"))
N_REF = 25  # the generator's dictionary (tools/gen_bam.cpp)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads():
    """Threads this process may use: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the
    pool), else every CPU."""
    return int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def make_shard(size, seed, rank, world, threads, dist, dev):
    """Rank's byte range of ONE file of world * m segments (+ the next rank's first segment).
    Returns (host bytes, own length, file offset, file length, records in own range)."""
    import genbam
    import torch
    t = time.time()
    probe = genbam.generate_range(1, 0, 1, seed=seed, threads=threads)
    m = max(1, int(round(size / len(probe))))
    total = world * m
    own = genbam.generate_range(total, rank * m, m, header=(rank == 0), tail=(rank == world - 1),
                                seed=seed, threads=threads)
    nxt = (genbam.generate_range(total, (rank + 1) * m, 1, seed=seed, threads=threads)
           if rank < world - 1 else np.zeros(0, np.uint8))
    sizes = [len(own)]
    if dist:
        st = torch.tensor([len(own)], dtype=torch.int64, device=dev)
        allv = [torch.zeros_like(st) for _ in range(world)]
        dist.all_gather(allv, st)
        sizes = [int(x.item()) for x in allv]
    off = sum(sizes[:rank])
    buf = np.concatenate([np.asarray(own), nxt]) if len(nxt) else np.asarray(own)
    log("rank %d: %d segments of %d, bytes [%d, %d) of a %.2f GB file, generated in %.1fs"
        % (rank, m, total, off, off + len(own), sum(sizes) / 1e9, time.time() - t))
    return buf, len(own), off, sum(sizes), int(own.n_records)


def cpu_baseline(data, budget_s, threads):
    """Oracle (C restatement) on host cores, local-mode MapReduce shape: a prefix of the file cut
    into Hadoop FileSplits (one per thread), each aligned by the oracle's BAMSplitGuesser and
    read by the oracle's BAMRecordReader on its own thread (ctypes releases the GIL), producing
    the same output as the device decode: the fixed columns and keys plus the lazy getters'
    pools (names, CIGAR, SEQ characters, QUAL, AUX; oracle/hbam_oracle.c or_read_split_pools)."""
    import oracle
    L = oracle.lib()
    sample = int(min(len(data), budget_s * threads * 0.06e9))
    block = int(np.ceil(sample / threads))
    begs = list(range(0, sample, block))
    ends = [min(b + block, sample) for b in begs]
    base = np.ascontiguousarray(data[:sample + (1 << 20) if sample < len(data) else len(data)])
    vs, ve = oracle.probabilistic_splits(base, np.array(begs, np.uint64), np.array(ends, np.uint64))
    counts = [0] * len(vs)
    ubytes = [0] * len(vs)
    pbytes = [0] * len(vs)
    status = [0] * len(vs)

    def work(i):
        n, rb, pb = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        status[i] = L.or_read_split_pools(base.ctypes.data_as(C.POINTER(C.c_uint8)), len(base), int(vs[i]),
                                          int(ve[i]), -1, C.byref(n), C.byref(rb), C.byref(pb))
        counts[i], ubytes[i], pbytes[i] = n.value, rb.value, pb.value

    t = time.time()
    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(vs))]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.time() - t
    rec, ub = sum(counts), sum(ubytes)
    return {"value": round(ub / dt / 1e9, 4), "unit": "GB/s", "cores": len(vs), "kind": "port",
            "label": "CPU restatement (oracle/hbam_oracle.c: zlib inflate + BAMRecordCodec "
                     "decode + getKey + the lazy getters' pools), not the Java reference",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "records_per_s": round(rec / dt, 1), "seconds": round(dt, 3),
            "status": sorted(set(status)), "pool_bytes": int(sum(pbytes)),
            "sample": "first %.2f GB of the same compressed file (%d records, %.2f GB uncompressed "
                      "record bytes, %.2f GB of pools built), %d FileSplits aligned by the oracle "
                      "guesser, one thread each" % (sample / 1e9, rec, ub / 1e9, sum(pbytes) / 1e9, len(vs))}


POOLS = (("names", "name_off"), ("cigars", "cigar_off"), ("seq", "seq_off"), ("qual", "seq_off"),
         ("aux", "aux_off"))


def same_records(a, i0, b, j0, n):
    """records [i0, i0+n) of host columns a == records [j0, j0+n) of b: every fixed column and
    every decoded field pool (names, CIGAR, SEQ, QUAL, AUX)"""
    for k in ("voffset", "key", "block_size", "ref_id", "pos", "flag", "l_seq", "tlen", "mapq",
              "bin", "n_cigar", "l_read_name", "next_ref_id", "next_pos", "layout_ok"):
        if not np.array_equal(a[k][i0:i0 + n], b[k][j0:j0 + n]):
            return False
    for pool, off in POOLS:
        x = a[pool][int(a[off][i0]):int(a[off][i0 + n])]
        y = b[pool][int(b[off][j0]):int(b[off][j0 + n])]
        if not np.array_equal(x, y):
            return False
    return True


def parity_at_size(ctx, buf, dbuf, n_splits, seed, threads, whole=None):
    """n_splits random 32 MiB Hadoop FileSplits inside the rank's range: guess + decode on the
    device vs guess + BAMRecordReader of the oracle, every column, every decoded field pool and
    every record byte; then the same records inside the timed whole-shard decode (`whole`, its
    host copy) against the split's verified decode, so the big launch itself is checked."""
    import oracle
    rng = np.random.default_rng(seed)
    span = len(buf) - (48 << 20)
    if span <= 0:
        return None
    begs = np.sort(rng.integers(0, span, n_splits)).astype(np.int64)
    ends = begs + (32 << 20)
    rc, g, err = ctx.guess_batch(dbuf, begs, ends, N_REF)
    assert rc == 0
    sub = np.ascontiguousarray(buf)
    mism, recs = 0, 0
    w_recs, w_max, w_mism = 0, 0, 0
    res = [None] * n_splits

    def ref_one(i):
        go, ge = oracle.guess_bam_record_start(sub, int(begs[i]), int(ends[i]), N_REF)
        if ge or go == int(ends[i]):
            res[i] = (go, None)
            return
        r = oracle.read_split(sub, go, (int(ends[i]) << 16) | 0xffff, n_ref=N_REF)
        res[i] = (go, r)

    ths = [threading.Thread(target=ref_one, args=(i,)) for i in range(n_splits)]
    for k in range(0, n_splits, threads):
        for th in ths[k:k + threads]:
            th.start()
        for th in ths[k:k + threads]:
            th.join()
    for i in range(n_splits):
        go, r = res[i]
        if int(g[i]) != go:
            mism += 1
            continue
        if r is None:
            continue
        d = ctx.decode_split(dbuf, go, (int(ends[i]) << 16) | 0xffff, n_ref=N_REF)
        recs += r["n"]
        same = d["rc"] == 0 and d["n"] == r["n"] and d["status"] == r["status"]
        for k in ("voffset", "key", "block_size", "ref_id", "pos", "flag", "l_seq", "tlen"):
            same = same and np.array_equal(d[k], r[k])
        if same:
            pay, _ = oracle.record_payloads(r)
            same = d["ubuf"].tobytes() == pay.tobytes()
        if same:
            op = oracle.pools(r)
            same = np.array_equal(d["layout_ok"], op["layout_ok"]) and all(
                np.array_equal(d[k], op[k]) for k in ("names", "cigars", "seq", "qual", "aux"))
        mism += 0 if same else 1
        if whole is not None and same and d["n"]:
            lo = int(np.searchsorted(whole["voffset"], d["voffset"][0]))
            ok = lo + d["n"] <= whole["n"] and same_records(whole, lo, d, 0, d["n"])
            w_recs += d["n"]
            w_max = max(w_max, lo + d["n"])
            w_mism += 0 if ok else 1
    out = {"splits": n_splits, "mismatches": mism, "records": recs,
           "what": "random 32 MiB FileSplits of the benchmarked file: guessed start, every "
                   "column, every decoded field pool and every record byte vs the oracle"}
    if whole is not None:
        out["whole_shard"] = {"records_checked": w_recs, "highest_record_index": w_max,
                              "shard_records": whole["n"], "mismatches": w_mism,
                              "what": "the same records inside the timed whole-shard decode "
                                      "(one launch per kernel) equal the verified split decodes"}
    return out


WHOLE_CHECK_GROUP = 4  # ranks holding a whole-launch host copy at once (N > 1)


def host_views(hc):
    """numpy views (no copy) of a host hbam_columns, keyed as _lib.host_columns_to_numpy"""
    from hadoop_bam import _lib
    n = int(hc.n_records)
    out = {"n": n, "status": int(hc.status), "err_record": int(hc.err_record)}

    def view(p, cnt, dt):
        if not cnt or not p:
            return np.zeros(cnt if p else 0, dt)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(cnt,))
    for name, dt in _lib.FIXED:
        out[name] = view(getattr(hc, name), n, dt)
    for name in ("name_off", "cigar_off", "seq_off", "aux_off"):
        out[name] = view(getattr(hc, name), n + 1, np.uint64)
    out["ubuf"] = view(hc.ubuf, int(hc.ubuf_len), np.uint8)
    for name, dt, off in (("names", np.uint8, "name_off"), ("cigars", np.uint32, "cigar_off"),
                          ("seq", np.uint8, "seq_off"), ("qual", np.uint8, "seq_off"),
                          ("aux", np.uint8, "aux_off")):
        out[name] = view(getattr(hc, name), int(out[off][-1]) if n else 0, dt)
    return out


def whole_shard_check(ctx, cols, buf, own_len, off, threads):
    """Every record of the timed launch (its host copy: columns, pools, record bytes) against the
    oracle's BAMRecordReader over the same FileVirtualSplit, cut into FileSplits read in parallel
    (oracle.check_whole, C).  Returns (result dict, the host copy to free, or None)."""
    import oracle
    from hadoop_bam import _lib
    t = time.time()
    hc = _lib.Columns()
    if ctx.L.hbam_columns_to_host(ctx.h, C.byref(cols), C.byref(hc)):
        return {"error": "hbam_columns_to_host: %s" % ctx.last_error()}, None
    t_copy = time.time() - t
    try:
        d = oracle.OrDevCols()
        d.n = int(hc.n_records)
        d.voff_base = off << 16
        d.ubuf_len = int(hc.ubuf_len)
        for name, _ in oracle.OrDevCols._fields_:
            if name not in ("n", "voff_base", "ubuf_len"):
                setattr(d, name, C.cast(getattr(hc, name), C.c_void_p).value)
        res = oracle.check_whole(np.ascontiguousarray(buf), own_len, N_REF, d, off << 16, 4 * threads, threads)
    except Exception as e:  # reported, never hidden
        res = {"error": "%s: %s" % (type(e).__name__, e)}
    res["host_copy_s"] = round(t_copy, 2)
    res["seconds"] = round(time.time() - t, 2)
    res["what"] = ("every record of the timed launch (host copy of its output) vs the oracle's "
                   "BAMRecordReader over the same FileVirtualSplit (its start = the oracle's own guess), "
                   "read in pieces cut at the device's voffsets, each piece required to end exactly where "
                   "the next begins: voffset, key, every fixed column, the record bytes and every "
                   "lazy-getter pool (names, CIGAR, SEQ, QUAL, AUX, layout_ok), record by record")
    return res, hc


def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N rank processes (one per GPU) with
    the torch.distributed env of a single-node job, before this process touches a GPU; wait for
    all, end the others when one fails, and return the worst exit status."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(os.environ.get("MASTER_PORT") or free_port()))
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e))
    rc = 0
    while procs:
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0:
                rc = rc or r
                for q in procs:  # a rank died: the others would wait at a collective forever
                    q.terminate()
        time.sleep(0.2)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=float, default=10e9, help="compressed bytes per GPU")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-splits", type=int, default=32)
    ap.add_argument("--no-whole-check", action="store_true",
                    help="skip the check of every record of the timed launch against the oracle")
    ap.add_argument("--sort-size", type=float, default=2e9,
                    help="N > 1: compressed bytes per GPU of the unsorted file of the Sort leg (config #5 "
                         "shape; 12.5e9 = config #5's per-GPU share at 8 GPUs)")
    ap.add_argument("--sort-steps", type=int, default=2)
    ap.add_argument("--no-sort", action="store_true", help="N > 1: skip the Sort leg")
    ap.add_argument("--deadline", type=float, default=420.0,
                    help="N > 1: seconds from process start by which the Sort leg must end; its watchdog "
                         "fires then (rank 0 prints the line with the leg's error, every rank exits 3), so "
                         "a hung exchange never outlives the driver's limit with the headline unprinted")
    ap.add_argument("--config4", action="store_true",
                    help="BASELINE config #4 instead of the headline: ONE --c4-total file sharded over the N "
                         "GPUs (strong scaling), each rank's share resident, decoded in windows (tools/config4.py)")
    ap.add_argument("--c4-total", type=float, default=200e9, help="config #4 file size (compressed bytes)")
    ap.add_argument("--c4-body", type=float, default=5e9, help="config #4: generated body repeated to fill the file")
    ap.add_argument("--c4-window", type=float, default=0, help="config #4: window bytes (0: from free HBM)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d (launch with N ranks, or without a "
                         "launcher and let bench.py start them)" % (args.gpus, world))
    threads = host_threads()
    import torch
    dist = None
    # RCCL between GPUs; HBAM_BENCH_BACKEND=gloo rehearses the N>1 path with several ranks on
    # one GPU (host-staged collectives), which is how it is tested on the one-GPU pool
    backend = os.environ.get("HBAM_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from hadoop_bam import _lib
    ctx = _lib.Context(local)
    if args.config4:
        import config4
        res = config4.run(ctx, dist, rank, world, args, dev, cdev, threads, N_REF, log, METRIC, parity_at_size)
        if rank == 0:
            body = res.pop("_body")
            if not args.no_cpu_baseline:
                try:
                    res["cpu_baseline"] = cpu_baseline(body, args.cpu_budget, threads)
                except Exception as e:  # baseline is reported, never the target
                    res["cpu_baseline"] = {"error": str(e)}
            print(json.dumps(res), flush=True)
        if dist:
            dist.destroy_process_group()
        return

    buf, own_len, off, file_len, n_own = make_shard(int(args.size), args.seed, rank, world,
                                                    threads, dist, cdev)
    dcomp = torch.empty(len(buf) + 64, dtype=torch.uint8, device=dev)
    dcomp[len(buf):].zero_()
    dcomp[:len(buf)].copy_(torch.from_numpy(buf), non_blocking=False)
    torch.cuda.synchronize()
    # FileVirtualSplit of this rank's FileSplit [off, off + own_len) (BAMInputFormat.java:181-190)
    rc, g, err = ctx.guess_batch(dcomp[:len(buf)], np.array([0], np.int64),
                                 np.array([own_len], np.int64), N_REF)
    if rc or err[0] or int(g[0]) == own_len:
        raise RuntimeError("no record start in rank %d's split (rc %d err %d)" % (rank, rc, err[0]))
    v_start = (off << 16) + int(g[0])  # the guess is relative to the window start
    v_end = ((off + own_len) << 16) | 0xffff

    def step():
        rc, cols = ctx.decode_split_device(dcomp[:len(buf)], v_start, v_end, N_REF, comp_base=off,
                                           file_len=file_len)
        if rc != 0 or cols.status != 0:
            raise RuntimeError("decode failed rc=%d status=%d: %s" % (rc, cols.status, ctx.last_error()))
        return cols

    for _ in range(args.warmup):
        cols = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    huff_ms, stages = [], []
    for _ in range(args.steps):
        cols = step()
        t = ctx.timing()
        huff_ms.append(t["huffman_ms"])
        stages.append(t)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.time() - t0

    # ---- outside the timed region: record-count check, roofline inputs, parity
    n_rec = int(cols.n_records)
    ubytes = int(stages[-1]["ubuf_bytes"])
    overlap = 0
    if rank > 0 and n_rec:
        # records of the block that starts exactly at this split's beginning: the previous split
        # reads them too (vEnd = end<<16 | 0xffff, BAMInputFormat.java:189)
        k = min(n_rec, 4096)
        perm = torch.arange(k, dtype=torch.int32, device=dev)
        head = torch.empty(k, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()  # libhbam runs on its own stream: torch's arange must have landed
        assert ctx.L.hbam_permute(ctx.h, C.cast(cols.voffset, C.c_void_p), 8,
                                  C.c_void_p(perm.data_ptr()), k, C.c_void_p(head.data_ptr())) == 0
        overlap = int(((head.cpu() >> 16) == off).sum())
    tot = torch.tensor([elapsed, float(ubytes), float(n_rec), float(own_len), float(n_own),
                        float(overlap)], dtype=torch.float64, device=cdev)
    if dist:
        mx = tot.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        ub_all, rec_all, comp_all, gen_all, ovl_all = (float(sm[i]) for i in range(1, 6))
    else:
        ub_all, rec_all, comp_all, gen_all, ovl_all = float(ubytes), float(n_rec), float(own_len), \
            float(n_own), 0.0
    if int(rec_all - ovl_all) != int(gen_all):
        raise RuntimeError("decoded %d records (%d in boundary blocks read twice), generator wrote %d"
                           % (rec_all, ovl_all, gen_all))
    parity = None
    whole_res = None
    if not args.no_whole_check:
        # every record of the timed launch against the oracle, on every rank (its own shard); at
        # most WHOLE_CHECK_GROUP ranks hold their host copy (~2.3 x U) at once
        for turn in range(0, world, WHOLE_CHECK_GROUP):
            if turn <= rank < turn + WHOLE_CHECK_GROUP:
                whole_res, hc = whole_shard_check(ctx, cols, buf, own_len, off, threads)
                if rank == 0 and args.parity_splits > 0 and hc is not None:
                    try:
                        parity = parity_at_size(ctx, buf, dcomp[:len(buf)], args.parity_splits,
                                                args.seed + 17, threads, whole=host_views(hc))
                    except Exception as e:  # reported, never hidden
                        parity = {"error": str(e)}
                if hc is not None:
                    ctx.L.hbam_free_host_columns(C.byref(hc))
            if dist:
                dist.barrier()
        if dist:
            # every rank's verdict to rank 0
            mine = json.dumps(whole_res)
            got = [None] * world
            dist.all_gather_object(got, mine)
            whole_res = [json.loads(x) for x in got]
        else:
            whole_res = [whole_res]
    elif rank == 0 and args.parity_splits > 0:
        try:
            hc = _lib.Columns()
            if ctx.L.hbam_columns_to_host(ctx.h, C.byref(cols), C.byref(hc)):
                raise RuntimeError("hbam_columns_to_host: %s" % ctx.last_error())
            parity = parity_at_size(ctx, buf, dcomp[:len(buf)], args.parity_splits, args.seed + 17,
                                    threads, whole=host_views(hc))
            ctx.L.hbam_free_host_columns(C.byref(hc))
        except Exception as e:  # reported, never hidden
            parity = {"error": str(e)}
    if rank == 0 and whole_res is not None:
        parity = parity if parity is not None else {}
        parity["whole_launch"] = whole_res
    result = headline(args, world, elapsed, stages, huff_ms, ubytes, n_rec, own_len, file_len,
                      ub_all, rec_all, parity) if rank == 0 else None
    del cols
    if dist and not args.no_sort:
        # config #5's leg across the ranks (cli/plugins/Sort.java:131-170), after the headline's timed
        # region: decode + device sort + split points + exchange by key range (hbam_sort_exchange
        # over RCCL on nccl), with its own parity (tools/sort_leg.py)
        res = guarded_sort_leg(ctx, dist, rank, world, args, threads, dev, cdev, result)
        if rank == 0:
            result["sort"] = res
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:  # the CPU baseline: rank 0 at N = 1 only
            try:
                result["cpu_baseline"] = cpu_baseline(buf, args.cpu_budget, threads)
            except Exception as e:  # baseline is reported, never the target
                result["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


T_START = time.time()
WATCHDOG_EXIT = 3
SORT_LEG_MIN_S = 30.0  # a leg given less than this is skipped, not started


def sort_leg_budget(deadline, elapsed):
    """seconds the Sort leg may run: what is left of the whole-run deadline, or 0 (skip the leg)
    when less than SORT_LEG_MIN_S is left"""
    left = deadline - elapsed
    return left if left >= SORT_LEG_MIN_S else 0.0


def guarded_sort_leg(ctx, dist, rank, world, args, threads, dev, cdev, result):
    """The Sort leg under a watchdog.  Its exchange runs through libhbam's own RCCL communicator,
    which has no timeout of its own: if a rank fails, the others would wait in a collective for
    ever.  An exception is reported in the line (never hidden); a leg still running at --deadline
    seconds after process start ends every rank's process with status WATCHDOG_EXIT (rank 0 first
    prints the headline line with the Sort leg's error), so the headline measurement is never lost
    to the leg and the failure is still visible to the launcher."""
    import threading
    import sort_leg as sl
    done = threading.Event()
    budget = sort_leg_budget(args.deadline, time.time() - T_START)
    if budget <= 0:
        return {"error": "skipped: %.0f s of the %.0f s deadline already used before the leg"
                         % (time.time() - T_START, args.deadline)}

    def fire():
        if done.is_set():
            return
        if rank == 0 and result is not None:
            result["sort"] = {"error": "timeout: the leg did not end within the %.0f s deadline "
                                       "(%.0f s for the leg)" % (args.deadline, budget)}
            print(json.dumps(result), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(WATCHDOG_EXIT)  # a hung or failed multi-GPU leg is a failure, not a pass
    tm = threading.Timer(budget, fire)
    tm.daemon = True
    tm.start()
    try:
        return sl.run(ctx, dist, rank, world, int(args.sort_size), args.seed + 101, threads, dev, cdev,
                      N_REF, steps=args.sort_steps, log=log)
    except Exception as e:  # reported in the line, never hidden
        log("sort leg rank %d failed: %s: %s" % (rank, type(e).__name__, e))
        return {"error": "%s: %s" % (type(e).__name__, e)}
    finally:
        done.set()
        tm.cancel()


def headline(args, world, elapsed, stages, huff_ms, ubytes, n_rec, own_len, file_len, ub_all, rec_all, parity):
    """rank 0: the bench line of the timed decode (value, stages, roofline, parity)"""
    per_step = elapsed / args.steps
    value = ub_all / per_step / 1e9
    avg = {k: float(np.mean([s[k] for s in stages])) for k in stages[0] if isinstance(stages[0][k], float)}
    C_b, U_b, R = float(own_len), float(ubytes), float(n_rec)
    pool_b = float(stages[-1]["pool_bytes"])
    nblk = float(stages[-1]["n_blocks"])
    cols_b = R * (64 + 8 + 8) + 4 * 8 * (R + 1) + pool_b  # fixed columns + key/voffset/rec_off + pools
    # algorithmic bytes per stage; achieved = bytes / that stage's HIP-event time
    stage_bytes = {
        "scan": (C_b + 24 * nblk, avg["scan_ms"]),
        "huffman": (C_b + U_b, avg["huffman_ms"]),
        "resolve": (2 * U_b, avg["resolve_ms"]),
        "inflate": (C_b + U_b, avg["inflate_ms"]),
        "walk": (R * 20, avg["walk_ms"]),
        "decode": (R * 116, avg["decode_ms"]),
        "pools": (U_b + pool_b, avg["pools_ms"]),
    }
    stage_frac = {k: {"gb_s": round(b / (ms / 1e3) / 1e9, 1), "frac": round(b / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                      "bytes": int(b), "ms": round(ms, 3)} for k, (b, ms) in stage_bytes.items() if ms > 0}
    pipe_b = C_b + 2 * U_b + cols_b
    inf_ms = float(np.mean(huff_ms))
    alg = C_b + U_b
    achieved = alg / (inf_ms / 1e3) / 1e9
    traffic, traffic_src = None, None
    # the newest committed PMC pass of this kernel over the same workload (tools/pmc_summarize.py)
    huff_kernel = "k_inflate_wave" if nblk <= WAVE_MAX_BLOCKS else "k_inflate_tokens"
    pmc_files = ((("r04", "round4-wave", "pmc_huffman.json"),) if huff_kernel == "k_inflate_wave" else
                 (("r06", "round6", "pmc_k_inflate_tokens.json"), ("r05", "round5", "pmc_k_inflate_tokens.json"),
                  ("r04", "round4", "pmc_k_inflate_tokens.json")))
    for rnd, tree, fname in pmc_files:
        pmc = os.path.join(ROOT, "profiles", rnd, fname)
        if traffic is None and os.path.exists(pmc):
            try:
                pj = json.load(open(pmc))
                if pj.get("comp_bytes") and abs(pj["comp_bytes"] - C_b) / C_b < 0.05 and \
                        pj.get("kernel") == huff_kernel and pj.get("tree") == tree:
                    traffic, traffic_src = pj.get("hbm_bytes_per_launch"), "profiles/%s/%s" % (rnd, fname)
            except Exception:
                traffic = None
    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(per_step * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (tools/gen_bam.cpp: seeded 150bp PE, zlib level 5, BGZF)",
        "config": {"workload": "config#2 per GPU (config#4 shape for N>1): ~10 GB compressed "
                               "coordinate-sorted 150bp PE BAM per GPU, one file of N x 10 GB "
                               "sharded by byte range into guess-aligned FileVirtualSplits, BGZF "
                               "inflate + record decode + keys + columnar pools, input resident in HBM",
                   "compressed_bytes_per_gpu": own_len, "uncompressed_bytes_per_gpu": ubytes,
                   "records_per_gpu": n_rec, "file_bytes": file_len,
                   "parallelism": "shard%d" % world},
        "records_per_s": round(rec_all / per_step, 1),
        "stages_ms": {k: round(avg[k], 3) for k in ("scan_ms", "inflate_ms", "huffman_ms",
                                                    "resolve_ms", "walk_ms", "decode_ms",
                                                    "pools_ms", "total_ms")},
        "roofline": {"bound": "hbm", "kernel": huff_kernel, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": int(alg),
                     "stages": stage_frac,
                     "pipeline": {"bytes": int(pipe_b), "ms": round(avg["total_ms"], 3),
                                  "gb_s": round(pipe_b / (avg["total_ms"] / 1e3) / 1e9, 1),
                                  "frac": round(pipe_b / (avg["total_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "what": "C + 2U + columns/pools over the whole decode"},
                     "issue": issue_roofline(huff_kernel)},
        "parity": parity,
    }
    return result


# waves per SIMD each pass runs at (LDS and VGPR limits)
WAVES_PER_SIMD = {"k_inflate_tokens": 2, "k_resolve_units": 8}


def issue_roofline(kernel, src=os.path.join("profiles", "r06", "closing", "pmc_sq_3g.json")):
    """The bound that actually holds the Huffman pass: instruction issue, from the committed SQ
    counter pass of the same tree (tools/sq_fold.py).  A wave issues at most one instruction per
    quad-cycle; a SIMD-32 runs a wave64 VALU instruction in two cycles, so its VALU pipe takes at
    most two per quad-cycle.  None when the file is absent."""
    try:
        k = json.load(open(os.path.join(ROOT, src)))["kernels"][kernel]
    except Exception:
        return None
    w = WAVES_PER_SIMD.get(kernel)
    valu = k["active_inst_valu_frac"]
    return {"kernel": kernel, "source": src, "waves_per_simd": w,
            "wave_issue_frac": round(k["active_inst_any_frac"], 4),
            "wave_valu_issue_frac": round(valu, 4),
            "simd_valu_pipe_frac": round(valu * w / 2.0, 4) if w else None,
            "wait_frac": round(k["wait_any_frac"], 4), "dependency_stall_frac": round(k["wait_inst_any_frac"], 4),
            "what": "SQ_ACTIVE_INST_ANY / _VALU, SQ_WAIT_ANY and SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES (quad-cycles) "
                    "per wave; the SIMD's VALU pipe share = VALU issue per wave x waves per SIMD / 2"}


if __name__ == "__main__":
    main()
