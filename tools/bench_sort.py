"""Config #5 benchmark: coordinate Sort plugin path on an unsorted synthetic BAM.

Per rank (one process per GPU; torchrun for N > 1, hbam_sort_exchange over RCCL): decode the rank's shard
(hbam_decode_split, compressed bytes resident in HBM), key-sort it on the device
(hbam_sort_keys + hbam_permute + hbam_gather_records), then — N > 1 — split points,
all_to_all by key range and the local stable re-sort (hadoop_bam/sort.py).  Prints one JSON
line (rank 0): records/s and uncompressed GB/s through decode+sort, stage times, and the radix
sort's own roofline (HBM bytes moved per pass / time).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=12.5e9, help="compressed bytes per GPU")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--parity", type=int, default=1)
    ap.add_argument("--oracle-splits", type=int, default=32)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import genbam
    from hadoop_bam import _lib, parallel, sort
    g = genbam.generate(target_bytes=int(a.size), seed=a.seed + 1000 * rank, sorted=0,
                        threads=int(os.environ.get("OMP_NUM_THREADS", 16)))
    data = np.asarray(g)
    print("rank %d generated %.2f GB, %d records" % (rank, len(data) / 1e9, g.n_records),
          file=sys.stderr, flush=True)
    d = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
    d[:len(data)].copy_(torch.from_numpy(data))
    ctx = _lib.Context(local)
    # N > 1: the exchange is libhbam's own (hbam_sort_exchange over an RCCL communicator)
    ops = sort.HipSortOps(ctx, sort.RcclComm.from_dist(ctx, dist) if dist else None)
    h = ctx.parse_header(d[:len(data)])
    ag = parallel.torch_all_gather_fn(dist, "cuda") if dist else None

    def step():
        t0 = time.time()
        rc, cols = ctx.decode_split_device(d[:len(data)], h["first_voffset"],
                                           (len(data) << 16) | 0xffff, h["n_ref"])
        assert rc == 0 and cols.status == 0, (rc, ctx.last_error())
        t1 = time.time()
        run = ops.run_from_columns(cols)
        sort_dev_ms = ctx.timing()["total_ms"]
        passes = ctx.timing()["n_blocks"]
        torch.cuda.synchronize()
        t2 = time.time()
        if dist:
            run = sort.sort_sharded(run, dist, ops, ag)
            torch.cuda.synchronize()
        t3 = time.time()
        return run, int(cols.n_records), ctx, (t1 - t0, t2 - t1, t3 - t2, sort_dev_ms, passes)

    for _ in range(a.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    st = []
    for _ in range(a.steps):
        run, n_dec, _, s = step()
        st.append(s)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.time() - t0
    ub = float(run.offsets[-1].item()) if run.n else 0.0
    # sanity: the output is sorted by key and covers every decoded record
    k = run.keys
    assert bool((k[1:] >= k[:-1]).all()) if run.n > 1 else True
    parity = None
    if a.parity and not dist:
        parity = sort_parity(ctx, ops, d[:len(data)], data, h, run, a)
    tot = torch.tensor([el, float(n_dec), float(run.n), ub], dtype=torch.float64, device="cuda")
    if dist:
        mx = tot.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        el, n_all, n_out, ub_all = float(mx[0]), float(sm[1]), float(sm[2]), float(sm[3])
    else:
        n_all, n_out, ub_all = float(n_dec), float(run.n), ub
    if rank == 0:
        assert n_out == n_all, (n_out, n_all)
        per = el / a.steps
        m = np.mean(np.array(st), axis=0)
        sort_ms = float(m[3])
        passes = int(st[-1][4])
        # radix: per pass, keys+idx read twice (count, scatter) and written once: 36 B/record
        alg = n_dec * (36.0 * passes + 8 + 12)  # + init (read key, write key+idx)
        print(json.dumps({
            "metric": "coordinate Sort plugin: records/s decoded + sorted (config #5)",
            "value": round(n_all / per, 1), "unit": "records/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(per * 1e3, 3),
            "uncompressed_GBps": round(ub_all / per / 1e9, 3),
            "stages_s": {"decode": round(float(m[0]), 4), "local_sort_pack": round(float(m[1]), 4),
                         "exchange_resort": round(float(m[2]), 4)},
            "radix": {"ms": round(sort_ms, 3), "passes": passes, "records": n_dec,
                      "achieved_GBps": round(alg / (sort_ms / 1e3) / 1e9, 1) if sort_ms else None},
            "parity": parity,
            "config": {"workload": "config#5 per GPU: unsorted synthetic 150bp PE BAM, decode + "
                                   "getKey + device radix sort + record pack%s" %
                                   (" + hbam_sort_exchange (RCCL grouped send/recv) by key range" if world > 1 else ""),
                       "compressed_bytes_per_gpu": len(data)},
        }), flush=True)
    if dist:
        dist.destroy_process_group()


def sort_parity(ctx, ops, dev, data, h, run, a):
    """The timed run's output at size (SortReducer's output order, Sort.java:191-205): ordered by
    (key, voffset) (the documented tie-break), its voffsets a permutation of the decoded split's,
    every payload the decoded record's bytes (re-gathered from the decode by voffset, compared on
    the device in chunks); then --oracle-splits random 32 MiB FileSplits decoded and sorted on the
    device against the oracle's read_split + sort order, payload bytes included."""
    import ctypes as C
    import torch
    import oracle
    t = time.time()
    n = run.n
    k, v = run.keys, run.voffset
    order_ok = bool(((k[1:] > k[:-1]) | ((k[1:] == k[:-1]) & (v[1:] > v[:-1]))).all()) if n > 1 else True
    # the decoded split again (the context's buffers): its voffsets in file order
    rc, cols = ctx.decode_split_device(dev, h["first_voffset"], (len(data) << 16) | 0xffff, h["n_ref"])
    assert rc == 0 and cols.status == 0
    m = int(cols.n_records)
    ident = torch.arange(m, dtype=torch.int32, device="cuda")
    dv = torch.empty(m, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # libhbam runs on its own stream: torch's arange must have landed
    assert ctx.L.hbam_permute(ctx.h, C.cast(cols.voffset, C.c_void_p), 8, C.c_void_p(ident.data_ptr()), m,
                              C.c_void_p(dv.data_ptr())) == 0
    del ident
    j = torch.searchsorted(dv, v)
    perm_ok = m == n and bool((j < m).all()) and bool((dv[j.clamp(max=m - 1)] == v).all())
    if perm_ok:
        seen = torch.zeros(m, dtype=torch.int8, device="cuda")
        seen[j] = 1
        perm_ok = bool(seen.all())
        del seen
    pay_bad = 0
    if perm_ok:
        jp = j.to(torch.int32)
        chunk = 1 << 22
        for c0 in range(0, n, chunk):
            c1 = min(n, c0 + chunk)
            lo, hi = int(run.offsets[c0]), int(run.offsets[c1])
            exp = torch.empty(hi - lo + 64, dtype=torch.uint8, device="cuda")
            off = torch.empty(c1 - c0 + 1, dtype=torch.int64, device="cuda")
            tot = C.c_uint64(0)
            assert ctx.L.hbam_gather_records(ctx.h, C.cast(cols.ubuf, C.c_void_p), C.cast(cols.rec_off, C.c_void_p),
                                             C.cast(cols.block_size, C.c_void_p), C.c_void_p(jp.data_ptr() + 4 * c0),
                                             c1 - c0, C.c_void_p(exp.data_ptr()), hi - lo + 64,
                                             C.c_void_p(off.data_ptr()), C.byref(tot)) == 0
            if int(tot.value) != hi - lo or not torch.equal(exp[:hi - lo], run.payload[lo:hi]):
                pay_bad += 1
    # oracle sample: random 32 MiB FileSplits, device decode + sort vs the oracle
    rng = np.random.default_rng(a.seed + 77)
    span = len(data) - (48 << 20)
    o_bad, o_recs = 0, 0
    host = np.ascontiguousarray(data)
    for beg in (np.sort(rng.integers(0, span, a.oracle_splits)) if span > 0 else []):
        end = int(beg) + (32 << 20)
        vs, ve = oracle.probabilistic_splits(host, np.array([beg], np.uint64), np.array([end], np.uint64))
        rc, dc = ctx.decode_split_device(dev, int(vs[0]), int(ve[0]), h["n_ref"])
        ref = oracle.read_split(host, int(vs[0]), int(ve[0]))
        pay, offs = oracle.record_payloads(ref)
        o = oracle.sort_order(ref["key"])
        noff, npay = oracle._regather(pay, offs, o)
        sr = ops.run_from_columns(dc)
        same = rc == 0 and sr.n == ref["n"] and np.array_equal(sr.keys.cpu().numpy(), ref["key"][o]) and \
            np.array_equal(sr.voffset.cpu().numpy(), ref["voffset"].astype(np.int64)[o]) and \
            sr.payload.cpu().numpy().tobytes() == npay.tobytes()
        o_bad += 0 if same else 1
        o_recs += ref["n"]
    return {"order_key_voffset": order_ok, "voffsets_permutation_of_decode": perm_ok,
            "payload_chunks_bad": pay_bad, "records": n,
            "oracle_splits": a.oracle_splits, "oracle_records": o_recs, "oracle_mismatches": o_bad,
            "mismatches": (0 if order_ok else 1) + (0 if perm_ok else 1) + pay_bad + o_bad,
            "seconds": round(time.time() - t, 1),
            "what": "whole timed output: (key, voffset) order, voffsets a permutation of the decoded "
                    "split's, every payload == the decoded record's bytes; plus random 32 MiB splits "
                    "sorted on the device == the oracle's order and payloads"}


if __name__ == "__main__":
    main()
