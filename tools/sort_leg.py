"""Config #5's leg of `bench.py --gpus N` (N > 1): the coordinate Sort plugin across the ranks.

Run after the headline's timed decode, by every rank (cli/plugins/Sort.java:84-188: SortRecordReader
keys, TotalOrderPartitioner over sampled split points :131-157, the shuffle, identity SortReducer
:191-205).  Each rank holds its byte range of ONE unsorted synthetic file (the same sharding as the
headline: a guess-aligned FileVirtualSplit per rank) and runs
  hbam_decode_split -> hbam_sort_split -> split points -> exchange -> hbam_sort_received;
on the nccl backend the split points and the exchange are libhbam's own (hbam_comm_init with rank
0's unique id broadcast over torch.distributed, hbam_comm_split_points, hbam_sort_exchange: one
grouped ncclSend/ncclRecv per peer over xGMI); on gloo (the one-GPU rehearsal) the host-staged
all_to_all of hadoop_bam/sort.py.

Parity of the timed output, outside the timed region:
  * order: every rank's records in (key, voffset) order, and across ranks the last record of rank r
    before the first of rank r+1 (the concatenation is the total order; a record read by both
    neighbouring splits — its block starts exactly at a split boundary — appears twice, adjacent);
  * permutation + payload: each record gets a fingerprint of its payload bytes (position-weighted,
    computed on the device); the sums over records of (voffset hash) and (fingerprint x voffset
    hash), all-reduced, equal between the decoded splits (in file order) and the sorted output, and
    so do the record counts: the output is a permutation of the decoded records, each with its own
    bytes;
  * oracle sample: random records of each rank's decoded split equal the oracle's record at the
    same virtual offset (oracle/, the CPU restatement) byte for byte.
"""
import ctypes as C
import threading
import time

import numpy as np

MIX = -7046029254386353131  # 0x9E3779B97F4A7C15 as a signed int64
MIX2 = -4658895280553007687  # 0xBF58476D1CE4E5B9


def _vhash(v):
    import torch
    h = v.to(torch.int64) * MIX
    h = h ^ (h >> 31)
    return h * MIX2


def fingerprints(pay, offs, chunk=1 << 20):
    """Per-record fingerprint of packed payloads (device uint8 `pay`, int64 `offs` [n+1]):
    sum over the record's bytes of (byte + 1) * hash(position in the record), wrapping int64."""
    import torch
    n = int(offs.numel()) - 1
    dev = pay.device
    fp = torch.zeros(max(n, 0), dtype=torch.int64, device=dev)
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        lo, hi = int(offs[c0]), int(offs[c1])
        starts = offs[c0:c1]
        lens = offs[c0 + 1:c1 + 1] - starts
        seg = torch.repeat_interleave(torch.arange(c1 - c0, device=dev), lens)
        pos = torch.arange(lo, hi, device=dev, dtype=torch.int64) - starts[seg]
        h = (pay[lo:hi].to(torch.int64) + 1) * _vhash(pos + 1)
        fp[c0:c1].scatter_add_(0, seg, h)
        del seg, pos, h
    return fp


def _stats(voff, fp):
    import torch
    g = _vhash(voff)
    return torch.stack([torch.tensor(int(voff.numel()), dtype=torch.int64, device=voff.device),
                        g.sum(), (fp * g).sum(), fp.sum()])


def run(ctx, dist, rank, world, size, seed, threads, dev, cdev, n_ref, steps=2, samples=256, log=print):
    import torch
    import genbam
    from hadoop_bam import parallel, sort
    native = dist.get_backend() == "nccl"
    t = time.time()
    probe = genbam.generate_range(1, 0, 1, seed=seed, threads=threads, sorted=0)
    m = max(1, int(round(size / len(probe))))
    total = world * m
    own = genbam.generate_range(total, rank * m, m, header=(rank == 0), tail=(rank == world - 1),
                                seed=seed, threads=threads, sorted=0)
    nxt = (genbam.generate_range(total, (rank + 1) * m, 1, seed=seed, threads=threads, sorted=0)
           if rank < world - 1 else np.zeros(0, np.uint8))
    st = torch.tensor([len(own)], dtype=torch.int64, device=cdev)
    allv = [torch.zeros_like(st) for _ in range(world)]
    dist.all_gather(allv, st)
    sizes = [int(x.item()) for x in allv]
    off, file_len, own_len = sum(sizes[:rank]), sum(sizes), len(own)
    buf = np.concatenate([np.asarray(own), nxt]) if len(nxt) else np.asarray(own)
    log("sort leg rank %d: unsorted bytes [%d, %d) of a %.2f GB file, generated in %.1fs"
        % (rank, off, off + own_len, file_len / 1e9, time.time() - t))
    d = torch.empty(len(buf) + 64, dtype=torch.uint8, device=dev)
    d[len(buf):].zero_()
    d[:len(buf)].copy_(torch.from_numpy(buf))
    torch.cuda.synchronize()
    rc, g, err = ctx.guess_batch(d[:len(buf)], np.array([0], np.int64), np.array([own_len], np.int64), n_ref)
    if rc or err[0] or int(g[0]) == own_len:
        raise RuntimeError("sort leg: no record start in rank %d's split" % rank)
    v_start, v_end = (off << 16) + int(g[0]), ((off + own_len) << 16) | 0xffff
    comm = sort.RcclComm.from_dist(ctx, dist) if native else None
    ops = sort.HipSortOps(ctx, comm)
    ag = parallel.torch_all_gather_fn(dist, cdev)

    def step():
        t0 = time.time()
        rc, cols = ctx.decode_split_device(d[:len(buf)], v_start, v_end, n_ref, comp_base=off, file_len=file_len)
        if rc or cols.status:
            raise RuntimeError("sort leg decode rc=%d status=%d: %s" % (rc, cols.status, ctx.last_error()))
        local = ops.run_from_columns(cols)
        torch.cuda.synchronize()
        t1 = time.time()
        out = sort.sort_sharded(local, dist, ops, ag)
        torch.cuda.synchronize()
        t2 = time.time()
        return out, int(cols.n_records), (t1 - t0, t2 - t1, ctx.timing()["exchange_ms"] if native else 0.0)

    out, n_dec, _ = step()  # warm-up (allocations, RCCL connections)
    del out
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.time()
    parts = []
    for _ in range(steps):
        out, n_dec, p = step()
        parts.append(p)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.time() - t0
    pm = np.mean(np.array(parts), axis=0)
    agg = torch.tensor([el, pm[0], pm[1], pm[2], float(n_dec), float(out.n),
                        float(int(out.offsets[-1]) if out.n else 0)], dtype=torch.float64, device=cdev)
    mx, sm = agg.clone(), agg.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)

    # ---- parity (outside the timed region)
    tp = time.time()
    n = out.n
    k, v = out.keys, out.voffset
    # (key, voffset) non-decreasing: equal pairs are the records of a block starting exactly at a
    # split boundary, which both neighbouring splits read (as the reference does)
    order_ok = bool(((k[1:] > k[:-1]) | ((k[1:] == k[:-1]) & (v[1:] >= v[:-1]))).all()) if n > 1 else True
    ends = torch.tensor([n, int(k[0]) if n else 0, int(v[0]) if n else 0, int(k[-1]) if n else 0,
                         int(v[-1]) if n else 0], dtype=torch.int64, device=cdev)
    ends_all = [torch.zeros_like(ends) for _ in range(world)]
    dist.all_gather(ends_all, ends)
    e = [x.cpu().numpy() for x in ends_all]
    boundary_ok, last = True, None
    for r in range(world):
        if e[r][0] == 0:
            continue
        if last is not None and not (last[0] < e[r][1] or (last[0] == e[r][1] and last[1] <= e[r][2])):
            boundary_ok = False
        last = (e[r][3], e[r][4])
    s_out = _stats(v, fingerprints(out.payload, out.offsets))
    del out, k, v
    # the decoded split again (file order), its records packed by hbam_gather_records
    rc, cols = ctx.decode_split_device(d[:len(buf)], v_start, v_end, n_ref, comp_base=off, file_len=file_len)
    assert rc == 0 and cols.status == 0
    nd = int(cols.n_records)
    ident = torch.arange(max(nd, 1), dtype=torch.int32, device=dev)
    dv = torch.empty(max(nd, 1), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()  # libhbam runs on its own stream: torch's arange must have landed
    assert ctx.L.hbam_permute(ctx.h, C.cast(cols.voffset, C.c_void_p), 8, C.c_void_p(ident.data_ptr()), nd,
                              C.c_void_p(dv.data_ptr())) == 0
    tot = C.c_uint64(0)
    poff = torch.empty(nd + 1, dtype=torch.int64, device=dev)
    assert ctx.L.hbam_gather_records(ctx.h, C.cast(cols.ubuf, C.c_void_p), C.cast(cols.rec_off, C.c_void_p),
                                     C.cast(cols.block_size, C.c_void_p), None, nd, None, 0,
                                     C.c_void_p(poff.data_ptr()), C.byref(tot)) == 0
    pay = torch.empty(int(tot.value) + 64, dtype=torch.uint8, device=dev)
    assert ctx.L.hbam_gather_records(ctx.h, C.cast(cols.ubuf, C.c_void_p), C.cast(cols.rec_off, C.c_void_p),
                                     C.cast(cols.block_size, C.c_void_p), None, nd, C.c_void_p(pay.data_ptr()),
                                     int(tot.value) + 64, C.c_void_p(poff.data_ptr()), C.byref(tot)) == 0
    torch.cuda.synchronize()
    s_dec = _stats(dv[:nd], fingerprints(pay, poff))
    both = torch.stack([s_dec, s_out]).to(cdev)
    dist.all_reduce(both)
    perm_ok = bool(torch.equal(both[0], both[1]))
    # oracle sample: random records of this rank's decoded split vs the oracle's record there
    import oracle
    rng = np.random.default_rng(seed + 31 * rank)
    pick = np.sort(rng.choice(nd, size=min(samples, nd), replace=False)) if nd else np.zeros(0, np.int64)
    vo = dv[:nd].cpu().numpy()
    po = poff.cpu().numpy()
    host_pay = {int(i): pay[int(po[i]):int(po[i + 1])].cpu().numpy().tobytes() for i in pick}
    sub = np.ascontiguousarray(buf)
    bad = [0]
    lock = threading.Lock()

    def chk(ix):
        for i in ix:
            rv = int(vo[i]) - (off << 16)
            ref = oracle.read_split(sub, rv, rv + 1, n_ref=n_ref)
            okk = ref["n"] == 1 and oracle.record_payloads(ref)[0].tobytes() == host_pay[int(i)]
            if not okk:
                with lock:
                    bad[0] += 1
    ths = [threading.Thread(target=chk, args=(pick[j::threads],)) for j in range(min(threads, max(len(pick), 1)))]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    flags = torch.tensor([0 if order_ok else 1, bad[0], len(pick)], dtype=torch.int64, device=cdev)
    dist.all_reduce(flags)
    if comm is not None:
        comm.close()
    del d, pay, poff, dv, ident
    torch.cuda.empty_cache()
    if rank != 0:
        return None
    el, n_all = float(mx[0]), float(sm[4])
    per = el / steps
    mism = int(flags[0]) + (0 if boundary_ok else 1) + (0 if perm_ok else 1) + int(flags[1])
    return {
        "workload": "config#5 shape across the ranks: ONE unsorted synthetic 150bp PE BAM of N x %.2f GB "
                    "sharded by byte range; decode + getKey + device radix sort + record pack, split points, "
                    "exchange by key range, re-sort" % (size / 1e9),
        "transport": ("hbam_sort_exchange: grouped ncclSend/ncclRecv per peer (RCCL, xGMI)" if native
                      else "host-staged torch.distributed all_to_all (gloo rehearsal)"),
        "records_per_s": round(n_all / per, 1), "records": int(n_all), "steps": steps,
        "ms_per_step": round(per * 1e3, 3),
        "stages_ms_max_over_ranks": {"decode_sort_pack": round(float(mx[1]) * 1e3, 3),
                                     "split_points_exchange_resort": round(float(mx[2]) * 1e3, 3),
                                     "exchange_rccl": round(float(mx[3]), 3) if native else None},
        "payload_bytes": int(sm[6]),
        "parity": {"order_key_voffset_every_rank": int(flags[0]) == 0, "rank_boundaries_ordered": boundary_ok,
                   "permutation_with_own_payload": perm_ok, "records_out": int(sm[5]), "records_decoded": int(sm[4]),
                   "oracle_sample": {"records": int(flags[2]), "mismatches": int(flags[1])},
                   "mismatches": mism, "seconds": round(time.time() - tp, 1)},
    }
