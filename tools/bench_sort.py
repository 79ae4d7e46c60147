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
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=12.5e9, help="compressed bytes per GPU")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed", type=int, default=5)
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
            "config": {"workload": "config#5 per GPU: unsorted synthetic 150bp PE BAM, decode + "
                                   "getKey + device radix sort + record pack%s" %
                                   (" + hbam_sort_exchange (RCCL grouped send/recv) by key range" if world > 1 else ""),
                       "compressed_bytes_per_gpu": len(data)},
        }), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
