"""Coordinate Sort plugin path (config #5).

Mirrors Sort.java:84-188: records keyed by BAMRecordReader.getKey (SortRecordReader,
Sort.java:279-295), a TotalOrderPartitioner over sampled split points (Sort.java:149-157),
identity SortReducer (Sort.java:191-205), output = the reducers' outputs concatenated in
partition order.  The value each record carries is its SAMRecordWritable wire form
(block_size + record bytes, SAMRecordWritable.java:62-63).

MI355X design — one process per GPU, one exchange step:
  1. every rank decodes its byte-range shard (hbam_decode_split) and sorts its keys on the
     device (hbam_sort_keys: stable LSD radix), carrying voffset / block_size (hbam_permute)
     and packing the record bytes in key order (hbam_gather_records);
  2. regular samples of the sorted local keys are all-gathered; the P-1 split points are their
     quantiles (deterministic, unlike the reference's unseeded RandomSampler — a partition
     choice never changes the concatenated order);
  3. one all_to_all_single per column (keys, voffsets, block sizes, record bytes) over RCCL /
     xGMI; every destination range is contiguous in the locally sorted order, so no packing
     kernel is needed beyond step 1;
  4. each rank stably sorts what it received (chunks arrive in source-rank order = file order),
     so the global order is (key, voffset) — the documented tie-break.

The exchange logic is written against a small ops interface so that the world-size-2 gloo tests
can drive it on the CPU with the oracle's sort; the product ops (HipSortOps) are libhbam calls
and fail loudly without the HIP library.
"""
import ctypes as C

import numpy as np


class SortedRun:
    """One rank's records in (key, input order) order: device (or CPU-test) tensors."""

    def __init__(self, keys, voffset, block_size, payload, offsets):
        self.keys = keys            # int64[n]   LongWritable keys, ascending (signed)
        self.voffset = voffset      # int64[n]   virtual offset of each record in its file
        self.block_size = block_size  # int32[n]
        self.payload = payload      # uint8[B]   concatenated SAMRecordWritable payloads
        self.offsets = offsets      # int64[n+1] payload offsets

    @property
    def n(self):
        return int(self.keys.numel())


def _addr(p):
    return C.cast(p, C.c_void_p).value


class HipSortOps:
    """Product ops: every step is a libhbam call on the context's device and stream."""

    def __init__(self, ctx):
        import torch
        self.torch = torch
        self.ctx = ctx
        self.L = ctx.L
        self.dev = torch.device("cuda", torch.cuda.current_device())

    def _after_torch(self):
        """libhbam runs on its own non-blocking HIP stream; tensors torch produced (an RCCL
        all_to_all, an asynchronous copy) are complete only on torch's current stream.  Every
        entry point below that hands torch tensors to libhbam waits for that stream first."""
        self.torch.cuda.current_stream().synchronize()

    def _chk(self, rc, what):
        if rc != 0:
            raise RuntimeError("%s failed (%d): %s" % (what, rc, self.ctx.last_error()))

    def _sort(self, key_ptr, n):
        t = self.torch
        keys_out = t.empty(n, dtype=t.int64, device=self.dev)
        perm = t.empty(max(n, 1), dtype=t.int32, device=self.dev)
        self._after_torch()
        self._chk(self.L.hbam_sort_keys(self.ctx.h, C.c_void_p(key_ptr), n,
                                        C.c_void_p(keys_out.data_ptr()), C.c_void_p(perm.data_ptr())),
                  "hbam_sort_keys")
        return keys_out, perm

    def _permute(self, src_ptr, elem, perm, n):
        t = self.torch
        out = t.empty(n, dtype=t.int64 if elem == 8 else t.int32, device=self.dev)
        self._after_torch()
        self._chk(self.L.hbam_permute(self.ctx.h, C.c_void_p(src_ptr), elem, C.c_void_p(perm.data_ptr()),
                                      n, C.c_void_p(out.data_ptr())), "hbam_permute")
        return out

    def _run(self, call, n_hint):
        """Size query, torch-owned outputs, then the call itself (hbam_sort_split/received)."""
        from ._lib import SortedRunC
        t = self.torch
        q = SortedRunC()
        self._chk(call(C.byref(q)), "sorted-run size query")
        n, nb = int(q.n), int(q.payload_bytes)
        keys = t.empty(max(n, 1), dtype=t.int64, device=self.dev)
        vo = t.empty(max(n, 1), dtype=t.int64, device=self.dev)
        bs = t.empty(max(n, 1), dtype=t.int32, device=self.dev)
        off = t.empty(n + 1, dtype=t.int64, device=self.dev)
        pay = t.empty(max(nb, 1), dtype=t.uint8, device=self.dev)
        r = SortedRunC(n, nb, keys.data_ptr(), vo.data_ptr(), bs.data_ptr(), off.data_ptr(),
                       pay.data_ptr())
        self._after_torch()
        self._chk(call(C.byref(r)), "sorted run")
        if n == 0:
            off.zero_()
        return SortedRun(keys[:n], vo[:n], bs[:n], pay[:nb], off)

    def run_from_columns(self, cols):
        """hbam_sort_split: sorted run of a decoded split (device hbam_columns)."""
        return self._run(lambda r: self.L.hbam_sort_split(self.ctx.h, C.byref(cols), r), cols.n_records)

    def sort_received(self, keys, voffset, block_size, payload):
        """hbam_sort_received: stable sort of an exchange's receive buffers (chunks in
        source-rank order)."""
        n = int(keys.numel())
        return self._run(lambda r: self.L.hbam_sort_received(
            self.ctx.h, C.c_void_p(keys.data_ptr()), C.c_void_p(voffset.data_ptr()),
            C.c_void_p(block_size.data_ptr()), C.c_void_p(payload.data_ptr()), n, r), n)

    def partition(self, run, split_points):
        """hbam_sort_partition: TotalOrderPartitioner record / byte bounds (host int64 arrays)."""
        from ._lib import SortedRunC
        sp = np.ascontiguousarray(split_points, np.int64)
        P = len(sp) + 1
        rb = np.zeros(P + 1, np.uint64)
        bb = np.zeros(P + 1, np.uint64)
        r = SortedRunC(run.n, int(run.offsets[-1].item()) if run.n else 0, run.keys.data_ptr(),
                       run.voffset.data_ptr(), run.block_size.data_ptr(), run.offsets.data_ptr(),
                       run.payload.data_ptr())
        self._after_torch()
        self._chk(self.L.hbam_sort_partition(self.ctx.h, C.byref(r), C.c_void_p(sp.ctypes.data), P,
                                             C.c_void_p(rb.ctypes.data), C.c_void_p(bb.ctypes.data)),
                  "hbam_sort_partition")
        return rb.astype(np.int64), bb.astype(np.int64)


def choose_split_points(keys_sorted, world, all_gather_fn, samples_per_rank=4096):
    """TotalOrderPartitioner split points (world-1 int64) from regular samples of every rank's
    sorted keys; deterministic.  all_gather_fn(np.int64 array) -> concatenation over ranks."""
    n = int(keys_sorted.numel())
    if n:
        k = min(n, samples_per_rank)
        idx = (np.arange(k, dtype=np.int64) * n) // k
        import torch
        local = keys_sorted[torch.as_tensor(idx, device=keys_sorted.device)].cpu().numpy()
    else:
        local = np.zeros(0, np.int64)
    allv = np.sort(all_gather_fn(np.asarray(local, np.int64)), kind="stable")
    if len(allv) == 0:
        return np.zeros(world - 1, np.int64)
    q = (np.arange(1, world, dtype=np.int64) * len(allv)) // world
    return allv[q].astype(np.int64)


def exchange(run, split_points, dist, ops, stage_cpu=None):
    """all_to_all of a SortedRun by key range; returns this rank's globally-ordered run.
    Rank r receives the keys in (sp[r-1], sp[r]].  With a CPU-only backend (gloo) and device
    runs, the collective's buffers are staged through host memory (stage_cpu, default: gloo)."""
    import torch
    world = dist.get_world_size()
    dev = run.keys.device
    if stage_cpu is None:
        stage_cpu = dev.type != "cpu" and dist.get_backend() == "gloo"
    xdev = torch.device("cpu") if stage_cpu else dev
    if hasattr(ops, "partition"):
        rb, bb = ops.partition(run, split_points)
        rec_cnt = torch.as_tensor(rb[1:] - rb[:-1], dtype=torch.int64)
        byte_cnt = torch.as_tensor(bb[1:] - bb[:-1], dtype=torch.int64)
    else:
        sp = torch.as_tensor(np.asarray(split_points, np.int64), device=dev)
        cuts = torch.searchsorted(run.keys, sp, right=True) if run.n else torch.zeros_like(sp)
        bounds = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), cuts.to(torch.int64),
                            torch.full((1,), run.n, dtype=torch.int64, device=dev)])
        rec_cnt = (bounds[1:] - bounds[:-1]).cpu()
        byte_b = run.offsets[bounds]
        byte_cnt = (byte_b[1:] - byte_b[:-1]).cpu()
    meta = torch.stack([rec_cnt, byte_cnt]).t().contiguous().to(xdev)  # [world, 2]
    rmeta = torch.empty_like(meta)
    dist.all_to_all_single(rmeta, meta)
    send_r = rec_cnt.tolist()
    send_b = byte_cnt.tolist()
    rm = rmeta.cpu().numpy()
    recv_r = [int(x) for x in rm[:, 0]]
    recv_b = [int(x) for x in rm[:, 1]]
    nr, nb = sum(recv_r), sum(recv_b)

    def a2a(src, n_out, dtype, s_split, r_split):
        out = torch.empty(n_out, dtype=dtype, device=xdev)
        dist.all_to_all_single(out, src.contiguous().to(xdev), r_split, s_split)
        return out.to(dev)

    keys = a2a(run.keys, nr, torch.int64, send_r, recv_r)
    vo = a2a(run.voffset, nr, torch.int64, send_r, recv_r)
    bs = a2a(run.block_size, nr, torch.int32, send_r, recv_r)
    payload = a2a(run.payload[:int(run.offsets[-1])] if run.n else run.payload[:0], nb, torch.uint8,
                  send_b, recv_b)
    return ops.sort_received(keys, vo, bs, payload)


def sort_sharded(run, dist, ops, all_gather_fn):
    """Steps 2-4 for one rank: split points, exchange, local stable sort."""
    sp = choose_split_points(run.keys, dist.get_world_size(), all_gather_fn)
    return exchange(run, sp, dist, ops)
