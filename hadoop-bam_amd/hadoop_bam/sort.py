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

    def _gather(self, ubuf_ptr, rec_off_ptr, bs_ptr, perm_ptr, n, size_only=False):
        t = self.torch
        off = t.empty(n + 1, dtype=t.int64, device=self.dev)
        self._after_torch()
        tot = C.c_uint64(0)
        self._chk(self.L.hbam_gather_records(self.ctx.h, C.c_void_p(ubuf_ptr), C.c_void_p(rec_off_ptr),
                                             C.c_void_p(bs_ptr), C.c_void_p(perm_ptr), n, None, 0,
                                             C.c_void_p(off.data_ptr()), C.byref(tot)),
                  "hbam_gather_records(size)")
        if size_only:
            return None, off
        out = t.empty(max(int(tot.value), 1), dtype=t.uint8, device=self.dev)
        self._chk(self.L.hbam_gather_records(self.ctx.h, C.c_void_p(ubuf_ptr), C.c_void_p(rec_off_ptr),
                                             C.c_void_p(bs_ptr), C.c_void_p(perm_ptr), n,
                                             C.c_void_p(out.data_ptr()), out.numel(),
                                             C.c_void_p(off.data_ptr()), C.byref(tot)),
                  "hbam_gather_records")
        return out[:int(tot.value)], off

    def run_from_columns(self, cols):
        """Sorted run of a decoded split (device hbam_columns from decode_split_device)."""
        n = int(cols.n_records)
        keys, perm = self._sort(_addr(cols.key), n)
        vo = self._permute(_addr(cols.voffset), 8, perm, n)
        bs = self._permute(_addr(cols.block_size), 4, perm, n)
        payload, off = self._gather(_addr(cols.ubuf), _addr(cols.rec_off), _addr(cols.block_size),
                                    perm.data_ptr(), n)
        return SortedRun(keys, vo, bs, payload, off)

    def sort_received(self, keys, voffset, block_size, payload):
        """Stable sort of an exchange's receive buffers (chunks in source-rank order)."""
        n = int(keys.numel())
        _, rec_off = self._gather(0, 0, block_size.data_ptr(), 0, n, size_only=True)  # offsets of received records
        keys_s, perm = self._sort(keys.data_ptr(), n)
        vo = self._permute(voffset.data_ptr(), 8, perm, n)
        bs = self._permute(block_size.data_ptr(), 4, perm, n)
        out, off = self._gather(payload.data_ptr(), rec_off.data_ptr(), block_size.data_ptr(),
                                perm.data_ptr(), n)
        return SortedRun(keys_s, vo, bs, out, off)


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


def exchange(run, split_points, dist, ops):
    """all_to_all of a SortedRun by key range; returns this rank's globally-ordered run.
    Keys <= split_points[r-1]... : rank r receives keys in (sp[r-1], sp[r]]."""
    import torch
    world = dist.get_world_size()
    dev = run.keys.device
    sp = torch.as_tensor(np.asarray(split_points, np.int64), device=dev)
    cuts = torch.searchsorted(run.keys, sp, right=True) if run.n else torch.zeros_like(sp)
    bounds = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), cuts.to(torch.int64),
                        torch.full((1,), run.n, dtype=torch.int64, device=dev)])
    rec_cnt = bounds[1:] - bounds[:-1]
    byte_b = run.offsets[bounds]
    byte_cnt = byte_b[1:] - byte_b[:-1]
    meta = torch.stack([rec_cnt, byte_cnt]).t().contiguous()  # [world, 2]
    rmeta = torch.empty_like(meta)
    dist.all_to_all_single(rmeta, meta)
    send_r = rec_cnt.cpu().tolist()
    send_b = byte_cnt.cpu().tolist()
    rm = rmeta.cpu().numpy()
    recv_r = [int(x) for x in rm[:, 0]]
    recv_b = [int(x) for x in rm[:, 1]]
    nr, nb = sum(recv_r), sum(recv_b)

    def a2a(src, n_out, dtype, s_split, r_split):
        out = torch.empty(n_out, dtype=dtype, device=dev)
        dist.all_to_all_single(out, src.contiguous(), r_split, s_split)
        return out

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
