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
  3. the exchange by key range: with an RcclComm (one GPU per rank) it is libhbam's own
     hbam_sort_exchange — a count all-gather and one grouped ncclSend/ncclRecv of keys,
     voffsets, block sizes and record bytes over xGMI, behind the C ABI a Java host binds too;
     with a gloo group (CPU tests, ranks sharing one GPU) one all_to_all_single per column
     staged through host memory.  Every destination range is contiguous in the locally sorted
     order, so no packing kernel is needed beyond step 1;
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


class RcclComm:
    """libhbam's RCCL communicator (hbam_comm_init): one rank per GPU, the Sort exchange's
    transport behind the C ABI (SURVEY.md §8(b) hbam_sort_multi_gpu).  Collective: every rank
    constructs it with the same 128-byte unique id (rank 0's hbam_comm_unique_id)."""

    ID_BYTES = 128

    def __init__(self, ctx, nranks, rank, unique_id):
        self.ctx = ctx
        self.L = ctx.L
        self.nranks, self.rank = int(nranks), int(rank)
        uid = (C.c_uint8 * self.ID_BYTES).from_buffer_copy(bytes(unique_id))
        self.h = C.c_void_p()
        rc = self.L.hbam_comm_init(ctx.h, uid, self.nranks, self.rank, C.byref(self.h))
        if rc:
            raise RuntimeError("hbam_comm_init failed (%d): %s" % (rc, ctx.last_error()))

    @staticmethod
    def unique_id(L):
        buf = (C.c_uint8 * RcclComm.ID_BYTES)()
        rc = L.hbam_comm_unique_id(buf)
        if rc:
            raise RuntimeError("hbam_comm_unique_id failed (%d): RCCL unavailable" % rc)
        return bytes(buf)

    @classmethod
    def from_dist(cls, ctx, dist):
        """Rank 0's unique id broadcast over an initialised torch.distributed group."""
        import torch
        rank, world = dist.get_rank(), dist.get_world_size()
        dev = (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl"
               else torch.device("cpu"))
        t = torch.zeros(cls.ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            t.copy_(torch.frombuffer(bytearray(cls.unique_id(ctx.L)), dtype=torch.uint8))
        dist.broadcast(t, 0)
        return cls(ctx, world, rank, t.cpu().numpy().tobytes())

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.L.hbam_comm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HipSortOps:
    """Product ops: every step is a libhbam call on the context's device and stream.  With an
    RcclComm the split points and the exchange are libhbam's too (hbam_comm_split_points,
    hbam_sort_exchange)."""

    def __init__(self, ctx, comm=None):
        import torch
        self.torch = torch
        self.ctx = ctx
        self.L = ctx.L
        self.comm = comm
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

    @staticmethod
    def _run_struct(run):
        from ._lib import SortedRunC
        return SortedRunC(run.n, int(run.offsets[-1].item()) if run.n else 0, run.keys.data_ptr(),
                          run.voffset.data_ptr(), run.block_size.data_ptr(), run.offsets.data_ptr(),
                          run.payload.data_ptr())

    def split_points_native(self, run, samples_per_rank=4096):
        """hbam_comm_split_points: regular samples of every rank's sorted keys all-gathered over
        RCCL, their nranks-1 quantiles (choose_split_points' rule)."""
        P = self.comm.nranks
        sp = np.zeros(max(P - 1, 1), np.int64)
        r = self._run_struct(run)
        self._after_torch()
        self._chk(self.L.hbam_comm_split_points(self.ctx.h, self.comm.h, C.byref(r), samples_per_rank,
                                                C.c_void_p(sp.ctypes.data)), "hbam_comm_split_points")
        return sp[:P - 1]

    def exchange_native(self, run, split_points):
        """hbam_sort_exchange: partition, count all-gather, grouped ncclSend/ncclRecv, re-sort."""
        sp = np.ascontiguousarray(split_points, np.int64)
        if len(sp) == 0:
            sp = np.zeros(1, np.int64)
        r = self._run_struct(run)
        return self._run(lambda o: self.L.hbam_sort_exchange(self.ctx.h, self.comm.h, C.byref(r),
                                                             C.c_void_p(sp.ctypes.data), o), run.n)

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
    if getattr(ops, "comm", None) is not None:
        return ops.exchange_native(run, split_points)
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
    if getattr(ops, "comm", None) is not None:
        return ops.exchange_native(run, ops.split_points_native(run))
    sp = choose_split_points(run.keys, dist.get_world_size(), all_gather_fn)
    return exchange(run, sp, dist, ops)


# ---- several inputs: Utils.getSAMHeaderMerger / correctSAMRecordForMerging -------------------
class SAMException(RuntimeError):
    """htsjdk.samtools.SAMException"""


def _header_records(text, tag):
    """(ID, [(tag, value), ...] without ID) of every @RG / @PG line of a header text, in order."""
    out = []
    for ln in text.split(b"\n"):
        if ln.startswith(tag + b"\t"):
            attrs = [(f[:2], f[3:]) for f in ln.split(b"\t")[1:] if len(f) >= 3]
            rid = next((v for k, v in attrs if k == b"ID"), b"")
            out.append((rid, [(k, v) for k, v in attrs if k != b"ID"]))
    return out


def _rec_key(attrs):
    """AbstractSAMHeaderRecord equality: the attribute map (last value of a repeated tag)."""
    return frozenset(dict(attrs).items())


def merge_header_records(records, taken, table, out):
    """SamFileHeaderMerger.mergeHeaderRecords (htsjdk 1.131, restated, parity unpinned).
    records: [(input index, ID, attrs)] in input order.  Records with one ID are grouped by their
    attributes in first-seen order; the first distinct record of an ID keeps it (unless an earlier
    round took it), every further one gets ID.1, ID.2 ... (the first free suffix).  table[input]
    maps each input's original ID -> merged ID; out receives (merged ID, attrs).  -> collisions?"""
    by_id = {}
    for h, rid, attrs in records:
        by_id.setdefault(rid, {}).setdefault(_rec_key(attrs), (attrs, []))[1].append(h)
    collided = False
    for rid, variants in by_id.items():
        for attrs, heads in variants.values():
            if rid not in taken:
                new = rid
            else:
                collided = True
                k = 1
                while rid + b"." + str(k).encode() in taken:
                    k += 1
                new = rid + b"." + str(k).encode()
            taken.add(new)
            for h in heads:
                table.setdefault(h, {})[rid] = new
            out.append((new, attrs))
    return collided


def _no_duplicate_ids(headers, tag):
    for h in headers:
        ids = [rid for rid, _ in _header_records(h.text, tag)]
        if len(ids) != len(set(ids)):
            raise SAMException("Input file contains more than one %s with the same id"
                               % tag.decode().lstrip("@"))


def merge_read_groups(headers):
    """mergeReadGroups: -> (collisions?, {input: {old: new}}, [(ID, attrs)] sorted by ID)."""
    _no_duplicate_ids(headers, b"@RG")
    recs = [(h, rid, attrs) for h, hd in enumerate(headers) for rid, attrs in _header_records(hd.text, b"@RG")]
    table, out = {}, []
    col = merge_header_records(recs, set(), table, out)
    return col, table, sorted(out, key=lambda r: r[0])


def merge_program_groups(headers):
    """mergeProgramGroups: the PP (previous program) chains merged root first — the records
    without PP, then each round the records whose PP names a record of the same input merged in
    the round before — IDs and PPs translated between rounds.  -> (collisions?, {input: {old:
    new}} (no entry for an input without @PG), [(ID, attrs)] sorted by ID)."""
    _no_duplicate_ids(headers, b"@PG")
    left = [[h, rid, list(attrs)] for h, hd in enumerate(headers) for rid, attrs in _header_records(hd.text, b"@PG")]
    pp = lambda attrs: next((v for k, v in attrs if k == b"PP"), None)
    cur = [r for r in left if pp(r[2]) is None]
    left = [r for r in left if pp(r[2]) is not None]
    taken, table, result, col = set(), {}, [], False
    while cur:
        out = []
        col |= merge_header_records([(h, rid, a) for h, rid, a in cur], taken, table, out)
        result += out

        def tr(rs, pp_too):
            res = []
            for h, rid, attrs in rs:
                t = table.get(h, {})
                nid = t.get(rid, rid)
                a = attrs
                if pp_too and pp(attrs) is not None and t.get(pp(attrs)) not in (None, pp(attrs)):
                    a = [(k, t[v] if k == b"PP" else v) for k, v in attrs]
                res.append([h, nid, a])
            return res
        cur = tr(cur, False)
        left = tr(left, True)
        nxt, rest = [], []
        for r in left:
            if any(r[0] == c[0] and pp(r[2]) == c[1] for c in cur):
                nxt.append(r)
            else:
                rest.append(r)
        left, cur = rest, nxt
    if left:
        raise SAMException("%d program groups weren't processed. Do their PP ids point to existing PGs?" % len(left))
    return col, table, sorted(result, key=lambda r: r[0])


def merge_sequences(into, frm):
    """SamFileHeaderMerger.mergeSequences (htsjdk 1.131, restated from its published behaviour:
    parity unpinned).  Sequences of `frm` missing from `into` are held and inserted before the
    next sequence both share; one shared sequence earlier than a previous shared one cannot be
    placed: SAMException.  Entries are (name, length); an existing entry keeps its length."""
    result = list(into)
    names = [n for n, _ in result]
    holder, prevloc, prev = [], -1, None
    for rec in frm:
        loc = names.index(rec[0]) if rec[0] in names else -1
        if loc == -1:
            holder.append(rec)
        elif prevloc > loc:
            raise SAMException("Cannot merge sequence dictionaries because sequence %s and %s are in "
                               "different orders in two input sequence dictionaries."
                               % (rec[0].decode(errors="replace"), prev[0].decode(errors="replace")))
        else:
            result[loc:loc] = holder
            names[loc:loc] = [n for n, _ in holder]
            prevloc = loc + len(holder)
            prev = rec
            holder = []
    result += holder
    return result


def _same_dictionary(a, b):
    """SequenceUtil.assertSequenceListsEqual: same size, names, and lengths (0 = unknown)."""
    return len(a) == len(b) and all(x[0] == y[0] and (x[1] == y[1] or 0 in (x[1], y[1])) for x, y in zip(a, b))


class SamFileHeaderMerger:
    """new SamFileHeaderMerger(sortOrder, headers, true) as Utils.getSAMHeaderMerger builds it
    (cli/Utils.java:252-283).  htsjdk 1.131 is absent here, so its behaviour is restated (parity
    unpinned): the dictionary is merged only when the inputs' dictionaries differ
    (hasMergedSequenceDictionary), by mergeSequences over the inputs in order; read groups and
    program groups by mergeReadGroups / mergeProgramGroups (an ID carried by records with different
    attributes is renamed ID.1, ID.2, ...: hasReadGroupCollisions / hasProgramGroupCollisions, with
    per-input translation tables); the merged header holds the merged dictionary, the merged @RG and
    @PG records (sorted by ID) and the comments, sort order `sort_order`."""

    def __init__(self, sort_order, headers):
        self.headers = list(headers)
        dicts = [h.refs for h in self.headers]
        if all(_same_dictionary(dicts[0], d) for d in dicts[1:]):
            self.merged_refs = list(dicts[0])
            self.has_merged_sequence_dictionary = False
        else:
            m = []
            for d in dicts:
                m = merge_sequences(m, d)
            self.merged_refs = m
            self.has_merged_sequence_dictionary = True
        names = {n: i for i, (n, _) in enumerate(self.merged_refs)}
        # createSequenceMapping: input index -> merged index, by name
        self.ref_maps = [np.array([names[n] for n, _ in d], np.int32) for d in dicts]
        self.has_read_group_collisions, self.rg_tables, self.merged_rg = merge_read_groups(self.headers)
        self.has_program_group_collisions, self.pg_tables, self.merged_pg = merge_program_groups(self.headers)
        self.sort_order = sort_order

    def getProgramGroupId(self, input_index, original):
        """samProgramGroupIdTranslation.get(header).get(id): NullPointerException when the input
        has no @PG record (no table), None when the id is not one of its program groups."""
        t = self.pg_tables.get(input_index)
        if t is None:
            from .formats import NullPointerException
            raise NullPointerException("no program-group table for input %d" % input_index)
        return t.get(original)

    def getReadGroupId(self, input_index, original):
        return self.rg_tables.get(input_index, {}).get(original)

    def group_table(self, input_index):
        """hbam_rewrite_groups' table for one input: what correctSAMRecordForMerging does to its
        PG and RG tags (cli/Utils.java:314-324; both looked up in the PROGRAM-group table)."""
        import struct
        t = self.pg_tables.get(input_index)
        out = b""
        for collides in (self.has_program_group_collisions, self.has_read_group_collisions):
            if not collides:
                out += struct.pack("<BH", 0, 0)
            elif t is None:
                out += struct.pack("<BH", 2, 0)
            else:
                out += struct.pack("<BH", 1, len(t))
                for old, new in t.items():
                    out += struct.pack("<H", len(old)) + old + struct.pack("<h", len(new)) + new
        return out

    def getMergedHeader(self):
        from .output import SAMFileHeader
        lines = [b"@HD\tVN:1.4\tSO:" + self.sort_order.encode()]
        for n, ln in self.merged_refs:
            lines.append(b"@SQ\tSN:" + n + b"\tLN:" + str(ln).encode())
        for tag, recs in ((b"@RG", self.merged_rg), (b"@PG", self.merged_pg)):
            for rid, attrs in recs:
                lines.append(b"\t".join([tag, b"ID:" + rid] + [k + b":" + v for k, v in attrs]))
        for h in self.headers:
            lines += [ln for ln in h.text.split(b"\n") if ln.startswith(b"@CO")]
        return SAMFileHeader(b"\n".join(lines) + b"\n", self.merged_refs)


def correct_for_merging(ctx, cols, merger, input_index, raise_error=True):
    """SortRecordReader.nextKeyValue's Utils.correctSAMRecordForMerging over a decoded split
    (device hbam_columns, modified in place) of input `input_index` (hbam_merge_remap).  Returns
    the first record whose merged index lies outside its own dictionary (or None); raises there
    unless raise_error is False."""
    if not merger.has_merged_sequence_dictionary:
        return None
    m = np.ascontiguousarray(merger.ref_maps[input_index], np.int32)
    bad = C.c_uint64(0)
    rc = ctx.L.hbam_merge_remap(ctx.h, C.byref(cols), C.c_void_p(m.ctypes.data), len(m), C.byref(bad))
    if rc:
        raise RuntimeError("hbam_merge_remap failed (%d): %s" % (rc, ctx.last_error()))
    if bad.value == (1 << 64) - 1:
        return None
    if raise_error:
        _raise_refid(bad.value, input_index)
    return int(bad.value)


def _raise_refid(record, input_index):
    raise ValueError("Reference index not found in sequence dictionary (record %d of input %d: "
                     "SAMRecord.setReferenceIndex against the input's header)" % (record, input_index))


def correct_split(ctx, cols, merger, input_index):
    """Both halves of correctSAMRecordForMerging (cli/Utils.java:286-324) in the reference's
    per-record order: record r's dictionary step, then its group step.  When the dictionary step
    refuses record `bad`, the records before it still get their group rewrite, and an exception
    the group step raises at an earlier record is the one the job sees."""
    bad = correct_for_merging(ctx, cols, merger, input_index, raise_error=False)
    if bad is not None:
        cols.n_records = bad
    correct_groups(ctx, cols, merger, input_index)
    if bad is not None:
        _raise_refid(bad, input_index)


def correct_groups(ctx, cols, merger, input_index):
    """correctSAMRecordForMerging's program-group / read-group rewrite (cli/Utils.java:314-324)
    over a decoded split of input `input_index` (hbam_rewrite_groups: cols then points at the
    rewritten records).  Raises the reference's exception at the first record that raises it."""
    if not (merger.has_program_group_collisions or merger.has_read_group_collisions):
        return
    tab = merger.group_table(input_index)
    buf = np.frombuffer(tab, np.uint8)
    st, er = C.c_int32(0), C.c_uint64(0)
    rc = ctx.L.hbam_rewrite_groups(ctx.h, C.byref(cols), C.c_void_p(buf.ctypes.data), len(buf), C.byref(st),
                                   C.byref(er))
    if rc:
        raise RuntimeError("hbam_rewrite_groups failed (%d): %s" % (rc, ctx.last_error()))
    if st.value:
        from .formats import raise_for
        raise_for(st.value, "record %d of input %d (correctSAMRecordForMerging)" % (er.value, input_index))


def sort_inputs(ctx, inputs, ops=None, sort_order="coordinate"):
    """Sort.run over several BAM inputs on one GPU (Sort.java:84-188 with
    HEADERMERGER_INPUTS = every input, :111-113): each input decoded as one split, corrected for
    the merged header, sorted on the device; the runs, concatenated in input order, stably
    sorted once more.  Returns (merged header, SortedRun): the total order (key, input index,
    voffset) — the documented tie-break."""
    from .output import read_sam_header
    import torch
    ops = ops or HipSortOps(ctx)
    heads = [read_sam_header(d, ctx) for d in inputs]
    merger = SamFileHeaderMerger(sort_order, heads)
    runs = []
    for i, data in enumerate(inputs):
        h = ctx.parse_header(data)
        if not isinstance(h, dict):
            raise RuntimeError("cannot read the header of input %d (%d)" % (i, h))
        n = len(data) if not hasattr(data, "numel") else data.numel()
        rc, cols = ctx.decode_split_device(data, h["first_voffset"], (n << 16) | 0xffff, h["n_ref"])
        if rc or cols.status:
            raise RuntimeError("decode of input %d failed rc=%d status=%d: %s" % (i, rc, cols.status, ctx.last_error()))
        correct_split(ctx, cols, merger, i)
        runs.append(ops.run_from_columns(cols))
    if len(runs) == 1:
        return merger.getMergedHeader(), runs[0]
    nb = [int(r.offsets[-1]) if r.n else 0 for r in runs]
    keys = torch.cat([r.keys for r in runs])
    vo = torch.cat([r.voffset for r in runs])
    bs = torch.cat([r.block_size for r in runs])
    pay = torch.cat([r.payload[:b] for r, b in zip(runs, nb)])
    return merger.getMergedHeader(), ops.sort_received(keys, vo, bs, pay)
