"""Coordinate Sort plugin path (Sort.java:84-188).

CPU (gloo, world size 2): the exchange — split points, all_to_all by key range, local stable
sort — with the oracle's numpy sort as the local op; the concatenation over ranks must equal
the oracle's total order over the whole file (key, then voffset), payload bytes included.
GPU: hbam_sort_keys against numpy's stable argsort (negative keys, ties, unmapped-hash keys,
skipped passes), hbam_gather_records / hbam_permute, and the single-GPU decode -> sort path
against the oracle on the same files.
"""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_sorted(data):
    import oracle
    h = oracle.read_header(data)
    cols = oracle.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    pay, off = oracle.record_payloads(cols)
    o = oracle.sort_order(cols["key"])
    new_off, new_pay = oracle._regather(pay, off, o)
    return cols["key"][o], cols["voffset"].astype(np.int64)[o], new_pay, new_off, cols


def _sort_worker(rank, world, port, fname, out_q):
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import oracle
    from hadoop_bam import parallel, sort
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = np.fromfile(os.path.join(GOLDEN, fname), dtype=np.uint8)
    # byte-range shards: FileSplits [k*C/P, (k+1)*C/P) aligned by the guesser (a-8/a-10)
    b = np.array([len(data) * k // world for k in range(world)], np.uint64)
    e = np.array([len(data) * (k + 1) // world for k in range(world)], np.uint64)
    vs, ve = oracle.probabilistic_splits(data, b, e)
    cols = oracle.read_split(data, int(vs[rank]), int(ve[rank])) if rank < len(vs) else None
    if cols is not None and cols["n"]:
        pay, off = oracle.record_payloads(cols)
        run = oracle.CpuSortOps.run_from_arrays(cols["key"], cols["voffset"], cols["block_size"],
                                                pay, off)
    else:
        import torch
        run = sort.SortedRun(torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64),
                             torch.zeros(0, dtype=torch.int32), torch.zeros(0, dtype=torch.uint8),
                             torch.zeros(1, dtype=torch.int64))
    out = sort.sort_sharded(run, dist, oracle.CpuSortOps, parallel.torch_all_gather_fn(dist, "cpu"))
    out_q.put((rank, out.keys.numpy().tolist(), out.voffset.numpy().tolist(),
               out.payload.numpy().tobytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("fname", ["edge_unsorted_l1.bam", "small_pe.bam"])
def test_two_rank_sort_matches_total_order(oracle_mod, fname):
    import torch.multiprocessing as mp
    data = np.fromfile(os.path.join(GOLDEN, fname), dtype=np.uint8)
    want_k, want_v, want_p, _, _ = _oracle_sorted(data)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sort_worker, args=(r, 2, port, fname, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    keys = np.concatenate([np.array(r[1], np.int64) for r in res])
    vo = np.concatenate([np.array(r[2], np.int64) for r in res])
    pay = b"".join(r[3] for r in res)
    assert np.array_equal(keys, want_k)
    assert np.array_equal(vo, want_v)
    assert pay == want_p.tobytes()
    assert len(res[0][1]) > 0 and len(res[1][1]) > 0  # both partitions non-empty


def test_oracle_payload_is_record_bytes(oracle_mod):
    """record_payloads reproduces the inflated record stream byte for byte."""
    import zlib
    data = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)
    blocks = oracle_mod.scan_blocks(data)
    u = b"".join(zlib.decompressobj(-15).decompress(bytes(data[int(c) + 18:int(c) + int(l) - 8]))
                 for c, l in zip(blocks["coff"], blocks["clen"]))
    h = oracle_mod.read_header(data)
    cols = oracle_mod.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    pay, off = oracle_mod.record_payloads(cols)
    start = h["header_ulen"]
    assert pay.tobytes() == u[start:start + len(pay)]


# ---- GPU -------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("n,kind", [(0, "rand"), (1, "rand"), (4095, "rand"), (4097, "dups"),
                                    (300001, "rand"), (1 << 20, "coord"), (200000, "const")])
def test_device_radix_sort_is_stable_signed(gpu_ctx, n, kind):
    import torch
    from hadoop_bam import sort
    rng = np.random.default_rng(n + 7)
    if kind == "rand":
        k = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64)
    elif kind == "dups":
        k = rng.integers(-3, 3, n).astype(np.int64)
    elif kind == "coord":  # refID<<32 | pos, plus unmapped (0x7fffffff<<32 | hash) incl. negative
        ref = rng.integers(-1, 25, n).astype(np.int64)
        pos = rng.integers(-1, 250_000_000, n).astype(np.int64)
        k = (ref << 32) | (pos & 0xffffffff)
        um = rng.random(n) < 0.05
        h = rng.integers(-(1 << 31), 1 << 31, n).astype(np.int64)
        k[um] = (np.int64(0x7fffffff) << 32) | (h[um] & 0xffffffff)
        k[um & (h < 0)] = h[um & (h < 0)]  # sign-extended (BAMRecordReader.java:92-95)
    else:
        k = np.full(n, 42, np.int64)
    ops = sort.HipSortOps(gpu_ctx)
    d = torch.from_numpy(k).cuda()
    keys_s, perm = ops._sort(d.data_ptr(), n)
    want = np.argsort(k, kind="stable")
    assert np.array_equal(perm[:n].cpu().numpy().astype(np.int64), want)
    assert np.array_equal(keys_s.cpu().numpy(), k[want])


@pytest.mark.gpu
@pytest.mark.parametrize("fname", ["small_pe.bam", "edge_unsorted_l1.bam", "edge_uniform_long.bam"])
def test_single_gpu_decode_sort_matches_oracle(gpu_ctx, oracle_mod, fname):
    import torch
    from hadoop_bam import sort
    data = np.fromfile(os.path.join(GOLDEN, fname), dtype=np.uint8)
    want_k, want_v, want_p, want_off, cols = _oracle_sorted(data)
    d = torch.from_numpy(data).cuda()
    h = gpu_ctx.parse_header(d)
    rc, dc = gpu_ctx.decode_split_device(d, h["first_voffset"], (len(data) << 16) | 0xffff,
                                         h["n_ref"])
    assert rc == 0 and dc.status == 0 and dc.n_records == cols["n"]
    run = sort.HipSortOps(gpu_ctx).run_from_columns(dc)
    assert np.array_equal(run.keys.cpu().numpy(), want_k)
    assert np.array_equal(run.voffset.cpu().numpy(), want_v)
    assert np.array_equal(run.offsets.cpu().numpy(), want_off)
    assert run.payload.cpu().numpy().tobytes() == want_p.tobytes()


@pytest.mark.gpu
def test_sort_received_chunks_equals_global_order(gpu_ctx, oracle_mod):
    """The receive side of the exchange on the device: two source chunks (file order), each
    locally sorted, re-sorted stably == the oracle's total order."""
    import torch
    from hadoop_bam import sort
    data = np.fromfile(os.path.join(GOLDEN, "edge_unsorted_l1.bam"), dtype=np.uint8)
    want_k, want_v, want_p, _, cols = _oracle_sorted(data)
    pay, off = oracle_mod.record_payloads(cols)
    n = cols["n"]
    cut = n // 2
    parts = []
    for lo, hi in ((0, cut), (cut, n)):
        o = lo + oracle_mod.sort_order(cols["key"][lo:hi])
        no, npay = oracle_mod._regather(pay, off, o)
        parts.append((cols["key"][o], cols["voffset"].astype(np.int64)[o], cols["block_size"][o], npay))
    cat = lambda i, dt: torch.from_numpy(np.concatenate([p[i] for p in parts]).astype(dt)).cuda()
    out = sort.HipSortOps(gpu_ctx).sort_received(cat(0, np.int64), cat(1, np.int64),
                                                 cat(2, np.int32), cat(3, np.uint8))
    assert np.array_equal(out.keys.cpu().numpy(), want_k)
    assert np.array_equal(out.voffset.cpu().numpy(), want_v)
    assert out.payload.cpu().numpy().tobytes() == want_p.tobytes()


def _gpu_sort_worker(rank, world, port, fname, out_q):
    """One rank of the Sort plugin path on the product ops: device decode of its byte-range
    FileVirtualSplit, hbam_sort_split, partition + gloo exchange of host-staged buffers,
    hbam_sort_received.  Both ranks share cuda:0 (the pool's boxes have one GPU)."""
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist
    from hadoop_bam import _lib, parallel, sort
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = np.fromfile(os.path.join(GOLDEN, fname), dtype=np.uint8)
        ctx = _lib.Context(0)
        d = torch.from_numpy(data).cuda()
        h = ctx.parse_header(d)
        b = np.array([len(data) * k // world for k in range(world)], np.uint64)
        e = np.array([len(data) * (k + 1) // world for k in range(world)], np.uint64)
        n, vs, ve = ctx.probabilistic_splits(d, b, e)
        rc, cols = ctx.decode_split_device(d, int(vs[rank]), int(ve[rank]), h["n_ref"])
        assert rc == 0 and cols.status == 0
        ops = sort.HipSortOps(ctx)
        run = ops.run_from_columns(cols)
        out = sort.sort_sharded(run, dist, ops, parallel.torch_all_gather_fn(dist, "cpu"))
        out_q.put((rank, out.keys.cpu().numpy().tolist(), out.voffset.cpu().numpy().tolist(),
                   out.payload.cpu().numpy().tobytes(), [int(x) for x in vs], [int(x) for x in ve]))
    except Exception as ex:  # surfaced by the parent
        out_q.put((rank, "error", repr(ex), b"", [], []))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("fname", ["edge_unsorted_l1.bam", "small_pe.bam"])
def test_two_process_gpu_sort_matches_total_order(oracle_mod, fname):
    """Config #5's exchange on the product ops with two processes on the one GPU: the
    concatenation of both ranks' outputs equals the oracle's total order over the records of
    the two splits (boundary-block records read by both splits appear twice, as they do in the
    reference's map output).  The transport here is gloo over host memory; RCCL over xGMI is the
    same code path with the nccl backend and stays unmeasured on one-GPU boxes."""
    import torch.multiprocessing as mp
    data = np.fromfile(os.path.join(GOLDEN, fname), dtype=np.uint8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_sort_worker, args=(r, 2, port, fname, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r[2]
    vs, ve = res[0][4], res[0][5]
    # oracle: the records of both splits (as the two map tasks read them), in total order
    keys, vo, pay = [], [], []
    for a, z in zip(vs, ve):
        cols = oracle_mod.read_split(data, a, z)
        p_, off = oracle_mod.record_payloads(cols)
        for i in range(cols["n"]):
            keys.append(int(cols["key"][i]))
            vo.append(int(cols["voffset"][i]))
            pay.append(p_[off[i]:off[i + 1]].tobytes())
    o = np.argsort(np.array(keys, np.int64), kind="stable")
    assert np.array_equal(np.concatenate([np.array(r[1], np.int64) for r in res]),
                          np.array(keys, np.int64)[o])
    assert np.array_equal(np.concatenate([np.array(r[2], np.int64) for r in res]),
                          np.array(vo, np.int64)[o])
    assert b"".join(r[3] for r in res) == b"".join(pay[i] for i in o)
    assert len(res[0][1]) > 0 and len(res[1][1]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("fname", ["edge_unsorted_l1.bam", "small_pe.bam", "edge_uniform_long.bam"])
def test_rccl_exchange_one_rank_matches_oracle(gpu_ctx, oracle_mod, fname):
    """The exchange behind the C ABI (hbam_comm_init + hbam_comm_split_points +
    hbam_sort_exchange) on a one-rank RCCL communicator: the count all-gather and the grouped
    ncclSend/ncclRecv (to itself) of keys, voffsets, block sizes and payload, then the re-sort,
    equal the oracle's total order, payload bytes included.  (A box has one GPU; RCCL refuses two
    ranks on one device, so N > 1 runs only on the driver's 8-GPU node.)"""
    import torch
    from hadoop_bam import sort
    data = np.fromfile(os.path.join(GOLDEN, fname), dtype=np.uint8)
    want_k, want_v, want_p, want_off, cols = _oracle_sorted(data)
    d = torch.from_numpy(data).cuda()
    h = gpu_ctx.parse_header(d)
    rc, dc = gpu_ctx.decode_split_device(d, h["first_voffset"], (len(data) << 16) | 0xffff, h["n_ref"])
    assert rc == 0 and dc.status == 0
    comm = sort.RcclComm(gpu_ctx, 1, 0, sort.RcclComm.unique_id(gpu_ctx.L))
    try:
        ops = sort.HipSortOps(gpu_ctx, comm)
        # a run in FILE order (not key order), so the re-sort after the exchange does the work
        n = int(dc.n_records)
        pay, off = oracle_mod.record_payloads(cols)
        run = sort.SortedRun(torch.from_numpy(cols["key"].astype(np.int64)).cuda(),
                             torch.from_numpy(cols["voffset"].astype(np.int64)).cuda(),
                             torch.from_numpy(cols["block_size"].astype(np.int32)).cuda(),
                             torch.from_numpy(pay).cuda(), torch.from_numpy(off.astype(np.int64)).cuda())
        assert run.n == n
        sp = ops.split_points_native(run)
        assert len(sp) == 0
        out = ops.exchange_native(run, sp)
        assert gpu_ctx.timing()["exchange_ms"] > 0
        assert out.n == n
        assert np.array_equal(out.keys.cpu().numpy(), want_k)
        assert np.array_equal(out.voffset.cpu().numpy(), want_v)
        assert np.array_equal(out.offsets.cpu().numpy(), want_off)
        assert out.payload.cpu().numpy().tobytes() == want_p.tobytes()
        # sort_sharded drives the same native path when the ops carry a communicator
        out2 = sort.sort_sharded(ops.run_from_columns(dc), None, ops, None)
        assert np.array_equal(out2.keys.cpu().numpy(), want_k)
        assert out2.payload.cpu().numpy().tobytes() == want_p.tobytes()
        # the exchange proper without its size query is refused
        from hadoop_bam._lib import SortedRunC
        import ctypes as C
        r = ops._run_struct(run)
        o = SortedRunC(out.n, int(out.offsets[-1]), out.keys.data_ptr(), out.voffset.data_ptr(),
                       out.block_size.data_ptr(), out.offsets.data_ptr(), out.payload.data_ptr())
        z = np.zeros(1, np.int64)
        assert gpu_ctx.L.hbam_sort_exchange(gpu_ctx.h, comm.h, C.byref(r), C.c_void_p(z.ctypes.data),
                                            C.byref(o)) == -11
    finally:
        comm.close()


@pytest.mark.gpu
def test_sort_gather_and_exchange_above_2gib(gpu_ctx, oracle_mod):
    """A sorted run whose payload offsets pass 2^31 (the regime of the round-5 readlane fault in
    k_gather_records_tile: a 64-bit destination offset above 2^31 sign-extended) and its one-rank
    RCCL exchange, whose payload goes out in several HBAM_XCHG_CHUNK (1 GiB) pieces.  Checked
    against the oracle: keys in its total order, every payload offset, the payload of ~3,000
    records (all of the last 1,000, where offsets exceed 2^31) byte for byte against the
    oracle's record bytes, and a byte-sum over the whole payload; the exchange must hand back the
    identical run."""
    import torch
    import genbam
    from hadoop_bam import sort
    data = np.asarray(genbam.generate(target_bytes=int(1.05e9), seed=11, sorted=0, threads=16))
    cols = oracle_mod.read_split(data, oracle_mod.read_header(data)["first_voffset"],
                                 (len(data) << 16) | 0xffff)
    assert cols["status"] == 0
    n = cols["n"]
    o = oracle_mod.sort_order(cols["key"])
    d = torch.from_numpy(data).cuda()
    h = gpu_ctx.parse_header(d)
    rc, dc = gpu_ctx.decode_split_device(d, h["first_voffset"], (len(data) << 16) | 0xffff, h["n_ref"])
    assert rc == 0 and dc.status == 0 and int(dc.n_records) == n
    ops = sort.HipSortOps(gpu_ctx)
    run = ops.run_from_columns(dc)
    assert np.array_equal(run.keys.cpu().numpy(), cols["key"][o])
    want_v = cols["voffset"].astype(np.int64)[o]
    assert np.array_equal(run.voffset.cpu().numpy(), want_v)
    lens = 4 + cols["block_size"].astype(np.int64)[o]
    off = run.offsets.cpu().numpy()
    assert off[0] == 0 and np.array_equal(np.diff(off), lens)
    assert off[-1] > (1 << 31) + (1 << 28), "payload must pass 2^31 well before its end"
    pay = run.payload.cpu().numpy()
    vo = cols["var_off"].astype(np.int64)
    assert int(pay.sum(dtype=np.uint64)) == int(
        cols["var"].sum(dtype=np.uint64) + oracle_mod.record_fixed_bytes(cols, np.arange(n)).sum(dtype=np.uint64))
    rng = np.random.default_rng(5)
    pick = np.unique(np.concatenate([rng.integers(0, n, 2000), np.arange(n - 1000, n)]))
    fixed = oracle_mod.record_fixed_bytes(cols, o[pick])
    for k, i in enumerate(pick):
        j = int(o[i])
        rec = pay[int(off[i]):int(off[i + 1])]
        assert rec[:36].tobytes() == fixed[k].tobytes(), i
        assert rec[36:].tobytes() == cols["var"][vo[j]:vo[j + 1]].tobytes(), i
    comm = sort.RcclComm(gpu_ctx, 1, 0, sort.RcclComm.unique_id(gpu_ctx.L))
    try:
        ops2 = sort.HipSortOps(gpu_ctx, comm)
        out = ops2.exchange_native(run, ops2.split_points_native(run))
        assert out.n == n
        assert torch.equal(out.keys, run.keys) and torch.equal(out.voffset, run.voffset)
        assert torch.equal(out.offsets, run.offsets)
        assert torch.equal(out.payload[:int(off[-1])], run.payload[:int(off[-1])])
    finally:
        comm.close()


@pytest.mark.gpu
def test_sort_received_after_async_device_op(gpu_ctx, oracle_mod):
    """sort_received's inputs produced by asynchronous torch work (pinned non_blocking copies
    and kernels still queued on torch's stream) must be complete before libhbam's own stream
    reads them (the size query ran before any sync)."""
    import torch
    from hadoop_bam import sort
    data = np.fromfile(os.path.join(GOLDEN, "edge_unsorted_l1.bam"), dtype=np.uint8)
    want_k, want_v, want_p, _, cols = _oracle_sorted(data)
    pay, off = oracle_mod.record_payloads(cols)

    def dev(a, dt):
        h = torch.from_numpy(np.ascontiguousarray(a).astype(dt)).pin_memory()
        x = h.cuda(non_blocking=True)
        for _ in range(20):  # queue work behind the copy on torch's stream
            x = x.flip(0).flip(0)
        return x

    out = sort.HipSortOps(gpu_ctx).sort_received(dev(cols["key"], np.int64),
                                                 dev(cols["voffset"].astype(np.int64), np.int64),
                                                 dev(cols["block_size"], np.int32), dev(pay, np.uint8))
    assert np.array_equal(out.keys.cpu().numpy(), want_k)
    assert np.array_equal(out.voffset.cpu().numpy(), want_v)
    assert out.payload.cpu().numpy().tobytes() == want_p.tobytes()


# ---- several inputs: header merge + correctSAMRecordForMerging (Sort.java:111-113, 279-295) ----
def _dicts():
    a = [(b"c%d" % i, 100 * i) for i in range(1, 6)]
    return a


def test_header_merger_matches_oracle_restatement():
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    import oracle
    from hadoop_bam.output import SAMFileHeader
    from hadoop_bam.sort import SamFileHeaderMerger, SAMException
    a = _dicts()
    cases = [
        [a, a],                                   # equal: no merge
        [a, a[1:] + [(b"x", 7)]],                 # shifted + appended
        [a[2:], a],                               # prefix missing in the first
        [a[:2] + [(b"y", 3)] + a[2:], a],         # an extra in the middle
        [a, [(b"z", 1)], a[:1]],                  # disjoint input
        [a, [(b"c1", 100), (b"c2", 0)] + a[2:]],  # a length 0 = unknown: still equal
    ]
    for ds in cases:
        hs = [SAMFileHeader(b"@HD\tVN:1.4\n", d) for d in ds]
        m = SamFileHeaderMerger("coordinate", hs)
        want, merged = oracle.merged_dictionary(ds)
        assert (m.merged_refs, m.has_merged_sequence_dictionary) == (want, merged), ds
        for d, mp in zip(ds, m.ref_maps):
            assert [m.merged_refs[i][0] for i in mp] == [n for n, _ in d]
        mh = m.getMergedHeader()
        assert mh.refs == want and b"SO:coordinate" in mh.text.split(b"\n")[0]
    # a shared pair in opposite orders cannot be merged
    bad = [a, [a[3], a[1]]]
    with pytest.raises(SAMException):
        SamFileHeaderMerger("coordinate", [SAMFileHeader(b"", d) for d in bad])
    with pytest.raises(ValueError):
        oracle.merged_dictionary(bad)


_GROUP_HEADERS = [
    # identical groups: nothing renamed
    [b"@RG\tID:g1\tSM:s1\n@PG\tID:p\tPN:x\n", b"@RG\tID:g1\tSM:s1\n@PG\tID:p\tPN:x\n"],
    # RG and PG collisions, a PP chain whose root is renamed (so its child differs too)
    [b"@RG\tID:g1\tSM:s1\n@PG\tID:bwa\tPN:bwa\n@PG\tID:gatk\tPN:gatk\tPP:bwa\n",
     b"@RG\tID:g1\tSM:other\n@RG\tID:g2\tSM:s2\n@PG\tID:bwa\tPN:bwa\tVN:2\n@PG\tID:gatk\tPN:gatk\tPP:bwa\n"],
    # three inputs, a taken suffix (g1.1 exists already), an input without @PG
    [b"@RG\tID:g1\tSM:a\n@RG\tID:g1.1\tSM:z\n@PG\tID:p\tPN:x\n", b"@RG\tID:g1\tSM:b\n",
     b"@RG\tID:g1\tSM:c\n@PG\tID:p\tPN:y\n@PG\tID:q\tPN:q\tPP:p\n@PG\tID:r\tPN:r\tPP:q\n"],
    # a chain in one input only, PG ids shared by unrelated records
    [b"@PG\tID:a\tPN:1\n@PG\tID:b\tPN:2\tPP:a\n", b"@PG\tID:b\tPN:2\n@PG\tID:a\tPN:3\tPP:b\n"],
]


@pytest.mark.parametrize("case", range(len(_GROUP_HEADERS)))
def test_header_merger_groups_match_oracle(case):
    """SamFileHeaderMerger's read-/program-group merge (mergeReadGroups / mergeProgramGroups:
    collisions renamed ID.1, ID.2 ..., PP chains merged root first) against the oracle's
    independent restatement (both parity unpinned: htsjdk 1.131 is absent)."""
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    import oracle
    from hadoop_bam.output import SAMFileHeader
    from hadoop_bam.sort import SamFileHeaderMerger
    texts = _GROUP_HEADERS[case]
    m = SamFileHeaderMerger("coordinate", [SAMFileHeader(t, _dicts()) for t in texts])
    want = oracle.header_groups(texts)
    assert m.has_read_group_collisions == want["rg_collisions"]
    assert m.has_program_group_collisions == want["pg_collisions"]
    assert m.rg_tables == want["rg"] and m.pg_tables == want["pg"]
    mh = m.getMergedHeader().text
    for i, t in enumerate(texts):  # every input's renamed ids are in the merged header
        for rid, new in list(m.rg_tables.get(i, {}).items()) + list(m.pg_tables.get(i, {}).items()):
            assert (b"\tID:" + new + b"\t") in mh or mh.count(b"ID:" + new + b"\n")
    if case == 1:
        assert m.pg_tables[1] == {b"bwa": b"bwa.1", b"gatk": b"gatk.1"}
        assert b"@PG\tID:gatk.1\tPN:gatk\tPP:bwa.1" in mh
    if case == 2:
        # ids are taken in processing order (idsThatAreAlreadyTaken grows as records merge), so
        # input 1 gets g1.1 and input 0's own g1.1 record, processed after, becomes g1.1.1
        assert m.rg_tables[1] == {b"g1": b"g1.1"} and m.rg_tables[0][b"g1.1"] == b"g1.1.1"
        assert 1 not in m.pg_tables


@pytest.mark.gpu
def test_multi_input_sort_matches_oracle(tmp_path):
    """Two inputs with different dictionaries (the second: a new first sequence, then the
    first's dictionary without its last sequence; the same records): the first input's refIDs
    move up by one in the merged dictionary.  Device decode + hbam_merge_remap + sort equals
    the oracle's (key, input, voffset) order over the corrected records (every record ties with
    its copy in the other input), payload bytes included; the merged BAM written through
    merge_sam_into carries the merged dictionary and reads back through the oracle in that
    order."""
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    import oracle
    from helpers import redictionary_bam
    from hadoop_bam import _lib
    from hadoop_bam.sort import sort_inputs
    from hadoop_bam.output import BAMRecordWriter, merge_sam_into
    a = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)
    b, refs_a, refs_b = redictionary_bam(a)
    ctx = _lib.Context(0)
    header, run = sort_inputs(ctx, [a, b])
    keys, pay, off, merged = oracle.sort_merged([a, b])
    assert header.refs == merged == [(b"chrNEW", 5000)] + refs_a
    assert run.n == len(keys) > 20000
    assert np.array_equal(run.keys.cpu().numpy(), keys)
    assert np.array_equal(run.offsets.cpu().numpy(), off)
    assert np.array_equal(run.payload.cpu().numpy()[:len(pay)], pay)
    # Utils.mergeSAMInto with the merged header
    part = tmp_path / "sorted-000000"
    with open(part, "wb") as f:
        w = BAMRecordWriter(f, header, write_header=False, ctx=ctx)
        w.write_device(run.payload, int(run.offsets[-1]))
        w.close()
    out = tmp_path / "out.bam"
    merge_sam_into(str(out), str(tmp_path), "", "", header, "sorted", ctx=ctx)
    data = np.fromfile(out, np.uint8)
    assert oracle.bam_dictionary(data) == merged
    h = oracle.read_header(data)
    back = oracle.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    bp, bo = oracle.record_payloads(back)
    assert back["n"] == len(keys) and np.array_equal(bp, pay)


@pytest.mark.gpu
def test_multi_input_sort_index_outside_input_dictionary():
    """With 25 new sequences merged in front, the first input's chr1 records map to index 25,
    beyond its own 25-sequence dictionary: SAMRecord.setReferenceIndex raises
    IllegalArgumentException in the reference; the device path reports it and the oracle
    agrees."""
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    import oracle
    from helpers import redictionary_bam
    from hadoop_bam import _lib
    from hadoop_bam.sort import sort_inputs
    a = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)
    b, _, _ = redictionary_bam(a, prepend=[(b"n%02d" % i, 1000) for i in range(25)], drop_last=0)
    with pytest.raises(ValueError):
        oracle.sort_merged([a, b])
    with pytest.raises(ValueError, match="input 0"):
        sort_inputs(_lib.Context(0), [a, b])


def _group_inputs(kind):
    """small_pe.bam and a second input whose @RG / @PG records collide with it (kind: "mixed" —
    RG values rewritten to a PG id, to an unknown id, dropped; "no_pg" — no @PG line in the second
    header; "non_string" — one record's RG typed 'A')."""
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    from helpers import regroup_bam
    a = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)

    def text(t):
        t = t.replace(b"SM:sample1", b"SM:sampleB").replace(b"PN:gen_bam\tVN:1", b"PN:gen_bam\tVN:2")
        if kind == "no_pg":
            t = b"".join(ln + b"\n" for ln in t.split(b"\n") if ln and not ln.startswith(b"@PG"))
        return t

    def rg(i, v):
        if kind == "mixed":
            return b"gen_bam" if i % 3 == 1 else b"zzz" if i % 5 == 2 else None if i % 7 == 3 else v
        if kind == "non_string" and i == 11:
            return (b"A", b"x")
        return v
    return a, regroup_bam(a, text, rg)


@pytest.mark.gpu
def test_multi_input_sort_group_collisions_match_oracle():
    """Colliding @RG and @PG records: every record carrying RG / PG is rewritten through the
    program-group table (cli/Utils.java:314-324; RG values that are not PG ids are removed, an RG
    value naming a PG id takes its merged id) and re-encoded, on the device (hbam_rewrite_groups);
    the sorted output equals the oracle's records byte for byte."""
    import oracle
    from hadoop_bam import _lib
    from hadoop_bam.sort import sort_inputs
    a, b = _group_inputs("mixed")
    header, run = sort_inputs(_lib.Context(0), [a, b])
    keys, pay, off, merged = oracle.sort_merged([a, b])
    assert b"@RG\tID:grp1.1\tSM:sampleB" in header.text and b"@PG\tID:gen_bam.1" in header.text
    assert run.n == len(keys)
    assert np.array_equal(run.keys.cpu().numpy(), keys)
    assert np.array_equal(run.offsets.cpu().numpy(), off)
    assert np.array_equal(run.payload.cpu().numpy()[:len(pay)], pay)
    # the quirk is visible: input 1's RG:gen_bam records now carry RG:gen_bam.1, and no record
    # carries RG:grp1 (not a program-group id: removed)
    assert pay.tobytes().count(b"RGZgen_bam.1\0") > 1000 and pay.tobytes().count(b"RGZgrp1\0") == 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind,exc", [("no_pg", "NullPointerException"), ("non_string", "ClassCastException")])
def test_multi_input_sort_group_rewrite_exceptions(kind, exc):
    """Where the reference's map task throws: an input without a program-group table meets a
    record carrying RG (NullPointerException), an RG that is not a string (ClassCastException);
    the oracle raises at the same record."""
    import oracle
    from hadoop_bam import _lib, formats
    from hadoop_bam.sort import sort_inputs
    a, b = _group_inputs(kind)
    with pytest.raises(oracle.GroupRewriteError) as ei:
        oracle.sort_merged([a, b])
    assert ei.value.kind == exc
    with pytest.raises(getattr(formats, exc), match="record %d of input 1" % ei.value.record):
        sort_inputs(_lib.Context(0), [a, b])


def _dictionary_and_group_inputs(bad_from, cce_at):
    """Input 0: small_pe.bam with records [bad_from, ...) moved to the last sequence and a
    non-string RG at record cce_at; input 1: the same records under one more (new, first)
    sequence and colliding @RG / @PG headers.  Merged, input 0's records from bad_from map past
    its own dictionary (IllegalArgumentException) and record cce_at's RG raises
    ClassCastException in the group step (cli/Utils.java:286-324)."""
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    from helpers import redictionary_bam, regroup_bam
    a = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)
    base = regroup_bam(a, lambda t: t, lambda i, v: v, ref_fn=lambda i, r: 24 if i >= bad_from else r)
    a0 = regroup_bam(base, lambda t: t, lambda i, v: (b"A", b"x") if i == cce_at else v)
    b, _, _ = redictionary_bam(base, prepend=[(b"chrNEW", 5000)], drop_last=0)
    b = regroup_bam(b, lambda t: t.replace(b"SM:sample1", b"SM:sampleB").replace(b"PN:gen_bam\tVN:1", b"PN:gen_bam\tVN:2"),
                    lambda i, v: v)
    return a0, b


@pytest.mark.parametrize("cce_at,first", [(11, "group"), (15000, "dictionary")])
def test_oracle_dictionary_and_group_errors_in_record_order(cce_at, first):
    """correctSAMRecordForMerging runs per record: with a dictionary error at record 10000 and a
    group error at cce_at, the earlier record's exception is the job's."""
    import oracle
    a0, b = _dictionary_and_group_inputs(10000, cce_at)
    if first == "group":
        with pytest.raises(oracle.GroupRewriteError) as ei:
            oracle.sort_merged([a0, b])
        assert ei.value.kind == "ClassCastException" and ei.value.record == cce_at
    else:
        with pytest.raises(ValueError, match="input 0 record 10000"):
            oracle.sort_merged([a0, b])


@pytest.mark.gpu
@pytest.mark.parametrize("cce_at,first", [(11, "group"), (15000, "dictionary")])
def test_multi_input_sort_dictionary_and_group_errors(cce_at, first):
    """The device path (hbam_merge_remap, then hbam_rewrite_groups over the records before the
    refused one) raises the exception of the earlier record, as the oracle does."""
    from hadoop_bam import _lib, formats
    from hadoop_bam.sort import sort_inputs
    a0, b = _dictionary_and_group_inputs(10000, cce_at)
    if first == "group":
        with pytest.raises(formats.ClassCastException, match="record %d of input 0" % cce_at):
            sort_inputs(_lib.Context(0), [a0, b])
    else:
        with pytest.raises(ValueError, match="record 10000 of input 0"):
            sort_inputs(_lib.Context(0), [a0, b])


_SORT_LEG_NCCL = r"""
import json, os, sys
root = sys.argv[1]
sys.path[:0] = [os.path.join(root, d) for d in ("hadoop-bam_amd", "tools", "oracle", "")]
import torch, torch.distributed as dist
import bench, sort_leg
from hadoop_bam import _lib
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
try:
    ctx = _lib.Context(0)
    x = torch.ones(4, device=dev)
    dist.all_reduce(x)  # torch's communicator before libhbam's exists
    res = sort_leg.run(ctx, dist, 0, 1, 0.15e9, 5, 8, dev, dev, bench.N_REF, steps=1, samples=64,
                       log=lambda *a: None)
    dist.all_reduce(x)  # and after libhbam's was created, used and closed
    res["torch_all_reduce"] = float(x[0])
    print(json.dumps(res))
finally:
    dist.destroy_process_group()
"""


@pytest.mark.gpu
def test_sort_leg_on_nccl_torch_and_libhbam_communicators_together(tmp_path):
    """bench.py's N > 1 Sort leg (tools/sort_leg.py) on the nccl backend, world size 1: torch's
    ProcessGroupNCCL (all_gather, broadcast of the unique id, barriers, all_reduce) and
    libhbam's own RCCL communicator (hbam_comm_split_points, hbam_sort_exchange) live in one
    process on one device, as on every rank of the driver's multi-GPU run (which this one-GPU
    pool cannot rehearse with two ranks: RCCL refuses two ranks on one device).  The leg's own
    parity (order, permutation with each record's payload, oracle sample) must be clean."""
    import json
    import subprocess
    script = tmp_path / "sort_leg_nccl.py"
    script.write_text(_SORT_LEG_NCCL)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, str(script), ROOT], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["transport"].startswith("hbam_sort_exchange"), res
    assert res["parity"]["mismatches"] == 0, res
    assert res["parity"]["permutation_with_own_payload"] and res["parity"]["order_key_voffset_every_rank"]
    assert res["records"] > 0 and res["parity"]["oracle_sample"]["records"] > 0
    assert res["stages_ms_max_over_ranks"]["exchange_rccl"] > 0
    assert res["torch_all_reduce"] == 1.0
