"""N>1 path on CPU: two gloo ranks shard one BAM file's FileSplits, all-gather their guesses
and reproduce BAMInputFormat.addProbabilisticSplits exactly (incl. empty-split merges across
the rank boundary).  The guesser/decoder stand-in here is the CPU oracle (test code only);
on the GPU box the sharded decode runs with the device guesser in
tests/test_gpu_parity.py::test_sharded_split_windows_match_oracle, the two-process device Sort in
tests/test_sort.py::test_two_process_gpu_sort_matches_total_order, and bench.py --gpus 2 in
tests/test_bench.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, split_size, out_q):
    sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle")]
    import oracle
    from hadoop_bam import parallel
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)
    n_ref = oracle.read_header(data)["n_ref"]

    def guess_fn(b, e):
        return [oracle.guess_bam_record_start(data, int(x), int(y), n_ref)[0] for x, y in zip(b, e)]

    mine_vs, mine_ve, (vs, ve) = parallel.sharded_virtual_splits(
        len(data), split_size, rank, world, guess_fn, parallel.torch_all_gather_fn(dist, "cpu"))
    n = 0
    for a, z in zip(mine_vs, mine_ve):
        n += oracle.read_split(data, int(a), int(z), keep_var=False)["n"]
    import torch
    t = torch.tensor([n], dtype=torch.int64)
    dist.all_reduce(t)
    out_q.put((rank, [int(x) for x in vs], [int(x) for x in ve], int(t.item()),
               [int(x) for x in mine_vs]))
    dist.destroy_process_group()


@pytest.mark.parametrize("split_size", [256 << 10, 40 << 10])
def test_two_rank_sharding_matches_reference_splits(oracle_mod, split_size):
    data = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)
    b, e = oracle_mod.file_splits(len(data), split_size)
    want_vs, want_ve = oracle_mod.probabilistic_splits(data, b, e)
    want_n = sum(oracle_mod.read_split(data, int(x), int(y), keep_var=False)["n"]
                 for x, y in zip(want_vs, want_ve))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, split_size, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, vs, ve, total, mine in res:
        assert vs == [int(x) for x in want_vs] and ve == [int(x) for x in want_ve]
        assert total == want_n
    # the ranks' own splits partition the global list
    assert sorted(res[0][4] + res[1][4]) == sorted(int(x) for x in want_vs)


def test_merge_rule_empty_split_extends_previous():
    from hadoop_bam import parallel
    beg = np.array([0, 100, 200], np.int64)
    end = np.array([100, 200, 300], np.int64)
    vs, ve, own = parallel.merge_guesses(beg, end, np.array([5 << 16, 200, 210 << 16]))
    assert list(vs) == [5 << 16, 210 << 16]
    assert list(ve) == [(200 << 16) | 0xffff, (300 << 16) | 0xffff]
    with pytest.raises(IOError):
        parallel.merge_guesses(beg, end, np.array([100, 200, 300]))
