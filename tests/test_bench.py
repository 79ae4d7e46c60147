"""bench.py's launch contract (the driver's `python bench.py --gpus N`): without a launcher it
starts N rank processes itself; with one, WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(kw)
    return e


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=_env(WORLD_SIZE="2", RANK="0"),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE 2" in r.stderr


@pytest.mark.gpu
def test_bench_spawns_two_ranks_gloo():
    """`bench.py --gpus 2` with no launcher: two ranks (gloo rehearsal, both on the one GPU of the
    pool's box), one JSON line with n_gpus 2, every parity split bit-exact."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--size", "2e8", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--parity-splits", "4", "--sort-size", "2e8"],
                       env=_env(HBAM_BENCH_BACKEND="gloo"), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "shard2"
    assert res["parity"]["mismatches"] == 0 and res["parity"]["splits"] == 4
    assert res["value"] > 0
    # every record of each rank's timed launch against the oracle
    assert len(res["parity"]["whole_launch"]) == 2
    for w in res["parity"]["whole_launch"]:
        assert w["mismatches"] == 0 and w["records_checked"] == w["shard_records"] > 0, w
    # config #5's leg across the ranks (tools/sort_leg.py), here over the host-staged gloo exchange
    srt = res["sort"]
    assert srt["parity"]["mismatches"] == 0, srt
    assert srt["parity"]["records_out"] == srt["parity"]["records_decoded"] > 100000
    assert srt["parity"]["oracle_sample"]["records"] > 0 and srt["records_per_s"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("gpus,extra", [(1, ["--c4-window", "2.5e8"]), (2, [])])
def test_bench_config4_windows(gpus, extra):
    """`bench.py --config4` (BASELINE config #4: one file sharded over the ranks, strong scaling) at a
    small total: several windows per step at N=1, two gloo ranks at N=2; every record of every window
    equals the body's resident decode, the body decode equals the oracle, the record count adds up."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--config4", "--c4-total", "8e8",
                        "--c4-body", "2e8", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
                        "--parity-splits", "2"] + extra,
                       env=_env(HBAM_BENCH_BACKEND="gloo"), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == gpus and res["scaling"] == "strong"
    p = res["parity"]
    assert p["mismatches"] == 0 and p["record_count_matches"], p
    assert p["records_checked_vs_body_decode"] == res["config"]["records_all_gpus"]
    if gpus == 1:
        assert res["config"]["windows_per_step_rank0"] > 1


def test_sort_leg_budget_from_the_whole_run_deadline():
    """The Sort leg's watchdog counts from process start (--deadline), not from the leg's start,
    so a hung exchange ends while the driver's own limit still leaves time to print the line."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.sort_leg_budget(420.0, 100.0) == 320.0
    assert bench.sort_leg_budget(420.0, 420.0 - bench.SORT_LEG_MIN_S) == bench.SORT_LEG_MIN_S
    assert bench.sort_leg_budget(420.0, 400.0) == 0.0  # too little left: the leg is skipped
    assert bench.sort_leg_budget(420.0, 500.0) == 0.0


_HANG = r"""
import json, sys, time, types
sys.path.insert(0, %r)
import bench
bench.SORT_LEG_MIN_S = 0.5
fake = types.ModuleType("sort_leg")
fake.run = lambda *a, **k: time.sleep(600)  # an exchange that never returns
sys.modules["sort_leg"] = fake
args = types.SimpleNamespace(deadline=time.time() - bench.T_START + 1.5, sort_size=1, seed=0, sort_steps=1)
res = {"value": 1.0}
bench.guarded_sort_leg(None, None, 0, 2, args, 1, None, None, res)
print("not reached")
"""


def test_sort_leg_watchdog_prints_the_line_and_exits_nonzero():
    """A hung Sort leg: rank 0 prints the headline line carrying the leg's timeout, and the
    process exits with WATCHDOG_EXIT (3), so launchers see the failure."""
    r = subprocess.run([sys.executable, "-c", _HANG % ROOT], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout
    res = json.loads(lines[0])
    assert res["value"] == 1.0 and "timeout" in res["sort"]["error"]


def test_cpu_baseline_builds_the_same_pools_as_the_oracle_reader():
    """bench.py's cpu_baseline does the device decode's whole work on host cores: every record of
    its FileVirtualSplits with the lazy getters' pools built (or_read_split_pools), the same
    records and pool bytes as oracle.read_split + oracle.pools over those splits."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for d in ("oracle", "tools", ""):
        sys.path.insert(0, os.path.join(root, d))
    import numpy as np
    import bench
    import genbam
    import oracle
    data = np.frombuffer(genbam.generate(records=20000, seed=11, odd_every=53), np.uint8)
    r = bench.cpu_baseline(data, 0.02, 3)
    assert r["status"] == [0] and r["kind"] == "port"
    sample = int(min(len(data), 0.02 * 3 * 0.06e9))
    block = int(np.ceil(sample / 3))
    begs = list(range(0, sample, block))
    ends = [min(b + block, sample) for b in begs]
    base = np.ascontiguousarray(data[:sample + (1 << 20) if sample < len(data) else len(data)])
    vs, ve = oracle.probabilistic_splits(base, np.array(begs, np.uint64), np.array(ends, np.uint64))
    n = pb = 0
    for a, b in zip(vs, ve):
        c = oracle.read_split(base, int(a), int(b))
        p = oracle.pools(c)
        n += c["n"]
        pb += sum(len(p[k]) * p[k].itemsize for k in ("names", "cigars", "seq", "qual", "aux"))
    assert n > 0 and r["records_per_s"] > 0
    assert r["pool_bytes"] == pb
    assert ("%d records" % n) in r["sample"]


def test_issue_roofline_reads_the_committed_sq_pass():
    """bench.py's roofline carries the instruction-issue view of the Huffman pass from the
    committed SQ counter pass (profiles/r06/closing/pmc_sq_3g.json)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    r = bench.issue_roofline("k_inflate_tokens")
    assert r is not None and r["waves_per_simd"] == 2
    assert 0.0 < r["simd_valu_pipe_frac"] <= 1.0 and 0.0 < r["wave_issue_frac"] <= 1.0
    assert abs(r["wave_issue_frac"] + r["wait_frac"] + r["dependency_stall_frac"] - 1.0) < 0.02
    assert bench.issue_roofline("k_no_such_kernel") is None
