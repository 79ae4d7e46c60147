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
