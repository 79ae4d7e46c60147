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
                        "--warmup", "1", "--no-cpu-baseline", "--parity-splits", "4"],
                       env=_env(HBAM_BENCH_BACKEND="gloo"), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "shard2"
    assert res["parity"]["mismatches"] == 0 and res["parity"]["splits"] == 4
    assert res["value"] > 0
