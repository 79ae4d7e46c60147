#!/bin/bash
# Round-2 bench line + rocprofv3 kernel stats of the same command (profiles/r02/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/b
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > gpurun_out/b/bench.json 2> gpurun_out/b/bench.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/b/rp -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --parity-splits 0 > gpurun_out/b/bench_rp.json 2> gpurun_out/b/bench_rp.err
