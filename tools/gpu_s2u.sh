#!/bin/bash
# Final tree: smoke, bench line and rocprof kernel stats of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/rp -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --parity-splits 0 > $O/bench_rp.json 2> $O/bench_rp.err
