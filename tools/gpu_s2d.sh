#!/bin/bash
# Two-stream slices A/B with the 8-wave LZ77 pass, then the bench line + rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so --slices 1 2 4 > $O/ab_slices.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/rp -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --parity-splits 0 > $O/bench_rp.json 2> $O/bench_rp.err
