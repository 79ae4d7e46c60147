#!/bin/bash
# Round-2 final evidence, part B: bench line, rocprof kernel stats of the same command,
# FETCH/WRITE passes of the decode kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fb
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > gpurun_out/fb/bench.json 2> gpurun_out/fb/bench.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/fb/rp -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --parity-splits 0 > gpurun_out/fb/bench_rp.json 2> gpurun_out/fb/bench_rp.err &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_inflate_tokens|k_decode_pools|k_resolve" -d gpurun_out/fb/fetch -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > gpurun_out/fb/fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_inflate_tokens|k_decode_pools|k_resolve" -d gpurun_out/fb/write -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > gpurun_out/fb/write.log 2>&1
