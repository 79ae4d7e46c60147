#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/n
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_output.py -x -q --timeout 120 --timeout-method thread > gpurun_out/n/out_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/bench_deflate.py --size 1e9 --reps 2 > gpurun_out/n/deflate.json 2> gpurun_out/n/deflate.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/n/rp -o df --output-format csv -- python3 tools/bench_deflate.py --size 1e9 --reps 1 > gpurun_out/n/deflate_rp.json 2>&1 &&
timeout -k 10 200 python -u tools/prof_deflate.py > gpurun_out/n/prof.txt 2>&1
