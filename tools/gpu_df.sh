#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/df
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_output.py -x -v --timeout 120 --timeout-method thread > gpurun_out/df/tests.txt 2>&1; r=$?
[ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 300 python -u tools/bench_deflate.py --size 1e9 --reps 2 > gpurun_out/df/bench.json 2> gpurun_out/df/bench.err
