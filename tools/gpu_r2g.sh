#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g/tests.txt 2>&1; r=$?
[ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 400 python -u tools/bench_guess.py --size 10e9 --check 10000 --reps 3 > gpurun_out/g/bg.json 2> gpurun_out/g/bg.err
