#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/m
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_output.py -x -v --timeout 120 --timeout-method thread > gpurun_out/m/out_tests.txt 2>&1; r=$?
[ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/m/tests.txt 2>&1; r=$?
[ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 300 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam_a.so libhbam.so > gpurun_out/m/ab10.txt 2>&1 &&
timeout -k 10 300 python -u tools/bench_deflate.py --size 1e9 --reps 2 > gpurun_out/m/deflate.json 2> gpurun_out/m/deflate.err
