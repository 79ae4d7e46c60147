#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam_a.so libhbam.so > gpurun_out/q/ab10.txt 2>&1
