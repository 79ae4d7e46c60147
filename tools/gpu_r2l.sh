#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/l
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/l/tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --slices 1 2 4 8 > gpurun_out/l/ab10.txt 2>&1
