#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/i
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/i/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 3 --libs libhbam_a.so libhbam.so > gpurun_out/i/ab10.txt 2>&1 &&
timeout -k 10 300 python -u tools/profile_inflate.py --size 2e9 --reps 2 --prof > gpurun_out/i/prof2g.txt 2>&1
