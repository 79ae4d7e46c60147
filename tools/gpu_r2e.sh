#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }   # pass or test failure: the GPU is fine
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e/tests.txt 2>&1; r=$?
ok $r || exit $r
timeout -k 10 300 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 3 --libs libhbam_a.so libhbam.so > gpurun_out/e/ab10.txt 2>&1 &&
timeout -k 10 300 python -u tools/prof_regions.py inflate --size 2e9 > gpurun_out/e/inflate_prof.txt 2>&1 &&
bash tools/pmc_inst.sh 2e9 gpurun_out/e/pmc_inst &&
timeout -k 10 400 python -u tools/diag_guess.py --batch 4197 7433 > gpurun_out/e/diag_batch.txt 2>&1
