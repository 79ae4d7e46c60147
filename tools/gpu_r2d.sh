#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/d
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/diag_guess.py guess_window_4197.bin guess_window_7433.bin > gpurun_out/d/diag.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/d/tests.txt 2>&1 ;
timeout -k 10 300 python -u tools/prof_regions.py inflate --size 2e9 > gpurun_out/d/inflate_prof.txt 2>&1 &&
timeout -k 10 300 python -u tools/profile_inflate.py --size 10e9 --reps 3 > gpurun_out/d/inflate10.txt 2>&1
