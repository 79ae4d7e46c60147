#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gm
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "guess" > gpurun_out/gm/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/prof_regions.py guess --size 10e9 > gpurun_out/gm/guess.txt 2>&1 &&
timeout -k 10 400 python -u tools/bench_guess.py --size 10e9 --check 1000 --reps 3 > gpurun_out/gm/bg.json 2> gpurun_out/gm/bg.err
