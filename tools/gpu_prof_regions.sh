#!/bin/bash
# Cycle-stamp breakdowns (libhbam_prof.so) + rocprof stats of the guesser.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pr
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prof_regions.py inflate --size 2e9 > gpurun_out/pr/inflate.txt 2>&1 &&
timeout -k 10 300 python -u tools/prof_regions.py guess --size 10e9 > gpurun_out/pr/guess.txt 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pr/rp -o guess -- python3 tools/bench_guess.py --size 10e9 --check 50 --reps 1 > gpurun_out/pr/bg.txt 2>&1
