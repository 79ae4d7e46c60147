#!/bin/bash
# After the shift fix: default and profiling builds on the 2 GB seed-3 file, the region profile,
# the parity suite and the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_inflate_kernel.py --size 2e9 --seed 3 --reps 1 --libs libhbam.so libhbam_prof.so > $O/ab2_seed3.txt 2>&1 &&
timeout -k 10 300 python -u tools/prof_regions.py inflate --size 2e9 > $O/inflate_regions.txt 2>&1 ;
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
