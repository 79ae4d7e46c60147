#!/bin/bash
# A/B of the LZ77 pass builds at 10 GB, then the remaining consumer tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam_a.so libhbam_b.so libhbam_c.so libhbam_d.so libhbam_e.so > $O/ab10.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_consumers.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/bench_consumers.py --size 2e9 > $O/bench_consumers.json 2> $O/bench_consumers.err
