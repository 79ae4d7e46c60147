#!/bin/bash
# LZ77 pass occupancy A/B (packed match records, window, waves/SIMD) + parity of the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_consumers.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam_a.so libhbam_b.so libhbam_c.so libhbam_d.so libhbam_e.so > $O/ab10.txt 2>&1
