#!/bin/bash
# Round 3, call W2: pools kernel software-pipelined by one unit (libhbam.so, 7 waves/SIMD; libhbam_wpe8.so
# asked for 8 waves/SIMD, spills) vs the one-unit-per-step kernel (libhbam_g16.so); outputs
# digested and compared; GPU parity tests of the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_decode.py --size 5e9 --reps 3 --libs libhbam.so libhbam_wpe8.so libhbam_g16.so libhbam.so libhbam_wpe8.so libhbam_g16.so > $O/ab2.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
echo "rc $?" >> $O/tests.txt
exit 0
