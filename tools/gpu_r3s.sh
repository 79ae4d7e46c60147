#!/bin/bash
# Round 3, call S: pools kernel loads in flight per lane (POOL_ILP 4 = libhbam.so, 2, 1) and the
# session-start library (r3start: block scan before the two-pass fallback refactor) on a 5 GB
# shard, outputs digested and compared; GPU parity tests of the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_decode.py --size 5e9 --reps 3 --libs libhbam.so libhbam_ilp2.so libhbam_ilp1.so libhbam_r3start.so libhbam.so > $O/ab_ilp_fixed.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
echo "rc $?" >> $O/tests.txt
exit 0
