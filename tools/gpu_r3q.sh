#!/bin/bash
# Round 3, call Q: pools kernel unit size A/B (16-byte units, libhbam.so, vs 8-byte,
# libhbam_pu8.so) on a 5 GB shard, outputs digested and compared; GPU parity tests of the
# pools (16-byte build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_decode.py --size 5e9 --reps 3 --libs libhbam.so libhbam_pu8.so libhbam.so libhbam_pu8.so > $O/ab_pool_unit8.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
echo "rc $?" >> $O/tests.txt
exit 0
