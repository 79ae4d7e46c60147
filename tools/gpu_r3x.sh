#!/bin/bash
# Round 3, call X: pools kernel with every field's units numbered together in source order
# (libhbam.so) vs field by field (libhbam_g16.so) on a 5 GB shard, digests compared; FETCH and
# WRITE of the new kernel at config #2 size (separate passes); GPU parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_decode.py --size 5e9 --reps 3 --libs libhbam.so libhbam_g16.so libhbam.so libhbam_g16.so > $O/ab.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_decode_pools" -d $O/pmc_fetch -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_decode_pools" -d $O/pmc_write -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > $O/pmc_write.log 2>&1
echo "rc $?" >> $O/tests.txt
exit 0
