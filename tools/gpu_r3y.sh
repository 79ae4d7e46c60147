#!/bin/bash
# Round 3, call Y: LZ77 pass A/B — pre-match copies as 16-byte units numbered over the lanes
# (libhbam_rsu.so, HBAM_RS_UNITS=1) vs one lane per match (libhbam.so) on a 5 GB shard, digests
# compared; CRC check of the units build on the 8 files (1 GB each) and its inflate tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_decode.py --size 5e9 --reps 3 --libs libhbam.so libhbam_rsu.so libhbam.so libhbam_rsu.so > $O/ab.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_rsu.so timeout -k 10 500 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_rsu.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_rsu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_rsu.txt 2>&1
echo "rc $?" >> $O/tests_rsu.txt
exit 0
