#!/bin/bash
# Round 3, call B: reproduce the r02 profiling-build decode failure (predicated fast path
# tok_fast_pred, HBAM_TOK_SPEC=0) at the r02 configuration (2 GB, seed 3) and record the exit
# state of the first bad blocks; then the CRC check of the profiling build with today's path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/diag_inflate_build.py --size 2e9 --seed 3 --out $O/diag --keep 8 --libs libhbam.so libhbam_s0.so libhbam_p_s0.so libhbam_p_s0_ns.so libhbam_p_s1.so > $O/diag.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_p_s1.so timeout -k 10 600 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_prof_s1.txt 2>&1
