#!/bin/bash
# Round 3, call H: does the r02 profiling-build failure follow the block's position in the launch
# or its contents, and does it need the profile buffer attached?  r02 source + HBAM_PROF on the
# 2 GB seed-3 file: whole launch with / without the buffer, and launches starting at block 40000
# and 49152 (the first bad block of call G).  Then call D (bench, rocprof, PMC, smoke).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/diag_inflate_build.py --size 2e9 --seed 3 --out $O/diag --keep 3 --libs libhbam_r2fix_prof.so --variants att:0 noatt:0 att:40000 att:49152 att:60000 > $O/diag.txt 2>&1 &&
bash tools/gpu_r3d.sh
echo "rc $?" >> $O/diag.txt
exit 0
