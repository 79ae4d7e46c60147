#!/bin/bash
# Round 3, call I (re-run of call H after the container reset): does the r02 profiling-build
# failure follow the block's position in the launch or its contents, and does it need the
# profile buffer?  r02 source (b49031e) + HBAM_PROF + HBAM_TOK_PRED=1 on the 2 GB seed-3 file:
# whole launch with / without the buffer, launches starting at blocks 40000, 49152, 60000.
# Then call D (bench, rocprof kernel stats, FETCH/WRITE passes, smoke).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/diag_inflate_build.py --size 2e9 --seed 3 --out $O/diag --keep 3 --libs libhbam_r2fix_prof.so libhbam_prof.so --variants att:0 noatt:0 att:40000 att:49152 att:60000 > $O/diag.txt 2>&1 &&
bash tools/gpu_r3d.sh
echo "rc $?" >> $O/diag.txt
exit 0
