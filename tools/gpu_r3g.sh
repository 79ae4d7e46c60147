#!/bin/bash
# Round 3, call G: the r02 profiling-build decode failure, root cause — the same 2 GB seed-3 file
# through the r02 source before the shift fix (default + HBAM_PROF builds), the r02 source after
# it (HBAM_PROF with the predicated path forced on), and today's source (default + HBAM_PROF,
# the PROF -> branching-path override removed); then CRC checks of both current builds on the
# 8 files of check_inflate_crc.py, and the GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/diag_inflate_build.py --size 2e9 --seed 3 --out $O/diag --keep 4 --libs libhbam.so libhbam_prof.so libhbam_r2pre.so libhbam_r2pre_prof.so libhbam_r2fix_prof.so > $O/diag.txt 2>&1 &&
timeout -k 10 400 python -u tools/check_inflate_crc.py --size 5e8 > $O/crc_default.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_prof.so timeout -k 10 400 python -u tools/check_inflate_crc.py --size 5e8 > $O/crc_prof.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
echo "rc $?" >> $O/tests.txt
exit 0
