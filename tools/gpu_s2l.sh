#!/bin/bash
# dot2 accumulation in the packed lookup (libhbam_d2.so) vs default, + parity of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so libhbam_d2.so libhbam.so libhbam_d2.so > $O/ab10.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_d2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_d2.txt 2>&1
