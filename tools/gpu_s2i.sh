#!/bin/bash
# With plain token stores: 3-literal iterations, the no-store lower bound, two-stream slices.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so libhbam_l3.so libhbam_nost.so libhbam_df.so libhbam.so libhbam_l3.so libhbam_df.so > $O/ab10.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so --slices 1 2 > $O/ab_slices.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_df.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_df.txt 2>&1
