#!/bin/bash
# Huffman pass: up to three literals per iteration (libhbam_l3.so) vs default — A/B at 10 GB,
# then parity of l3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so libhbam_l3.so libhbam.so libhbam_l3.so > $O/ab10.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_l3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_l3.txt 2>&1
