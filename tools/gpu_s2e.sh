#!/bin/bash
# Huffman pass: predicated fast path (libhbam_p.so) vs default — A/B at 10 GB, then parity of p.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so libhbam_p.so libhbam.so libhbam_p.so > $O/ab10.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_p.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_p.txt 2>&1
