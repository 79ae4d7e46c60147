#!/bin/bash
# Third literal per fast-path iteration on the packet sink (HBAM_TOK_LIT3=1) vs the default;
# GPU suite of the default tree (its packet insert now admits 6-byte packets), CRC for both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 500 python -u tools/ab_inflate_kernel.py --size 10e9 --seed 2 --reps 2 --libs libhbam.so libhbam_l3.so libhbam.so libhbam_l3.so > $O/ab_lit3_10g.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_l3.so timeout -k 10 400 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_l3.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_l3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_l3.txt 2>&1 &&
timeout -k 10 400 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_default.txt 2>&1
