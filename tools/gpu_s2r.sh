#!/bin/bash
# Block order A/B for the Huffman pass: file order vs compressed length descending vs shuffled
# (host-side permutation of the block list), and the device-side order (HBAM_TOK_ORDER=1
# library: counting sort by compressed length before the pass); CRC + parity with the latter.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_inflate_kernel.py --size 10e9 --seed 2 --reps 2 --libs libhbam.so libhbam_ord.so --orders file clen shuffle > $O/ab_order_10g.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_ord.so timeout -k 10 400 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_ord.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_ord.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_ord.txt 2>&1
