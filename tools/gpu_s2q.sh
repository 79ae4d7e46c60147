#!/bin/bash
# A/B: pre matches in 32-byte pieces over the lanes (HBAM_RS_PIECES=1) vs whole matches per
# lane, 10 GB, same box; CRC-checked inflate and the parity file with the variant library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_inflate_kernel.py --size 10e9 --seed 2 --reps 2 --libs libhbam.so libhbam_pc.so libhbam.so libhbam_pc.so > $O/ab_pieces_10g.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_pc.so timeout -k 10 400 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_pc.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_pc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_pc.txt 2>&1
