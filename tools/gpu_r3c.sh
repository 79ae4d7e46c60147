#!/bin/bash
# Round 3, call C: r02 profiling-build failure reproduction (tok_fast_pred, HBAM_TOK_SPEC=0);
# LZ77 pass A/B (dataflow rounds vs round 1 + in-order tail); CRC check of the new pass; GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/diag_inflate_build.py --size 2e9 --seed 3 --out $O/diag --keep 8 --libs libhbam.so libhbam_s0.so libhbam_p_s0.so libhbam_p_s0_ns.so libhbam_p_s1.so > $O/diag.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_inflate_kernel.py --size 5e9 --seed 2 --reps 2 --libs libhbam_rs0.so libhbam.so > $O/ab_resolve.txt 2>&1 &&
timeout -k 10 400 python -u tools/check_inflate_crc.py --size 5e8 > $O/crc_rs1.txt 2>&1 &&
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
echo "rc $?" >> $O/tests.txt
exit 0
