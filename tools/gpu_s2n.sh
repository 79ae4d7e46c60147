#!/bin/bash
# CRC-checked whole-file inflate of 8 generated BAMs (seeds, quality models, levels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_check.txt 2>&1
