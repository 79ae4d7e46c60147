#!/bin/bash
# Cycle-stamp breakdown of the Huffman and LZ77 passes (libhbam_prof.so) at 2 GB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prof_regions.py inflate --size 2e9 > $O/inflate_regions.txt 2>&1
