#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/j
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/profile_inflate.py --size 2e9 --reps 2 --prof > gpurun_out/j/prof2g.txt 2>&1
