#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/diag_align.py guess_window_4197.bin guess_window_7433.bin > gpurun_out/f/align.txt 2>&1 &&
timeout -k 10 300 python -u tools/profile_inflate.py --size 2e9 --reps 2 --prof > gpurun_out/f/prof2g.txt 2>&1
