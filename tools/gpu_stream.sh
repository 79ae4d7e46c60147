#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_stream.py --size 20e9 --window 4e9 --reps 2 > gpurun_out/s/stream.json 2> gpurun_out/s/stream.err
