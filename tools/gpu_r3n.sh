#!/bin/bash
# Round 3, call N: streamed config #4 shape — the H2D copy stream confined to k CUs (A/B:
# 0 = all, 8, 16, 32) at 2 and 4 GB windows on the 20 GB shard; the box's SDMA-related env.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3n
mkdir -p $O
export TMPDIR=/tmp
(env | grep -i -E "sdma|blit|HIP_|ROC_|GPU_" || true) > $O/env.txt
timeout -k 10 600 python -u tools/bench_stream.py --size 20e9 --window 2e9 4e9 --reps 2 --copy-cus 0 8 16 32 > $O/stream_cus.json 2> $O/stream_cus.err
echo "rc $?" >> $O/stream_cus.err
exit 0
