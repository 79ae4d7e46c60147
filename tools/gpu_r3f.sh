#!/bin/bash
# Round 3, call F: config #4's streamed shape (a 20 GB shard from page-locked host memory through
# hbam_split_open/next, copy overlapped with decode) and config #5's per-GPU sort at 10 GB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_stream.py --size 20e9 --window 4e9 > $O/stream_20g.json 2> $O/stream_20g.err &&
timeout -k 10 400 python -u tools/bench_sort.py --size 10e9 > $O/bench_sort_10g.json 2> $O/bench_sort_10g.err
echo "rc $?" >> $O/bench_sort_10g.err
exit 0
