#!/bin/bash
# Round 3, call Z: config #4 and #5 per-GPU shares on the final tree — 25 GB streamed from
# page-locked host memory (2 GB windows) and the 12.5 GB Sort path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_decode.py --size 5e9 --reps 3 --libs libhbam.so libhbam_spf.so libhbam.so libhbam_spf.so > $O/ab_scan_pf.txt 2>&1 &&
timeout -k 10 500 python -u tools/bench_stream.py --size 25e9 --window 2e9 --reps 2 > $O/stream_25g.json 2> $O/stream_25g.err &&
timeout -k 10 400 python -u tools/bench_sort.py --size 12.5e9 > $O/bench_sort_12g.json 2> $O/bench_sort_12g.err
echo "rc $?" >> $O/bench_sort_12g.err
exit 0
