#!/bin/bash
# Round 3, call R: tail-store cost of the pools kernel (A/B build that writes every unit as a
# full 16-byte store, wrong past the segment end: timing only); config #2 bench line + rocprof
# kernel stats of the tree; config #4 per-GPU share streamed (25 GB = 200 GB / 8 GPUs, 2 and
# 4 GB windows); config #5 per-GPU share sort (12.5 GB = 100 GB / 8 GPUs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_decode.py --size 5e9 --reps 3 --digest 0 --libs libhbam.so libhbam_tailab.so libhbam.so > $O/ab_tail.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench10g.json 2> $O/bench10g.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --parity-splits 0 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 500 python -u tools/bench_stream.py --size 25e9 --window 2e9 4e9 --reps 2 > $O/stream_25g.json 2> $O/stream_25g.err &&
timeout -k 10 400 python -u tools/bench_sort.py --size 12.5e9 > $O/bench_sort_12g.json 2> $O/bench_sort_12g.err
echo "rc $?" >> $O/ab_tail.txt
exit 0
