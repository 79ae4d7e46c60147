#!/bin/bash
# Round 3, call O: pools kernel rewritten (thread per record, 16-byte copies, grid-stride: the
# r02 grid of 64 x records threads wrapped past 2^32 above 67 M records) and the record gather
# made grid-stride.  GPU suite; config #2 bench line with parity extended to the field pools and
# to the timed whole-shard launch; rocprof kernel stats; streamed 2/4 GB windows on the 20 GB
# shard; config #5 per-GPU share (12.5 GB) sort.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench10g.json 2> $O/bench10g.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --parity-splits 0 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 400 python -u tools/bench_stream.py --size 20e9 --window 2e9 4e9 --reps 2 > $O/stream_20g.json 2> $O/stream_20g.err &&
timeout -k 10 400 python -u tools/bench_sort.py --size 12.5e9 > $O/bench_sort_12g.json 2> $O/bench_sort_12g.err
echo "rc $?" >> $O/tests.txt
exit 0
