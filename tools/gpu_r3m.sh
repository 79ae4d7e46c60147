#!/bin/bash
# Round 3, call M: GPU suite + config #2 bench line (block scan and fixed-field decode read
# through 16-byte loads); config #4 streamed shape — window-size sweep (1/2/4 GB) on the 20 GB
# shard, then a kernel + memory-copy trace of a smaller streamed read (how the H2D copies
# overlap the decode kernels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $O/bench10g.json 2> $O/bench10g.err &&
timeout -k 10 500 python -u tools/bench_stream.py --size 20e9 --window 1e9 2e9 4e9 --reps 2 > $O/stream_sweep.json 2> $O/stream_sweep.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 tools/bench_stream.py --size 8e9 --window 2e9 --reps 1 > $O/trace_stream.json 2> $O/trace_stream.err
echo "rc $?" >> $O/tests.txt
exit 0
