#!/bin/bash
# Round 3, call P: pools kernel as a wave per 64-record tile with 16-byte units spread over the
# lanes.  GPU suite; config #2 bench line (parity incl. pools and the whole-shard launch);
# rocprof kernel stats of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench10g.json 2> $O/bench10g.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --parity-splits 0 > $O/bench_prof.json 2> $O/bench_prof.err
echo "rc $?" >> $O/tests.txt
exit 0
