#!/bin/bash
# Round 3, call T (re-run on the final tree): closing check — GPU suite, config #2 bench line, rocprof kernel
# stats of the same command, smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3t3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; echo "rc $?" >> $O/tests.txt
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench10g.json 2> $O/bench10g.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --parity-splits 0 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo "rc $?" >> $O/smoke.txt
exit 0
