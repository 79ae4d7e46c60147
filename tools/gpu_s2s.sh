#!/bin/bash
# Closing check of the committed tree: full GPU suite, smoke, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
