#!/bin/bash
# Round-2 final evidence, part A: full GPU suite, smoke, deflate bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fa
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fa/tests.txt 2>&1; r=$?
[ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fa/smoke.txt 2>&1 &&
timeout -k 10 300 python -u tools/bench_deflate.py --size 1e9 --reps 2 > gpurun_out/fa/deflate.json 2> gpurun_out/fa/deflate.err
