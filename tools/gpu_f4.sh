#!/bin/bash
# f-4 consumers: GPU parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_consumers.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/f4/tests.txt 2>&1
