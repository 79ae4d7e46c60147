#!/bin/bash
# Round 3, call A: build-dependence diagnosis of the Huffman pass (default vs profiling builds,
# CRC-checked, exit state of the first bad blocks), then the GPU suite and a bench line on a fresh box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag_inflate_build.py --size 5e8 --out $O/diag --libs libhbam.so libhbam_pp.so libhbam_ppns.so libhbam_prof.so > $O/diag.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
