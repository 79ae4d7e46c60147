#!/bin/bash
# LZ77 pass late write-back / Huffman epoch length / non-temporal input loads A/B at 10 GB, then
# parity + bench of the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam_ewb.so libhbam.so libhbam_k2.so libhbam_nl.so libhbam_ewb.so libhbam.so > $O/ab10.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
