#!/bin/bash
# Huffman pass store/epoch A/B (non-temporal token stores off, 8-iteration epochs) + parity and
# bench of the default build (parallel chain repair).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so libhbam_ns.so libhbam_k8.so libhbam_nsk8.so libhbam.so > $O/ab10.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
