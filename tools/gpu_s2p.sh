#!/bin/bash
# Packet sink as default: GPU parity suite, epoch period A/B (K = 2 / 4 / 8), bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 500 python -u tools/ab_inflate_kernel.py --size 10e9 --seed 2 --reps 2 --libs libhbam.so libhbam_k2.so libhbam_k8.so libhbam.so libhbam_k8.so > $O/ab_k_10g.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
