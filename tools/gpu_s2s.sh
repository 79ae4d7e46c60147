#!/bin/bash
# Closing check of the committed tree: full GPU suite, smoke, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 500 python -u tools/ab_inflate_kernel.py --size 10e9 --seed 2 --reps 2 --libs libhbam.so libhbam_mk.so libhbam.so libhbam_mk.so > $O/ab_mark_10g.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_mk.so timeout -k 10 400 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_mk.txt 2>&1
