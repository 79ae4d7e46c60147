#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/h
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/profile_inflate.py --size 2e9 --reps 2 --prof > gpurun_out/h/prof2g.txt 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-include-regex "k_resolve|k_inflate_tokens" -d gpurun_out/h/sq -o run --output-format csv -- python3 tools/profile_inflate.py --size 2e9 --reps 1 > gpurun_out/h/sq.log 2>&1
