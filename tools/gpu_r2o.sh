#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/o
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_lz77_tokens|k_deflate_encode" -d gpurun_out/o/a -o run --output-format csv -- python3 tools/bench_deflate.py --size 2.5e8 --reps 1 > gpurun_out/o/a.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR --kernel-include-regex "k_lz77_tokens|k_deflate_encode" -d gpurun_out/o/b -o run --output-format csv -- python3 tools/bench_deflate.py --size 2.5e8 --reps 1 > gpurun_out/o/b.log 2>&1
