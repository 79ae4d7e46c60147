#!/bin/bash
# Instruction mix of the two inflate kernels (one PMC pass, SQ block only): VALU/SALU/LDS/VMEM
# instructions and waves, for instructions per loop iteration.  Usage: pmc_inst.sh SIZE OUTDIR
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
SZ=${1:-2e9}
O=${2:-gpurun_out/pmc_inst}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "k_inflate_tokens|k_resolve" -d $O -o run --output-format csv -- python3 tools/profile_inflate.py --size $SZ --reps 1 > $O/log.txt 2>&1
