# PMC passes over one decode of a synthetic BAM (one kernel, default k_inflate_tokens); summaries -> gpurun_out/pmc_*
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SZ=${1:-2.5e8}
KR=${2:-k_inflate_tokens}
run() { local tag=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KR" -d gpurun_out/pmc_$tag -o run --output-format csv -- python3 tools/profile_inflate.py --size $SZ --reps 1 > gpurun_out/pmc_$tag.log 2>&1; }
timeout -k 10 120 python3 tools/profile_inflate.py --size $SZ --reps 2 > gpurun_out/pmc_plain.log 2>&1 &&
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES &&
run b SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
