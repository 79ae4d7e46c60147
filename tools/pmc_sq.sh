# SQ pass (LDS bank conflicts, wave issue/wait split) for the two inflate kernels at one size.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
SZ=${1:-2e9}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "k_inflate_tokens|k_resolve" -d $O/pmc_sq -o run --output-format csv -- python3 tools/profile_inflate.py --size $SZ --reps 1 > $O/pmc_sq.log 2>&1
