# SQ counters of k_inflate_tokens (issue vs stall) over one 2 GB decode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
run() { local tag=$1; shift; timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "k_inflate_tokens|k_resolve" -d $O/pmt_$tag -o run --output-format csv -- python3 tools/profile_inflate.py --size 2e9 --reps 1 > $O/pmt_$tag.log 2>&1; }
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES &&
run b SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
