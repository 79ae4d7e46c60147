#!/bin/bash
# Round 3, call V: PMC of the fixed tree at config #2 size — FETCH_SIZE and WRITE_SIZE (separate
# passes) of the pools kernel, the fixed-field decode, the block scan and the Huffman/LZ77
# passes; SQ wait / LDS counters of the pools kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3v
mkdir -p $O
export TMPDIR=/tmp
K="k_inflate_tokens|k_resolve|k_decode_pools|k_decode_fixed|k_scan_chunks"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/pmc_fetch -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/pmc_write -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > $O/pmc_write.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "k_decode_pools|k_decode_fixed" -d $O/pmc_sq -o run --output-format csv -- python3 tools/profile_inflate.py --size 2e9 --reps 1 > $O/pmc_sq.log 2>&1
echo "rc $?" >> $O/pmc_sq.log
exit 0
