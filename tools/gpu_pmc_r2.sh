#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter group each) for the Huffman pass and the pools
# kernel over one 10 GB decode; folded into profiles/pmc_*.json by tools/pmc_summarize.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p
export TMPDIR=/tmp
run() { local tag=$1 ctr=$2; timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "k_inflate_tokens|k_decode_pools|k_resolve" -d gpurun_out/p/$tag -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > gpurun_out/p/$tag.log 2>&1; }
run fetch FETCH_SIZE && run write WRITE_SIZE
