#!/bin/bash
# Round 3, call D: evidence of the current tree at config #2 — bench line, rocprofv3 kernel
# stats of the same command, FETCH_SIZE / WRITE_SIZE passes of the Huffman pass (separate runs),
# smoke.  Outputs under gpurun_out/r3d (copied into profiles/r03 afterwards).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $O/bench10g.json 2> $O/bench10g.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_inflate_tokens|k_resolve|k_decode_pools" -d $O/pmc_fetch -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_inflate_tokens|k_resolve|k_decode_pools" -d $O/pmc_write -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > $O/pmc_write.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo "rc $?" >> $O/smoke.txt
exit 0
