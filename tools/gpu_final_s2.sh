#!/bin/bash
# Round-2 (session 2) evidence on the committed tree: full GPU suite, smoke, bench line, rocprof
# kernel stats of the same command, FETCH/WRITE passes of the decode kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fs2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/rp -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --parity-splits 0 > $O/bench_rp.json 2> $O/bench_rp.err &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_inflate_tokens|k_decode_pools|k_resolve" -d $O/fetch -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > $O/fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_inflate_tokens|k_decode_pools|k_resolve" -d $O/write -o run --output-format csv -- python3 tools/profile_inflate.py --size 10e9 --reps 1 > $O/write.log 2>&1
