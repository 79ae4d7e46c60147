#!/bin/bash
# Round 3, call E: config #3 at 50 GB — 10,000 guesses over per-guess windows (the file is
# generated in chunks and never staged), all checked against the oracle on the same windows.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/bench_guess.py --size 50e9 --guesses 10000 --check 10000 > $O/bench_guess_50g.json 2> $O/bench_guess_50g.err
echo "rc $?" >> $O/bench_guess_50g.err
exit 0
