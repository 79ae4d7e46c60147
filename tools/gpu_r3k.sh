#!/bin/bash
# Round 3, call K: GPU suite (exact two-pass block scan for tiny blocks, launch-position test);
# the launch-position test against the r02 profiling build (expected to fail: the r02 defect)
# and the current profiling build; config #3 at 50 GB (10,000 windowed guesses, all checked).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3k
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }  # pytest: 0 pass, 1 test failure; anything else stops
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; r=$?; echo "rc $r" >> $O/tests.txt; ok $r || exit 0
for L in libhbam_r2fix_prof.so libhbam_prof.so; do
  HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/$L timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k launch_position -v --timeout 150 --timeout-method thread > $O/position_$L.txt 2>&1; r=$?; echo "rc $r" >> $O/position_$L.txt; ok $r || exit 0
done
timeout -k 10 700 python -u tools/bench_guess.py --size 50e9 --guesses 10000 --check 10000 > $O/bench_guess_50g.json 2> $O/bench_guess_50g.err
echo "rc $?" >> $O/bench_guess_50g.err
exit 0
