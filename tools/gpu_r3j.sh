#!/bin/bash
# Round 3, call J: GPU suite (with the launch-position test); the launch-position test against
# the r02 profiling build (expected to fail: it reproduces the r02 defect) and the current
# profiling build; LZ77 pass A/B (conditional match-copy loads); SQ counters of both inflate
# kernels (waits, LDS bank conflicts, instruction mix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3j
mkdir -p $O
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }  # pytest: 0 pass, 1 test failure; anything else stops
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; r=$?; echo "rc $r" >> $O/tests.txt; ok $r || exit 0
for L in libhbam_r2fix_prof.so libhbam_prof.so; do
  HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/$L timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k launch_position -v --timeout 150 --timeout-method thread > $O/position_$L.txt 2>&1; r=$?; echo "rc $r" >> $O/position_$L.txt; ok $r || exit 0
done
timeout -k 10 300 python -u tools/ab_inflate_kernel.py --size 5e9 --seed 2 --reps 3 --libs libhbam.so libhbam_rscl.so libhbam.so libhbam_rscl.so > $O/ab_condld.txt 2>&1 &&
bash tools/pmc_sq.sh 2e9 && mv gpurun_out/pmc_sq gpurun_out/pmc_sq.log $O/ &&
bash tools/pmc_inst.sh 2e9 $O/pmc_inst
echo "rc $?" >> $O/ab_condld.txt
exit 0
