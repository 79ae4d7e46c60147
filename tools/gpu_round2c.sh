# GPU parity file (default + W=512 builds), guesser bench, A/B variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r2c_test.log 2>&1; rc=$?
echo "suite rc=$rc" >> $O/r2c_test.log
[ $rc -gt 1 ] && exit $rc
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_w512.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $O/r2c_w512.log 2>&1; rc2=$?
echo "w512 rc=$rc2" >> $O/r2c_w512.log
[ $rc2 -gt 1 ] && exit $rc2
timeout -k 10 400 python3 -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so libhbam_nost.so > $O/r2c_ab.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/bench_guess.py --size 10e9 > $O/r2c_guess.log 2>&1
