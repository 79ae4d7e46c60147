# GPU suite (continue past failures), W=512 parity file, A/B variants, SQ pass on k_inflate_tokens
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r2b_test.log 2>&1; rc=$?
echo "suite rc=$rc" >> $O/r2b_test.log
[ $rc -gt 1 ] && exit $rc
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_w512.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $O/r2b_w512.log 2>&1; rc2=$?
echo "w512 rc=$rc2" >> $O/r2b_w512.log
[ $rc2 -gt 1 ] && exit $rc2
timeout -k 10 400 python3 -u tools/ab_inflate_kernel.py --size 10e9 --reps 2 --libs libhbam.so libhbam_nost.so libhbam_k8.so libhbam_k2.so libhbam_r1.so > $O/r2b_ab.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex "k_inflate_tokens|k_resolve" -d $O/r2b_sq -o run --output-format csv -- python3 tools/ab_inflate_kernel.py --size 10e9 --reps 1 > $O/r2b_sq.log 2>&1
