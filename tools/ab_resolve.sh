# A/B of resolver builds (timing only) + inflate/decode parity under the candidate build.
# usage: ab_resolve.sh SIZE CANDIDATE_LIB   (paths relative to hadoop-bam_amd/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
SZ=$1; CAND=$2
for L in libhbam.so $CAND; do
  HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/$L timeout -k 10 150 python3 tools/profile_inflate.py --size $SZ --reps 3 > $O/abr_$L.log 2>&1 || exit $?
done
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/$CAND timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/abr_parity.log 2>&1
