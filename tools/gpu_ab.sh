# parity subset + A/B of libhbam builds on one synthetic BAM
# usage: bash tools/gpu_ab.sh SIZE "<pytest -k expr>" lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
SZ=$1; K="$2"; shift 2
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/ab_test.log 2>&1 || exit $?
fi
timeout -k 10 400 python3 -u tools/ab_inflate_kernel.py --size $SZ --reps 3 --libs "$@" > $O/ab_time.log 2>&1
