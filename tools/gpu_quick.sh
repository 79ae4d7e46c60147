# usage: bash tools/gpu_quick.sh "<pytest -k expr>" [extra command...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K="$1"; shift
timeout -k 10 200 python -u -m pytest tests -m gpu -x -v --timeout 60 --timeout-method thread -k "$K" > gpurun_out/quick.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $# -gt 0 ]; then timeout -k 10 200 "$@" > gpurun_out/quick_extra.log 2>&1; fi
