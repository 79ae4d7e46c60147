# iterate: GPU parity tests (inflate/decode) + one 2 GB decode timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/iter_test.log 2>&1 &&
timeout -k 10 200 python3 tools/profile_inflate.py --size ${1:-2e9} --reps 2 > $O/iter_prof.log 2>&1
