set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_sort.py -m gpu -x -v --timeout 100 --timeout-method thread > $O/sorttest.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_sort.py --size ${1:-2e9} > $O/bench_sort.json 2> $O/bench_sort.log
