set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> gpurun_out/steps.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal in $name rc=$rc"; exit $rc; fi; }
step tests timeout -k 10 240 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread -k "not guess" > gpurun_out/gputest.log 2>&1
step bench timeout -k 10 300 python -u bench.py --size 2e9 --steps 3 --warmup 1 --cpu-budget 5 > gpurun_out/bench2g.json 2> gpurun_out/bench2g.log
step prof timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python -u tools/profile_inflate.py --size 1e9 --reps 2 > gpurun_out/prof.log 2>&1
step guess timeout -k 10 100 python -u tools/guess_timing.py > gpurun_out/guess.log 2>&1
