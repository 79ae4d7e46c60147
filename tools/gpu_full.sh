# Round GPU pass: gpu tests, smoke, 10 GB bench, rocprof kernel-trace of the bench, PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >> $O/steps.log; if [ $rc -ne 0 ]; then echo "fatal in $name rc=$rc"; exit $rc; fi; }
rm -f $O/steps.log
[ "${SKIP_TESTS:-0}" = 1 ] || step tests timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 400 python -u bench.py > $O/bench10g.json 2> $O/bench10g.log
step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof10g -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof10g.log 2>&1
step pmc_f timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_inflate_tokens -d $O/pmc_f -o run --output-format csv -- python3 -u tools/profile_inflate.py --size 10e9 --reps 1 > $O/pmc_f.log 2>&1
step pmc_w timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_inflate_tokens -d $O/pmc_w -o run --output-format csv -- python3 -u tools/profile_inflate.py --size 10e9 --reps 1 > $O/pmc_w.log 2>&1
