#!/bin/bash
# One parameterised GPU call (replaces the per-call gpu_r3*.sh scripts of round 3):
#   gpurun -- bash tools/gpu_run.sh OUT STEP[,ARG...] ...
# Steps run in order, each under its own time limit, and the first one that fails hard (a
# fault, an abort, a time limit) ends the call; pytest's "some tests failed" (rc 1) does not.
#   tests[,EXPR]         pytest -m gpu (optionally -k EXPR)
#   testslib,LIB[,EXPR] the same against hadoop-bam_amd/LIB (HBAM_LIB)
#   smoke                __graft_entry__.smoke()
#   bench[,STEPS]        python bench.py (default --steps 20 --warmup 3)
#   prof                 rocprofv3 --kernel-trace --stats of a short bench.py run
#   pmc,COUNTERS[,SIZE[,LIB]]  one rocprofv3 --pmc pass (COUNTERS separated by '+') over a decode
#   pmcbytes[,SIZE]      FETCH_SIZE + WRITE_SIZE passes over a decode, folded by tools/pmc_summarize.py
#   bin,PATH             run a probe executable (tools/probes/*)
#   abdecode,SIZE,LIBS   tools/ab_decode.py A/B of library builds (LIBS separated by '+')
#   stream,SIZE,WINDOW   tools/bench_stream.py (config #4 share)
#   sort,SIZE[,LIB]      tools/bench_sort.py (config #5 share), optionally against hadoop-bam_amd/LIB
#   guess,SIZE           tools/bench_guess.py (config #3)
#   crc                  tools/check_inflate_crc.py
#   calib                rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/pmc_calib (known bytes per shape)
#   py,SCRIPT[,ARGS..]   any repo script (ARGS separated by ',')
#   pyo,NAME,SCRIPT[,ARGS..]  the same, output to NAME.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
shift
mkdir -p $O
export TMPDIR=/tmp
hard() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
for spec in "$@"; do
  IFS=, read -r step a1 a2 a3 <<< "$spec"
  echo "== $spec $(date +%T)" >> $O/steps.log
  case $step in
    tests)
      K=(); [ -n "$a1" ] && K=(-k "$a1")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread "${K[@]}" > $O/tests.txt 2>&1; r=$? ;;
    testslib)  # testslib,LIB[,EXPR]: pytest -m gpu against another build of the library
      K=(); [ -n "$a2" ] && K=(-k "$a2")
      HBAM_LIB=hadoop-bam_amd/$a1 timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread "${K[@]}" > $O/tests_$a1.txt 2>&1; r=$? ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; r=$? ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps ${a1:-20} --warmup 3 > $O/bench.json 2> $O/bench.err; r=$? ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --parity-splits 0 --no-whole-check > $O/bench_prof.json 2> $O/prof.err; r=$? ;;
    pmc)  # pmc,COUNTERS[,SIZE[,LIB]]: one counter pass over a decode (csv per dispatch)
      P=$O/pmc_${a1//+/_}${a3:+_$a3}
      timeout -s KILL 300 rocprofv3 --pmc ${a1//+/ } -d $P -o run --output-format csv -- python3 tools/ab_decode.py --size ${a2:-2e9} --reps 1 --digest 0 --libs ${a3:-libhbam.so} > $P.txt 2>&1; r=$? ;;
    pmcbytes)  # pmcbytes[,SIZE]: FETCH_SIZE and WRITE_SIZE passes over one decode -> tools/pmc_summarize.py
      timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmcb_fetch -o run --output-format csv -- python3 tools/ab_decode.py --size ${a1:-10e9} --reps 1 --digest 0 --libs libhbam.so > $O/pmcb_fetch.txt 2>&1 &&
      timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmcb_write -o run --output-format csv -- python3 tools/ab_decode.py --size ${a1:-10e9} --reps 1 --digest 0 --libs libhbam.so > $O/pmcb_write.txt 2>&1; r=$?
      if [ $r -eq 0 ]; then
        COMP=$(grep -m1 '^comp_bytes' $O/pmcb_fetch.txt | cut -d' ' -f2)
        STG=""; [ -s $O/bench.json ] && STG=$O/bench.json
        python3 tools/pmc_summarize.py $(ls $O/pmcb_fetch/*counter_collection.csv $O/pmcb_fetch/*/*counter_collection.csv 2>/dev/null | head -1) $(ls $O/pmcb_write/*counter_collection.csv $O/pmcb_write/*/*counter_collection.csv 2>/dev/null | head -1) $COMP $O/pmcsum ${PMC_TREE:-round6} $STG > $O/pmcsum.txt 2>&1
      fi ;;
    bin)  # bin,PATH: a probe executable of the repository
      timeout -k 10 300 ./$a1 > $O/$(basename $a1).txt 2>&1; r=$? ;;
    abdecode)
      timeout -k 10 900 python -u tools/ab_decode.py --size ${a1:-5e9} --reps ${a3:-3} --libs ${a2//+/ } > $O/ab_${a2//+/_}.txt 2>&1; r=$? ;;
    stream)
      timeout -k 10 600 python -u tools/bench_stream.py --size ${a1:-25e9} --window ${a2:-2e9} --reps 2 > $O/stream.json 2> $O/stream.err; r=$? ;;
    sort)  # sort[,SIZE[,LIB]]
      if [ -n "$a2" ]; then export HBAM_LIB=hadoop-bam_amd/$a2; fi
      timeout -k 10 600 python -u tools/bench_sort.py --size ${a1:-12.5e9} > $O/sort${a2:+_$a2}.json 2> $O/sort${a2:+_$a2}.err; r=$?
      unset HBAM_LIB ;;
    guess)
      timeout -k 10 700 python -u tools/bench_guess.py --size ${a1:-50e9} --guesses 10000 --check 10000 > $O/guess.json 2> $O/guess.err; r=$? ;;
    calib)  # FETCH_SIZE / WRITE_SIZE per access shape (tools/pmc_calib.hip, tools/pmc_calib.py)
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- ./tools/pmc_calib > $O/calib.txt 2>&1 &&
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- ./tools/pmc_calib > $O/calib_w.txt 2>&1; r=$?
      [ $r -eq 0 ] && python3 tools/pmc_calib.py $O/calib.txt $(ls $O/calib_fetch/*counter_collection.csv $O/calib_fetch/*/*counter_collection.csv 2>/dev/null | head -1) $(ls $O/calib_write/*counter_collection.csv $O/calib_write/*/*counter_collection.csv 2>/dev/null | head -1) $O/calib.json > $O/calib_summary.txt 2>&1 ;;
    crc)
      timeout -k 10 900 python -u tools/check_inflate_crc.py > $O/crc.txt 2>&1; r=$? ;;
    pyo)
      rest="${spec#pyo,$a1,$a2}"; rest="${rest#,}"; ARGS=(); [ -n "$rest" ] && IFS=, read -r -a ARGS <<< "$rest"
      timeout -k 10 900 python -u "$a2" "${ARGS[@]}" > $O/$a1.txt 2>&1; r=$? ;;
    py)
      rest="${spec#py,$a1}"; rest="${rest#,}"; ARGS=(); [ -n "$rest" ] && IFS=, read -r -a ARGS <<< "$rest"
      timeout -k 10 900 python -u "$a1" "${ARGS[@]}" > $O/$(basename $a1 .py).txt 2>&1; r=$? ;;
    *)
      echo "unknown step $spec" >> $O/steps.log; r=2 ;;
  esac
  echo "rc $r $(date +%T)" >> $O/steps.log
  if hard $r; then exit 0; fi
done
exit 0
