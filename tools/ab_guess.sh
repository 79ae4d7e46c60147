# A/B of k_guess_bam lane counts: config#3 bench (2 GB file) per lib + guesser parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
for L in "$@"; do
  HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/$L timeout -k 10 150 python3 -u tools/bench_guess.py --size 2e9 --check 100 > $O/abg_$L.json 2> $O/abg_$L.log || exit $?
  HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/$L timeout -k 10 200 python3 -u -m pytest tests -m gpu -k "guess or split" -x -q --timeout 150 --timeout-method thread > $O/abg_par_$L.log 2>&1 || exit $?
done
