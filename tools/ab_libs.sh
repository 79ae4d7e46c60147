# A/B of libhbam builds: timing + FETCH/WRITE of k_inflate_tokens at one size
# usage: ab_libs.sh SIZE lib1 lib2 ...   (paths relative to hadoop-bam_amd/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
SZ=$1; shift
for L in "$@"; do
  export HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/$L
  timeout -k 10 120 python3 tools/profile_inflate.py --size $SZ --reps 2 > $O/ab_$L.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_inflate_tokens -d $O/abf_$L -o run --output-format csv -- python3 tools/profile_inflate.py --size $SZ --reps 1 > $O/abf_$L.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_inflate_tokens -d $O/abw_$L -o run --output-format csv -- python3 tools/profile_inflate.py --size $SZ --reps 1 > $O/abw_$L.log 2>&1 || exit $?
done
