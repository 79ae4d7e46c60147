# timing-only A/B of libhbam builds: usage ab_time.sh SIZE lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for L in "$@"; do
  [ "$L" = "$1" ] && continue
  HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/$L timeout -k 10 120 python3 tools/profile_inflate.py --size $1 --reps 2 > gpurun_out/abt_$L.log 2>&1 || exit $?
done
