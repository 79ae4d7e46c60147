# A/B of the Huffman passes (inflate_mode 0 = wave-parallel, 1 = lane-per-block) at one size
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SZ=${1:-2e9}
timeout -k 10 200 python3 tools/profile_inflate.py --size $SZ --reps 3 --mode 0 > gpurun_out/ab_mode0.log 2>&1 &&
timeout -k 10 200 python3 tools/profile_inflate.py --size $SZ --reps 3 --mode 1 > gpurun_out/ab_mode1.log 2>&1
