#!/bin/bash
# Round 3, call L: Huffman pass A/B — symbol tables lane-contiguous (libhbam.so) vs interleaved
# across the lanes by dword (libhbam_ilv.so, HBAM_TOK_ILV=1); CRC check of the interleaved build
# on the 8 files of check_inflate_crc.py (2 GB each: > 3 waves per slot) and its launch-position
# test; SQ counters of the interleaved build (LDS bank conflicts); config #4 streamed 20 GB shard
# and config #5 per-GPU sort at 10 GB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3l
mkdir -p $O
export TMPDIR=/tmp
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_r2fix_prof.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k launch_position -v --timeout 150 --timeout-method thread > $O/position_r2fix_prof.txt 2>&1; r=$?; echo "rc $r" >> $O/position_r2fix_prof.txt; { [ $r -eq 0 ] || [ $r -eq 1 ]; } || exit 0
timeout -k 10 400 python -u tools/ab_inflate_kernel.py --size 5e9 --seed 2 --reps 3 --libs libhbam.so libhbam_ilv.so libhbam.so libhbam_ilv.so > $O/ab_ilv.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_ilv.so timeout -k 10 500 python -u tools/check_inflate_crc.py --size 2e9 > $O/crc_ilv.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_ilv.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "launch_position or tiny_blocks or deflate_variants or misalignment or corrupted" -v --timeout 150 --timeout-method thread > $O/tests_ilv.txt 2>&1 &&
export HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_ilv.so && bash tools/pmc_sq.sh 2e9 && mv gpurun_out/pmc_sq gpurun_out/pmc_sq.log $O/ && unset HBAM_LIB &&
timeout -k 10 400 python -u tools/bench_stream.py --size 20e9 --window 4e9 > $O/stream_20g.json 2> $O/stream_20g.err &&
timeout -k 10 400 python -u tools/bench_sort.py --size 10e9 > $O/bench_sort_10g.json 2> $O/bench_sort_10g.err
echo "rc $?" >> $O/ab_ilv.txt
exit 0
