#!/bin/bash
# A/B: tok_fast_spec (decode before output; SPEC=1) and the one-packet sink (SPEC=2) vs the
# shipped predicated path, 10 GB, same box; CRC-checked inflate of the variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_inflate_kernel.py --size 10e9 --seed 2 --reps 2 --libs libhbam.so libhbam_s1.so libhbam_s2.so libhbam.so libhbam_s1.so libhbam_s2.so > $O/ab_spec_10g.txt 2>&1 &&
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_s2.so timeout -k 10 400 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_s2.txt 2>&1 ;
HBAM_LIB=$GRAFT_REPO_ROOT/hadoop-bam_amd/libhbam_s1.so timeout -k 10 400 python -u tools/check_inflate_crc.py --size 1e9 > $O/crc_s1.txt 2>&1
