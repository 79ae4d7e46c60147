#!/bin/bash
# Cycle-stamp breakdown of the Huffman and LZ77 passes (profiling builds) at 2 GB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2k
mkdir -p $O
export TMPDIR=/tmp
for L in libhbam_prof_rs.so libhbam_prof_tk.so libhbam_prof.so; do
  PROF_LIB=$L timeout -k 10 300 python -u tools/prof_regions.py inflate --size 2e9 > $O/inflate_regions_$L.txt 2>&1
done
exit 0
