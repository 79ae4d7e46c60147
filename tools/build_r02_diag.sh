#!/bin/bash
# Rebuild the r02 library that showed the launch-position decode failure:
# source of commit b49031e (predicated fast path, round 2) with the cycle-stamp profiling build
# and the predicated path forced on -> hadoop-bam_amd/libhbam_r2fix_prof.so; and the current
# source's profiling build -> hadoop-bam_amd/libhbam_prof.so.  Run from the repository root.
set -e
mkdir -p build/r2fix
git archive b49031e hadoop-bam_amd/csrc include | tar -x -C build/r2fix
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
F="-O3 -std=c++17 -fPIC -shared --offload-arch=gfx950"
$HIPCC $F -DHBAM_PROF -DHBAM_TOK_PRED=1 -Ibuild/r2fix/include -o hadoop-bam_amd/libhbam_r2fix_prof.so \
  build/r2fix/hadoop-bam_amd/csrc/hbam_capi.hip
$HIPCC $F -DHBAM_PROF -Iinclude -o hadoop-bam_amd/libhbam_prof.so hadoop-bam_amd/csrc/hbam_capi.hip
