#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pd
timeout -k 10 200 python -u tools/prof_deflate.py > gpurun_out/pd/prof.txt 2>&1
