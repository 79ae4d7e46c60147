#!/bin/bash
# N=2 rehearsal of bench.py's sharded path on the one-GPU box: two ranks on cuda:0, gloo
# collectives (the 8-GPU RCCL run is the driver's).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mr
export TMPDIR=/tmp HBAM_BENCH_BACKEND=gloo LOCAL_RANK_OVERRIDE=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/bench_rank0gpu.py --gpus 2 --steps 2 --warmup 1 --size 1e9 --parity-splits 4 --no-cpu-baseline > gpurun_out/mr/bench2.json 2> gpurun_out/mr/bench2.err
