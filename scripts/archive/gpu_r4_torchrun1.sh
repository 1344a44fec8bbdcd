#!/bin/bash
# The driver's launcher at N = 1: torch.distributed.run around bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_torchrun1.json 2> gpurun_out/r4_torchrun1.err
