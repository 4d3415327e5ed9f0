#!/bin/bash
# 2 ranks on the box's single GPU (BZR_BENCH_DEVICE=0): exercises bench.py's RCCL path end to end.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
BZR_BENCH_BACKEND=gloo BZR_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --cpu-baseline off \
  > gpurun_out/rehearse2.log 2>&1
echo "rc=$?" >> gpurun_out/rehearse2.log
