#!/bin/bash
# 2 ranks on the box's single GPU (BZR_BENCH_DEVICE=0, gloo: RCCL refuses two ranks on one device):
# exercises bench.py's multi-rank path end to end -- strong-scaling tile deal, padded double-buffered
# gather to rank 0, max-over-ranks timing.  Not a scaling measurement.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
BZR_BENCH_BACKEND=gloo BZR_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-baseline off ${BENCH_ARGS:-} \
  > gpurun_out/rehearse2.log 2>&1
echo "rc=$?" >> gpurun_out/rehearse2.log
