#!/bin/bash
# temporary A/B of k_traverse parts (variant bits: 1 = no histogram, 4 = no BVH walk)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in 0 1 4 5; do
  BZR_EXP_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/exp_$v.log 2>&1 || exit $?
done
