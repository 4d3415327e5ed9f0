#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
X="$GRAFT_REPO_ROOT/cuda-bezier-triangle-raytracer_amd/lib/exp/libbzr.so"
for v in 0 8 16 24; do
  BZR_EXP_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/exp_$v.log 2>&1 || exit $?
done
BZR_LIBRARY=$X timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/exp_it1.log 2>&1 || exit $?
