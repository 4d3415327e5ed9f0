#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L="$GRAFT_REPO_ROOT/cuda-bezier-triangle-raytracer_amd/lib"
timeout -k 10 300 python scripts/exp_intersect.py > gpurun_out/v_default.log 2>&1 || exit $?
for v in ${VARIANTS:-it0 skip it8}; do
  BZR_LIBRARY=$L/exp_$v/libbzr.so timeout -k 10 300 python scripts/exp_intersect.py > gpurun_out/v_$v.log 2>&1 || exit $?
done
