#!/bin/bash
# temporary A/B: default build vs lib/exp/libbzr.so, parity tests on the variant first
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
X="$GRAFT_REPO_ROOT/cuda-bezier-triangle-raytracer_amd/lib/exp/libbzr.so"
BZR_LIBRARY=$X timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/exp_pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline off > gpurun_out/exp_a.log 2>&1 || exit $?
BZR_LIBRARY=$X timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline off > gpurun_out/exp_b.log 2>&1 || exit $?
