#!/bin/bash
# round-3: slim staged pair records -- A/B vs the previous build on cfg5/cfg3/cfg2 staged, staged parity tests,
# PMC traffic of cfg5 staged, and the tile-order probe (true dealing order)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03c5}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
for c in cfg5 cfg3 cfg2; do
  timeout -k 10 300 python scripts/ab.py --config $c --pipeline staged --rounds 3 --steps 5 prepairs base > "$OUT/ab_${c}_staged.txt" 2>&1; st "ab $c" $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_golden.py tests/test_gpu_fused.py -x -v -m gpu \
  -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python scripts/tile_order_probe.py > "$OUT/tile_order_probe.log" 2> "$OUT/probe.err"; st probe $?
TAG=r03_cfg5_staged_v2 BENCH="--config cfg5 --pipeline staged" WORKLOAD=cfg5/staged/parity/8192 bash scripts/prof_run.sh; st prof $?
exit 0
