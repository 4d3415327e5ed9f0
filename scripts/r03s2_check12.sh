#!/bin/bash
# round-3 session 2: staged profiles of the final k_traverse (bundle walk + leaf pre-test + leaf pairs)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c12"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
TAG=r03s2_cfg5_staged_v2 BENCH="--config cfg5 --pipeline staged" WORKLOAD=cfg5/staged/parity/8192 STEPS=3 bash scripts/prof_run.sh; st prof5 $?
TAG=r03s2_cfg3_staged_v2 BENCH="--config cfg3 --pipeline staged" WORKLOAD=cfg3/staged/parity/2048 bash scripts/prof_run.sh; st prof3 $?
cd "$R" && timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_fused.py -x -q -m gpu -p no:cacheprovider --timeout 130 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
exit 0
