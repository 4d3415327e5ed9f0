#!/bin/bash
# round-3 session 2: cfg4 fused profile of the final tree (kernel trace + PMC passes)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c16"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
TAG=r03s2_cfg4_fused_v1 BENCH="--config cfg4" WORKLOAD=cfg4/fused/parity/4096 bash scripts/prof_run.sh; st prof4 $?
exit 0
