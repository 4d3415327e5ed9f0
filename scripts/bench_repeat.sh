#!/bin/bash
# The headline bench line repeated (default 5 runs, --cpu-baseline off) on one box: its run-to-run spread.
# GPU box; output gpurun_out/r05rep/repeat.jsonl
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r05rep"; mkdir -p "$OUT"; cd "$R" || exit 2
for k in $(seq 1 ${RUNS:-5}); do
  timeout -k 10 300 python bench.py --cpu-baseline off > "$OUT/b$k.log" 2>&1 || exit $?
  grep -h '^{' "$OUT/b$k.log" | sed "s/^{/{\"run\": $k, /" >> "$OUT/repeat.jsonl"
done
