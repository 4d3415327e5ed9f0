#!/bin/bash
# bench.py cfg5 staged at 2, 3 and 4 frames in flight, two rounds interleaved (GPU box; gpurun_out/r05if5/inflight.jsonl)
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r05if5"; mkdir -p "$OUT"; cd "$R" || exit 2
for r in 1 2; do for f in 2 3 4; do
  timeout -k 10 300 python bench.py --config cfg5 --pipeline staged --inflight $f --steps 60 --cpu-baseline off \
    > "$OUT/b_${f}_$r.log" 2>&1 || exit $?
  grep -h '^{' "$OUT/b_${f}_$r.log" | sed "s/^{/{\"inflight\": $f, \"round\": $r, /" >> "$OUT/inflight.jsonl"
done; done
