#!/bin/bash
# bench.py cfg4 at 1..4 frames in flight, two rounds interleaved (GPU box; output gpurun_out/r05l/inflight.jsonl)
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r05l"; mkdir -p "$OUT"; cd "$R"
for r in 1 2; do for f in 1 2 3 4; do
  timeout -k 10 300 python bench.py --inflight $f --steps 100 --cpu-baseline off > "$OUT/b_${f}_$r.log" 2>&1 || exit $?
  grep -h '^{' "$OUT/b_${f}_$r.log" | sed "s/^{/{\"inflight\": $f, \"round\": $r, /" >> "$OUT/inflight.jsonl"
done; done
