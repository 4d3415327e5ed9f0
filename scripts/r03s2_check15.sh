#!/bin/bash
# round-3 session 2: cfg4 bench with 3 / 4 / 3 frames in flight (interleaved)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c15"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
for k in 3a 4a 3b 4b; do
  timeout -k 10 200 python bench.py --inflight ${k:0:1} --cpu-baseline off > "$OUT/bench_if$k.json" 2> "$OUT/bench_if$k.err"; st "if$k" $?
done
exit 0
