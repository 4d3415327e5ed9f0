#!/bin/bash
# One config and pipeline at several frames-in-flight counts, REPS interleaved rounds, bench defaults otherwise:
# one JSON line per run into gpurun_out/inflight_sweep.jsonl.  Each run has its own time limit; a timeout or crash
# stops the sweep.   CONFIG=cfg2 PIPE=fused INFLIGHTS="3 4 6" REPS=2 bash scripts/inflight_sweep.sh
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
OUT=gpurun_out/inflight_sweep.jsonl
: > "$OUT"
for r in $(seq ${REPS:-2}); do
  for f in ${INFLIGHTS:-3 4 6}; do
    timeout -k 10 240 python bench.py --config "${CONFIG:-cfg2}" --pipeline "${PIPE:-fused}" --inflight "$f" \
      --cpu-baseline off ${BENCH_ARGS:-} > gpurun_out/inflight_one.log 2>&1 || exit $?
    grep '^{' gpurun_out/inflight_one.log | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'config': '${CONFIG:-cfg2}', 'pipeline': '${PIPE:-fused}', 'inflight': $f, 'rep': $r, 'mrays_s': d['value'],
                  'ms_per_step': d['ms_per_step'], 'steps': d['steps']}))" >> "$OUT"
    tail -1 "$OUT"
  done
done
