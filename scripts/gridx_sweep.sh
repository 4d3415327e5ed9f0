#!/bin/bash
# Persistent staged kernels' grid (BZR_NEWTON_GRIDX / BZR_RESOLVE_BLOCKS: multiples of the resident capacity / k_resolve blocks) at
# bench level, frames in flight: one JSON line per run into gpurun_out/gridx_sweep.jsonl, REPS interleaved rounds.
# Each run has its own time limit; a timeout or crash stops the sweep.
#   CONFIG=cfg5 PIPE=staged GRIDS="1:1024 2:1024 2:512" INFLIGHTS="2 3" REPS=2 bash scripts/gridx_sweep.sh
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
OUT=gpurun_out/gridx_sweep.jsonl
: > "$OUT"
for r in $(seq ${REPS:-2}); do
  for f in ${INFLIGHTS:-2}; do
    for g in ${GRIDS:-1:1024 2:1024}; do
      ng=${g%%:*}; rg=${g##*:}
      BZR_NEWTON_GRIDX=$ng BZR_RESOLVE_BLOCKS=$rg timeout -k 10 240 python bench.py --config "${CONFIG:-cfg5}" \
        --pipeline "${PIPE:-staged}" --inflight "$f" --cpu-baseline off ${BENCH_ARGS:-} > gpurun_out/gridx_one.log 2>&1 || exit $?
      grep '^{' gpurun_out/gridx_one.log | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'config': '${CONFIG:-cfg5}', 'pipeline': '${PIPE:-staged}', 'inflight': $f, 'newton_gridx': $ng,
                  'resolve_blocks': $rg, 'rep': $r, 'mrays_s': d['value'], 'ms_per_step': d['ms_per_step'],
                  'steps': d['steps'], 'verified': d.get('frame_verified')}))" >> "$OUT"
      tail -1 "$OUT"
    done
  done
done
