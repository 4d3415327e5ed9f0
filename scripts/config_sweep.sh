#!/bin/bash
# bench.py over the BASELINE configs x pipelines x frames in flight (1 GPU, parity): one JSON line each
# into gpurun_out/config_sweep.jsonl.  Every run has its own time limit; a timeout or crash stops the sweep.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
OUT=gpurun_out/config_sweep.jsonl
: > "$OUT"
for spec in "cfg2 fused" "cfg2 staged" "cfg3 fused" "cfg3 staged" "cfg4 fused" "cfg4 staged" "cfg5 fused" "cfg5 staged"; do
  set -- $spec
  for f in ${INFLIGHTS:-1 2 3}; do
    timeout -k 10 240 python bench.py --config "$1" --pipeline "$2" --inflight "$f" --steps ${STEPS:-10} --warmup 2 \
      --cpu-baseline off > gpurun_out/sweep_one.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "{\"config\": \"$1\", \"pipeline\": \"$2\", \"inflight\": $f, \"rc\": $rc}" >> "$OUT"; [ $rc -ge 124 ] && exit $rc; continue; fi
    grep '^{' gpurun_out/sweep_one.log | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'config': '$1', 'pipeline': '$2', 'inflight': $f, 'mrays_s': d['value'], 'ms_per_step': d['ms_per_step'],
                  'segments_per_step': d['config']['segments_per_step'], 'kernels': {k: v['ms_per_step'] for k, v in d['roofline']['per_kernel'].items()}}))" >> "$OUT"
  done
done
