#!/bin/bash
# A/B builds at bench level (frames in flight): each build in LIBS ("base" = the in-tree lib/libbzr.so, else
# lib/<name>/libbzr.so through BZR_LIBRARY) runs `bench.py --config $CONFIG --pipeline $PIPE`, REPS interleaved
# rounds; one JSON line per run into gpurun_out/lib_sweep.jsonl.  Each run has its own time limit; a timeout
# or crash stops the sweep.
# ENVS: environment settings run per build ("-" = none), e.g. ENVS="- BZR_BENCH_SLOT_PRIO=lead".
#   CONFIG=cfg5 PIPE=staged LIBS="base travprio3" REPS=3 bash scripts/lib_sweep.sh
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
OUT=gpurun_out/lib_sweep.jsonl
: > "$OUT"
L=cuda-bezier-triangle-raytracer_amd/lib
for r in $(seq ${REPS:-2}); do
  for c in ${CONFIGS:-${CONFIG:-cfg5}}; do
    for v in ${LIBS:-base}; do
     for e in ${ENVS:--}; do
      if [ "$v" = base ]; then lib="$L/libbzr.so"; else lib="$L/$v/libbzr.so"; fi
      if [ "$e" = - ]; then ev=""; else ev="$e"; fi
      env $ev BZR_LIBRARY="$PWD/$lib" timeout -k 10 240 python bench.py --config "$c" --pipeline "${PIPE:-staged}" \
        --cpu-baseline off ${BENCH_ARGS:-} > gpurun_out/lib_sweep_one.log 2>&1 || exit $?
      grep '^{' gpurun_out/lib_sweep_one.log | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'config': '$c', 'pipeline': '${PIPE:-staged}', 'lib': '$v', 'env': '$e', 'rep': $r, 'mrays_s': d['value'],
                  'ms_per_step': d['ms_per_step'], 'steps': d['steps'],
                  'inflight': d['config'].get('frames_in_flight')}))" >> "$OUT"
      tail -1 "$OUT"
     done
    done
  done
done
