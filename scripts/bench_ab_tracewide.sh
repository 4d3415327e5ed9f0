#!/bin/bash
# Interleaved bench.py lines of library builds (BZR_LIBRARY; "base" = lib/libbzr.so), on the GPU box.
# Env: RUN (output dir under gpurun_out), VARIANTS (default "base tracewide"), ROUNDS (default 2),
#      CONFIGS (default "cfg4"; each as "cfg:pipeline", pipeline optional), STEPS (default 100)
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${RUN:-.}"; mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CONFIGS:-cfg4}; do
    cfg=${c%%:*}; pipe=""; [ "$c" != "$cfg" ] && pipe="--pipeline ${c#*:}"
    for v in ${VARIANTS:-base tracewide}; do
      if [ "$v" = base ]; then unset BZR_LIBRARY; else export BZR_LIBRARY="$R/cuda-bezier-triangle-raytracer_amd/lib/$v/libbzr.so"; fi
      timeout -k 10 300 python bench.py --config $cfg $pipe --steps ${STEPS:-100} --cpu-baseline off \
        > "$OUT/bench_${cfg}_${v}_$r.log" 2>&1 || exit $?
      grep -h '^{' "$OUT/bench_${cfg}_${v}_$r.log" | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> "$OUT/bench_ab.jsonl"
    done
  done
done
