#!/bin/bash
# round-3: register-pressure fix A/B (cfg4 vs the pre-wedge build, cfg5 vs the wedge-only build), bench, sustained
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03c4}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 300 python scripts/ab.py --config cfg4 --pipeline fused --rounds 5 --steps 10 prewedge base > "$OUT/ab_cfg4.txt" 2>&1; st ab_cfg4 $?
timeout -k 10 300 python scripts/ab.py --config cfg5 --pipeline fused --rounds 3 --steps 5 nobundle base > "$OUT/ab_cfg5_fused.txt" 2>&1; st ab_cfg5 $?
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; st bench $?
timeout -k 10 300 python scripts/sustained_clock.py --seconds 3 > "$OUT/sustained.json" 2> "$OUT/sustained.err"; st sustained $?
exit 0
