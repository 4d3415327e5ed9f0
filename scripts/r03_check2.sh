#!/bin/bash
# round-3: wedge pre-test A/B on cfg5 (both pipelines) + full-size cfg5 brute-force parity + stack4 variant
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03c2"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 300 python scripts/ab.py --config cfg5 --pipeline staged --rounds 3 --steps 5 prewedge base > "$OUT/ab_cfg5_staged.txt" 2>&1; st ab_staged $?
timeout -k 10 300 python scripts/ab.py --config cfg5 --pipeline fused --rounds 3 --steps 5 prewedge base > "$OUT/ab_cfg5_fused.txt" 2>&1; st ab_fused $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_variants.py -v -m gpu -k "cfg5_full or tiny" \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
exit 0
