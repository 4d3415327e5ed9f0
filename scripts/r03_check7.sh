#!/bin/bash
# round-3: staged knob A/B (k_newton occupancy, k_traverse block) on cfg5/cfg3 + the always-list stress test
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03c7}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -v -m gpu -k "open_wedges" -p no:cacheprovider --timeout 200 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
for c in cfg5 cfg3; do
  timeout -k 10 300 python scripts/ab.py --config $c --pipeline staged --rounds 3 --steps 5 base nwpe6 nwpe7 trav128 > "$OUT/ab_${c}.txt" 2>&1; st "ab $c" $?
done
exit 0
