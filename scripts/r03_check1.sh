#!/bin/bash
# round-3 check: new full-size brute-force parity tests, parity suite, cfg4/cfg5 bench lines
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03c1"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_variants.py tests/test_gpu_parity.py -x -v -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/steps.txt"; [ $rc -ge 124 ] && exit $rc
for c in "cfg4" "cfg5 --pipeline fused" "cfg5 --pipeline staged"; do
  timeout -k 10 300 python bench.py --config $c --cpu-baseline off >> "$OUT/bench.jsonl" 2>> "$OUT/bench.err"
  rc=$?; echo "bench $c rc=$rc" >> "$OUT/steps.txt"; [ $rc -ge 124 ] && exit $rc
done
exit 0
