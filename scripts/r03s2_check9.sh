#!/bin/bash
# round-3 session 2: k_traverse with the wave-level leaf pre-test (BZR_TRAV_PRETEST) vs without
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c9"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 200 python scripts/ab.py --config cfg5 --pipeline staged --rounds 5 --steps 3 base pretest > "$OUT/ab_cfg5s.jsonl" 2> "$OUT/ab_cfg5s.err"; st ab5s $?
timeout -k 10 200 python scripts/ab.py --config cfg3 --pipeline staged --rounds 7 --steps 10 base pretest > "$OUT/ab_cfg3s.jsonl" 2> "$OUT/ab_cfg3s.err"; st ab3s $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --pipeline staged --rounds 7 --steps 20 base pretest > "$OUT/ab_cfg2s.jsonl" 2> "$OUT/ab_cfg2s.err"; st ab2s $?
BZR_LIBRARY="$R/cuda-bezier-triangle-raytracer_amd/lib/pretest/libbzr.so" timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_pretest.log" 2>&1; st pytest_pretest $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -x -v -m gpu -p no:cacheprovider --timeout 130 --timeout-method thread > "$OUT/pytest_variants.log" 2>&1; st pytest_variants $?
exit 0
