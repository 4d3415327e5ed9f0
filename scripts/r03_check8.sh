#!/bin/bash
# round-3: intersect-kernel parking A/B on cfg5/cfg3 fused (+ parity of the variant on the intersect tests)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03c8}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
for c in cfg5 cfg3; do
  timeout -k 10 300 python scripts/ab.py --config $c --pipeline fused --rounds 3 --steps 5 base parkhits > "$OUT/ab_${c}_fused.txt" 2>&1; st "abf $c" $?
done
BZR_LIBRARY="$R/cuda-bezier-triangle-raytracer_amd/lib/parkhits/libbzr.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py tests/test_golden.py -x -v -m gpu -k "fused" -p no:cacheprovider --timeout 200 --timeout-method thread \
  > "$OUT/pytest_parkhits.log" 2>&1; st pytest $?
exit 0
