#!/bin/bash
# round-3 session 2: the bundle walk with the stack-room rule, 128-entry chain stack and the per-lane walk for
# wide bundles (bundle / bundlew7 / bundlenar = no wide fallback), all configs and both pipelines; then the
# GPU suite on the bundle build.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03s2c4}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 240 python scripts/ab.py --config cfg4 --rounds 7 --steps 10 base bundle bundlew7 bundlenar > "$OUT/ab_cfg4.jsonl" 2> "$OUT/ab_cfg4.err"; st ab4 $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --rounds 7 --steps 20 base bundle bundlew7 bundlenar > "$OUT/ab_cfg2.jsonl" 2> "$OUT/ab_cfg2.err"; st ab2 $?
timeout -k 10 200 python scripts/ab.py --config cfg3 --rounds 5 --steps 10 base bundle bundlenar > "$OUT/ab_cfg3.jsonl" 2> "$OUT/ab_cfg3.err"; st ab3 $?
timeout -k 10 200 python scripts/ab.py --config cfg5 --rounds 3 --steps 3 base bundle > "$OUT/ab_cfg5.jsonl" 2> "$OUT/ab_cfg5.err"; st ab5 $?
timeout -k 10 200 python scripts/ab.py --config cfg5 --pipeline staged --rounds 3 --steps 3 base bundle > "$OUT/ab_cfg5s.jsonl" 2> "$OUT/ab_cfg5s.err"; st ab5s $?
timeout -k 10 200 python scripts/ab.py --config cfg3 --pipeline staged --rounds 5 --steps 10 base bundle > "$OUT/ab_cfg3s.jsonl" 2> "$OUT/ab_cfg3s.err"; st ab3s $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --pipeline staged --rounds 5 --steps 20 base bundle > "$OUT/ab_cfg2s.jsonl" 2> "$OUT/ab_cfg2s.err"; st ab2s $?
BZR_LIBRARY="$R/cuda-bezier-triangle-raytracer_amd/lib/bundle/libbzr.so" timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread --deselect tests/test_gpu_variants.py > "$OUT/pytest_bundle.log" 2>&1; st pytest_bundle $?
exit 0
