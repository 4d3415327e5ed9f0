#!/bin/bash
# round-3 session 2: A/B of the bundle walk (BZR_TRACE_BUNDLE), the paired node loads and the branch-free
# pass, then the GPU parity suite on the bundle-walk build (BZR_LIBRARY), then smoke + bench of the default.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03s2c2}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 200 python scripts/ab.py --config cfg4 --rounds 7 --steps 10 base bundle nodeasm passflat > "$OUT/ab_cfg4.jsonl" 2> "$OUT/ab_cfg4.err"; st ab4 $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --rounds 7 --steps 20 base bundle nodeasm > "$OUT/ab_cfg2.jsonl" 2> "$OUT/ab_cfg2.err"; st ab2 $?
timeout -k 10 200 python scripts/ab.py --config cfg3 --rounds 5 --steps 10 base bundle > "$OUT/ab_cfg3.jsonl" 2> "$OUT/ab_cfg3.err"; st ab3 $?
timeout -k 10 200 python scripts/ab.py --config cfg5 --rounds 3 --steps 3 base bundle > "$OUT/ab_cfg5.jsonl" 2> "$OUT/ab_cfg5.err"; st ab5 $?
BZR_LIBRARY="$R/cuda-bezier-triangle-raytracer_amd/lib/bundle/libbzr.so" timeout -k 10 700 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread --deselect tests/test_gpu_variants.py > "$OUT/pytest_bundle.log" 2>&1; st pytest_bundle $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; st smoke $?
exit 0
