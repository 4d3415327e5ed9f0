#!/bin/bash
# round-3 session 2: the default build (k_traverse bundle walk on): GPU suite, smoke, the cfg4 bench line and
# bench lines of cfg5 / cfg3 / cfg2 on the staged and fused pipelines (bench defaults).
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03s2c5}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 240 python bench.py > "$OUT/bench_cfg4.json" 2> "$OUT/bench_cfg4.err"; st bench4 $?
for spec in "cfg5 staged" "cfg3 staged" "cfg5 fused" "cfg3 fused" "cfg2 fused" "cfg2 staged"; do
  set -- $spec
  timeout -k 10 240 python bench.py --config "$1" --pipeline "$2" --cpu-baseline off > "$OUT/bench_$1_$2.json" 2> "$OUT/bench_$1_$2.err"; st "bench_$1_$2" $?
done
exit 0
