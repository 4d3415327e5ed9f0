#!/bin/bash
# round-3 session 2: GPU tests + smoke + bench of HEAD, then in-process A/B of walk/pass latency variants
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03s2c1}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 200 python scripts/ab.py --config cfg4 --rounds 7 --steps 10 base nodeasm passflat pf7 both both7 > "$OUT/ab_cfg4.jsonl" 2> "$OUT/ab_cfg4.err"; st ab4 $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --rounds 7 --steps 20 base nodeasm passflat pf7 both both7 > "$OUT/ab_cfg2.jsonl" 2> "$OUT/ab_cfg2.err"; st ab2 $?
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; st bench $?
exit 0
