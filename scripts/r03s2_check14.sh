#!/bin/bash
# round-3 session 2: final-tree GPU suite + smoke + cfg4 bench; k_trace fetching a node's leaves in pairs (tpairs)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c14"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 240 python bench.py > "$OUT/bench_cfg4.json" 2> "$OUT/bench_cfg4.err"; st bench4 $?
timeout -k 10 240 python scripts/ab.py --config cfg4 --rounds 9 --steps 10 base tpairs > "$OUT/ab_cfg4.jsonl" 2> "$OUT/ab_cfg4.err"; st ab4 $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --rounds 9 --steps 20 base tpairs > "$OUT/ab_cfg2.jsonl" 2> "$OUT/ab_cfg2.err"; st ab2 $?
exit 0
