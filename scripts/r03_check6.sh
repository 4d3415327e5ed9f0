#!/bin/bash
# round-3 final-state check: whole GPU suite, smoke, bench, 4-queue bench, configs, cfg3/cfg2 staged profiles
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03c6}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; st bench $?
BZR_BENCH_HW_QUEUES=4 timeout -k 10 300 python bench.py --cpu-baseline off > "$OUT/bench_4queues.json" 2>> "$OUT/bench.err"; st bench4q $?
for c in "cfg2" "cfg2 --pipeline staged" "cfg3 --pipeline staged" "cfg3" "cfg5 --pipeline staged" "cfg5"; do
  timeout -k 10 300 python bench.py --config $c --cpu-baseline off >> "$OUT/configs.jsonl" 2>> "$OUT/configs.err"; st "cfg $c" $?
done
TAG=r03_cfg5_fused_v1 BENCH="--config cfg5 --pipeline fused" WORKLOAD=cfg5/fused/parity/8192 bash scripts/prof_run.sh; st prof5f $?
TAG=r03_cfg4_fused_v2 BENCH="--config cfg4 --pipeline fused" WORKLOAD=cfg4/fused/parity/4096 bash scripts/prof_run.sh; st prof4 $?
exit 0
