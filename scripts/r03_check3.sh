#!/bin/bash
# round-3 milestone check: whole GPU suite, smoke, bench (driver default), 2-rank compact-gather rehearsal,
# sustained-clock run, per-config bench lines.  Every GPU step under its own timeout; stop on a hang/crash.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03c3}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
for s in ${STEPS:-ab pytest smoke bench rehearse sustained configs}; do
case $s in
ab) for p in staged fused; do timeout -k 10 300 python scripts/ab.py --config cfg5 --pipeline $p --rounds 3 --steps 5 ${AB:-nobundle base} \
      > "$OUT/ab_cfg5_$p.txt" 2>&1; st "ab $p" $?; done ;;
pytest) timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
          > "$OUT/pytest.log" 2>&1; st pytest $? ;;
smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; st smoke $? ;;
bench) timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; st bench $? ;;
rehearse) BZR_BENCH_BACKEND=gloo BZR_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
          --cpu-baseline off --gather compact > "$OUT/rehearse_compact.json" 2> "$OUT/rehearse_compact.err"; st rehearse $? ;;
sustained) timeout -k 10 300 python scripts/sustained_clock.py --seconds 3 > "$OUT/sustained.json" 2> "$OUT/sustained.err"; st sustained $?
          timeout -k 10 300 python bench.py --steps 450 --cpu-baseline off > "$OUT/bench_450.json" 2>> "$OUT/sustained.err"; st bench450 $? ;;
configs) for c in "cfg2" "cfg2 --pipeline staged" "cfg3 --pipeline staged" "cfg3" "cfg5 --pipeline staged" "cfg5"; do
           timeout -k 10 300 python bench.py --config $c --cpu-baseline off >> "$OUT/configs.jsonl" 2>> "$OUT/configs.err"; st "cfg $c" $?
         done ;;
esac
done
exit 0
