R="$GRAFT_REPO_ROOT"; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
STEPS="pytest smoke bench" bash scripts/gpu_check.sh
cd "$R" && timeout -k 10 300 python bench.py --accel none --steps 5 --cpu-baseline off > "$OUT/bench_none.log" 2>&1
echo "bench_none rc=$?" >> "$OUT/steps.txt"
