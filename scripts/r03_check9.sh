#!/bin/bash
# round-3: one rank's loop at N-rank frame sizes (packing cost), the bench with its pre-warm, and the
# 2-rank gloo rehearsal of the bench loop (compact gather) on the single GPU
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03c9b}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 300 python scripts/rank_loop_probe.py > "$OUT/rank_loop.jsonl" 2> "$OUT/rank_loop.err"; st rankloop $?
timeout -k 10 300 python bench.py --cpu-baseline off > "$OUT/bench.json" 2> "$OUT/bench.err"; st bench $?
BZR_BENCH_BACKEND=gloo BZR_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 --cpu-baseline off --gather compact \
  > "$OUT/rehearse2_compact.json" 2> "$OUT/rehearse2.err"; st rehearse $?
exit 0
