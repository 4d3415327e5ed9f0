#!/bin/bash
# round-3: bzr_pack_frame parity tests, one rank's loop at N-rank frame sizes (torch vs HIP packers), the
# 2-rank gloo rehearsal of bench.py's loop with the compact gather (HIP packer)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${TAG:-r03c11}"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame_pack.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; st pytest $?
[ -f "$OUT/steps.txt" ] && grep -q "pytest rc=0" "$OUT/steps.txt" || exit 1
timeout -k 10 300 python scripts/rank_loop_probe.py > "$OUT/rank_loop.jsonl" 2> "$OUT/rank_loop.err"; st rankloop $?
BZR_BENCH_BACKEND=gloo BZR_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 --cpu-baseline off --gather compact \
  > "$OUT/rehearse2_compact.json" 2> "$OUT/rehearse2.err"; st rehearse $?
exit 0
