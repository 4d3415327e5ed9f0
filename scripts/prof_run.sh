#!/bin/bash
# rocprofv3 passes over bench.py on the GPU box: kernel-trace stats, FETCH_SIZE, WRITE_SIZE and two SQ
# counter sets, each in its own run (PMC passes with --kernel-trace only).  Output under gpurun_out/$TAG.
# usage: TAG=name BENCH="--config cfg4 ..." [WORKLOAD=cfg4/fused/parity/4096] bash scripts/prof_run.sh
# The rocprofv3 databases are summarised on the box (scripts/prof_summary.py -> $TAG/summary.txt and
# $TAG/pmc_traffic.json) and then deleted, so the pulled gpurun_out/ stays small.
if [ -z "$GRAFT_REPO_ROOT" ] || [ ! -f "$GRAFT_REPO_ROOT/bench.py" ]; then
  echo "prof_run.sh: GRAFT_REPO_ROOT must name the repo root (the GPU box exports it)" >&2
  echo "usage: TAG=name BENCH=\"--config cfg4 ...\" [WORKLOAD=cfg4/fused/parity/4096] bash scripts/prof_run.sh" >&2
  exit 2
fi
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${TAG:-prof}"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
# the rocprofv3 databases are large: delete them however the script ends, or a failed pass leaves them behind and
# the pulled gpurun_out/ outgrows gpurun's merge limit (round 4's "prof rc=2 with an empty prof.log": the passes'
# own logs, under $OUT, never came back)
trap 'find "$OUT" -name "*.db" -delete 2>/dev/null' EXIT
echo "prof_run.sh: outputs under $OUT (each pass: <name>.log; summary.txt)"
# --inflight 1: each launch runs alone, so the trace's per-launch durations compare with bench.py's
# roofline.avg_launch_ms (measured on serialized launches); with two frames in flight the launches overlap.
B="$R/bench.py --steps ${PROF_STEPS:-5} --warmup 1 --prewarm-s 0.3 --cpu-baseline off --inflight 1 ${BENCH:-}"
run() {  # run <name> <rocprof args...>
  local name=$1; shift
  echo "prof_run.sh: $name: rocprofv3 $*"
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run -- python3 $B > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ]; then echo "prof_run.sh: $name failed (rc=$rc); the tail of $OUT/$name.log:"; tail -n 20 "$OUT/$name.log"; fi
  return $rc
}
run trace --kernel-trace --stats &&
run fetch --pmc FETCH_SIZE --kernel-trace &&
run write --pmc WRITE_SIZE --kernel-trace &&
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace &&
run sq2 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM SQ_INSTS_LDS SQ_LEVEL_WAVES --kernel-trace &&
timeout -k 10 120 python3 "$R/scripts/prof_summary.py" "$OUT" "$OUT/summary.txt" --note "rocprofv3 over bench.py ${BENCH:-} (steps ${PROF_STEPS:-5})" \
  --traffic-json "$OUT/pmc_traffic.json" --workload "${WORKLOAD:-$TAG}" --source "profiles/${TAG:-prof}.txt" > "$OUT/summary.log" 2>&1 &&
find "$OUT" -name "*.db" -delete
