#!/bin/bash
# The Newton site's issue ceiling on the GPU box (scripts/newton_ceiling.hip; build it first, in this container:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize \
#     -Icuda-bezier-triangle-raytracer_amd/csrc/device -Iinclude scripts/newton_ceiling.hip -o scripts/_bin/newton_ceiling)
# Outputs under gpurun_out/newton_ceiling: cfg4.jsonl / cfg5.jsonl (the probe's lines with cfg4's and cfg5's records),
# pmc.jsonl (scripts/newton_ceiling_pmc.py over a rocprofv3 kernel trace and one SQ counter pass of the cfg4 run).
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/newton_ceiling"; mkdir -p "$OUT"
BIN="$R/scripts/_bin/newton_ceiling"
trap 'rm -f "$R"/gpurun_out/nc_*.f32; find "$OUT" -name "*.db" -delete 2>/dev/null' EXIT
timeout -k 10 120 python3 "$R/scripts/newton_ceiling.py" > "$OUT/inputs.txt" || exit $?
N4=$(awk '/nc_cfg4/{print $2}' "$OUT/inputs.txt"); N5=$(awk '/nc_cfg5/{print $2}' "$OUT/inputs.txt")
timeout -k 10 120 "$BIN" "$R/gpurun_out/nc_cfg4.f32" $N4 ${PASSES:-64} > "$OUT/cfg4.jsonl" || exit $?
timeout -k 10 120 "$BIN" "$R/gpurun_out/nc_cfg5.f32" $N5 ${PASSES:-64} > "$OUT/cfg5.jsonl" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- "$BIN" "$R/gpurun_out/nc_cfg4.f32" $N4 ${PASSES:-64} \
  > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d "$OUT/sq1" -o run -- "$BIN" "$R/gpurun_out/nc_cfg4.f32" $N4 ${PASSES:-64} \
  > "$OUT/sq1.log" 2>&1 || exit $?
find "$OUT" -name "*.db" | head -5 > "$OUT/dbs.txt"
timeout -k 10 120 python3 "$R/scripts/newton_ceiling_pmc.py" "$OUT" > "$OUT/pmc.jsonl" 2> "$OUT/pmc.err"
