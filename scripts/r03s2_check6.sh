#!/bin/bash
# round-3 session 2: rocprofv3 profiles (kernel trace + PMC passes) of cfg5 / cfg3 staged with the bundle-walk
# k_traverse, then an A/B of the chain kernel at waves_per_eu(7) (basew7) against the default.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c6"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
TAG=r03s2_cfg5_staged_v1 BENCH="--config cfg5 --pipeline staged" WORKLOAD=cfg5/staged/parity/8192 STEPS=3 bash scripts/prof_run.sh; st prof5 $?
TAG=r03s2_cfg3_staged_v1 BENCH="--config cfg3 --pipeline staged" WORKLOAD=cfg3/staged/parity/2048 bash scripts/prof_run.sh; st prof3 $?
cd "$R" && timeout -k 10 240 python scripts/ab.py --config cfg4 --rounds 9 --steps 10 base basew7 > "$OUT/ab_cfg4.jsonl" 2> "$OUT/ab_cfg4.err"; st ab4 $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --rounds 9 --steps 20 base basew7 > "$OUT/ab_cfg2.jsonl" 2> "$OUT/ab_cfg2.err"; st ab2 $?
exit 0
