#!/bin/bash
# round-3 session 2: k_traverse fetching queued leaves in pairs (BZR_TRAV_LEAF_PAIRS) vs one at a time
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c7"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 200 python scripts/ab.py --config cfg5 --pipeline staged --rounds 5 --steps 3 base pairs > "$OUT/ab_cfg5s.jsonl" 2> "$OUT/ab_cfg5s.err"; st ab5s $?
timeout -k 10 200 python scripts/ab.py --config cfg3 --pipeline staged --rounds 7 --steps 10 base pairs > "$OUT/ab_cfg3s.jsonl" 2> "$OUT/ab_cfg3s.err"; st ab3s $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --pipeline staged --rounds 7 --steps 20 base pairs > "$OUT/ab_cfg2s.jsonl" 2> "$OUT/ab_cfg2s.err"; st ab2s $?
exit 0
