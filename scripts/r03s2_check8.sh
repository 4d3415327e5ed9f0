#!/bin/bash
# round-3 session 2: k_trace with the bundle walk (lane index laundered: 74 VGPRs / 6 waves; bundle7 at
# waves_per_eu(7): 72 VGPRs, 7 waves) against the per-lane walk; the default build's staged lines.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c8"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 240 python scripts/ab.py --config cfg4 --rounds 9 --steps 10 base bundle bundle7 > "$OUT/ab_cfg4.jsonl" 2> "$OUT/ab_cfg4.err"; st ab4 $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --rounds 9 --steps 20 base bundle bundle7 > "$OUT/ab_cfg2.jsonl" 2> "$OUT/ab_cfg2.err"; st ab2 $?
timeout -k 10 200 python scripts/ab.py --config cfg3 --rounds 5 --steps 10 base bundle bundle7 > "$OUT/ab_cfg3.jsonl" 2> "$OUT/ab_cfg3.err"; st ab3 $?
timeout -k 10 200 python scripts/ab.py --config cfg5 --rounds 3 --steps 3 base bundle bundle7 > "$OUT/ab_cfg5.jsonl" 2> "$OUT/ab_cfg5.err"; st ab5 $?
exit 0
