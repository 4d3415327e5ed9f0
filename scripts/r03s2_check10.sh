#!/bin/bash
# round-3 session 2: k_trace with plane-window nodes (BZR_NODE_WIN) vs default; illumination with the
# bundle-walk k_traverse (default) vs the per-lane walk (dfs build)
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/r03s2c10"; mkdir -p "$OUT"
st() { echo "$1 rc=$2" >> "$OUT/steps.txt"; [ "$2" -ge 124 ] && exit "$2"; return 0; }
timeout -k 10 240 python scripts/ab.py --config cfg4 --rounds 9 --steps 10 base win > "$OUT/ab_cfg4.jsonl" 2> "$OUT/ab_cfg4.err"; st ab4 $?
timeout -k 10 200 python scripts/ab.py --config cfg2 --rounds 9 --steps 20 base win > "$OUT/ab_cfg2.jsonl" 2> "$OUT/ab_cfg2.err"; st ab2 $?
timeout -k 10 200 python scripts/ab.py --config cfg3 --rounds 5 --steps 10 base win > "$OUT/ab_cfg3.jsonl" 2> "$OUT/ab_cfg3.err"; st ab3 $?
timeout -k 10 200 python scripts/ab.py --config cfg5 --rounds 3 --steps 3 base win > "$OUT/ab_cfg5.jsonl" 2> "$OUT/ab_cfg5.err"; st ab5 $?
timeout -k 10 200 python scripts/bench_illum.py > "$OUT/illum_base.json" 2> "$OUT/illum_base.err"; st illum_base $?
BZR_LIBRARY="$R/cuda-bezier-triangle-raytracer_amd/lib/dfs/libbzr.so" timeout -k 10 200 python scripts/bench_illum.py > "$OUT/illum_dfs.json" 2> "$OUT/illum_dfs.err"; st illum_dfs $?
timeout -k 10 200 python scripts/bench_illum.py > "$OUT/illum_base2.json" 2> "$OUT/illum_base2.err"; st illum_base2 $?
exit 0
