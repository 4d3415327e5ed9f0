#!/bin/bash
# rocprofv3 kernel trace of scripts/aos_probe.py (the record-layout conversion kernels at the bench frame size);
# summary in gpurun_out/r05aosprof/summary.txt (GPU box)
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r05aosprof"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
trap 'find "$OUT" -name "*.db" -delete 2>/dev/null' EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/scripts/aos_probe.py" > "$OUT/probe.log" 2>&1 &&
timeout -k 10 120 python3 "$R/scripts/prof_summary.py" "$OUT" "$OUT/summary.txt" --note "rocprofv3 over scripts/aos_probe.py" \
  > "$OUT/summary.log" 2>&1
