#!/bin/bash
# GPU-box check: parity tests, smoke, bench, rocprof.  Ordinary failures (exit 1) continue to the
# next step; a timeout, abort, segfault or signal stops the script (nothing more touches the GPU).
# Env: STEPS="pytest smoke bench prof" selects steps; BENCH_ARGS / PROF_ARGS pass bench flags.
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 2
OUT="$R/gpurun_out"
mkdir -p "$OUT"
STEPS=${STEPS:-"pytest smoke bench prof"}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/steps.txt"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)" >> "$OUT/steps.txt"; exit $rc; fi
  return 0
}
: > "$OUT/steps.txt"
nproc > "$OUT/host.txt"; lscpu | grep -m1 "Model name" >> "$OUT/host.txt"
for s in $STEPS; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof)   (cd /tmp && export TMPDIR=/tmp && step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
               -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-baseline off ${PROF_ARGS:-}) || exit $? ;;
    pmc)    (cd /tmp && export TMPDIR=/tmp && \
             step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run \
               -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-baseline off ${PROF_ARGS:-} && \
             step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run \
               -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-baseline off ${PROF_ARGS:-}) || exit $? ;;
  esac
done
