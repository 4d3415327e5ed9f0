#!/bin/bash
# GPU-box check: the one entry point for GPU runs (rounds 1-3's one-off scripts/r03*_check*.sh were folded
# into these steps; git history keeps them).  Ordinary failures (exit 1) continue to the next step; a
# timeout, abort, segfault or signal stops the script (nothing more touches the GPU).
# Env:
#   STEPS="pytest smoke bench ..." selects steps (default: pytest smoke bench prof)
#   RUN=name       output directory gpurun_out/$RUN (default gpurun_out)
#   BENCH_ARGS     bench.py flags of the bench / rehearse2 steps
#   PYTEST_K       pytest -k expression of the pytest step (e.g. "tiled or dropin")
#   PYTEST_ARGS    other extra pytest args of the pytest step
#   PROF_TAG, PROF_BENCH, PROF_WORKLOAD   the prof step: scripts/prof_run.sh (kernel trace + PMC passes)
#   AB_ARGS, AB2_ARGS, AB3_ARGS   the ab / ab2 / ab3 steps: scripts/ab.py arguments
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 2
OUT="$R/gpurun_out/${RUN:-.}"
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
    pytest) step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 \
              --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-} ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    # 2 ranks on the box's one GPU, launched by bench.py itself (no torch.distributed.run): gloo, every rank
    # on device 0 (RCCL refuses two ranks on one device).  Exercises the launcher, the tile deal and the
    # per-frame gather; not a scaling measurement.
    rehearse2) step rehearse2 300 env BZR_BENCH_BACKEND=gloo BZR_BENCH_DEVICE=0 python bench.py --gpus 2 --steps 5 \
              --warmup 2 --cpu-baseline off ${BENCH_ARGS:-} ;;
    prof)   step prof 1500 env TAG="${PROF_TAG:-prof}" BENCH="${PROF_BENCH:-}" WORKLOAD="${PROF_WORKLOAD:-}" \
              bash scripts/prof_run.sh ;;
    dropin) step dropin 400 bash scripts/dropin_latency.sh ;;
    # the C++ host path (tests/cpp/tiled_bench.cpp: bzr::TiledChain frames on device outputs);
    # CPPBENCH_ARGS e.g. "--host-frames 3"; appends its JSON line to cppbench.jsonl
    cppbench) step cppbench_build 180 g++ -O2 -std=c++17 -ffp-contract=off -D__HIP_PLATFORM_AMD__ tests/cpp/tiled_bench.cpp \
              -Iinclude/bzr -Iinclude -I/opt/rocm/include -Lcuda-bezier-triangle-raytracer_amd/lib -lbzr -L/opt/rocm/lib \
              -lamdhip64 -Wl,-rpath,"$R/cuda-bezier-triangle-raytracer_amd/lib" -Wl,-rpath,/opt/rocm/lib -o /tmp/tiled_bench &&
              step cppbench 300 /tmp/tiled_bench ${CPPBENCH_ARGS:-} &&
              grep -h '^{' "$OUT/cppbench.log" >> "$OUT/cppbench.jsonl" ;;
    # bench lines of the other configs on both pipelines (bench defaults, 100 timed steps): configs.jsonl
    configs) for c in cfg5 cfg3 cfg2; do for p in staged fused; do
               step "configs_${c}_$p" 300 python bench.py --config $c --pipeline $p --steps 100 --cpu-baseline off &&
               grep -h '^{' "$OUT/configs_${c}_$p.log" >> "$OUT/configs.jsonl"
             done; done ;;
    ab)     step ab 900 python scripts/ab.py ${AB_ARGS:-} ;;
    ab2)    step ab2 900 python scripts/ab.py ${AB2_ARGS:-} ;;
    ab3)    step ab3 900 python scripts/ab.py ${AB3_ARGS:-} ;;
    # the far-origin overflow count of the default and the bundle-walk builds
    bundleprobe) step bundleprobe_base 300 python scripts/bundle_overflow_probe.py &&
              step bundleprobe_bundle 300 env BZR_LIBRARY="$R/cuda-bezier-triangle-raytracer_amd/lib/tracebundle/libbzr.so" \
                python scripts/bundle_overflow_probe.py ;;
  esac
done
