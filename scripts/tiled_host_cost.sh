#!/bin/bash
# The C++ multi-device plan's host cost per frame (tests/cpp/tiled_bench.cpp host_enqueue_ms_per_frame) at 1, 2, 4
# and 8 list devices, all on the box's one GPU (--one-gpu: peer transport, every share traced on device 0), so the
# per-frame launch and copy calls one host thread queues for an N-device frame are timed beside the GPU frame.
# GPU box; output gpurun_out/r05host/host_cost.jsonl
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r05host"; mkdir -p "$OUT"; cd "$R" || exit 2
g++ -O2 -std=c++17 -ffp-contract=off -D__HIP_PLATFORM_AMD__ tests/cpp/tiled_bench.cpp -Iinclude/bzr -Iinclude \
  -I/opt/rocm/include -Lcuda-bezier-triangle-raytracer_amd/lib -lbzr -L/opt/rocm/lib -lamdhip64 \
  -Wl,-rpath,"$R/cuda-bezier-triangle-raytracer_amd/lib" -Wl,-rpath,/opt/rocm/lib -o /tmp/tiled_bench || exit 1
for d in 1 2 4 8; do
  timeout -k 10 180 /tmp/tiled_bench --frames 50 --devices $d --one-gpu > "$OUT/d$d.log" 2>&1 || exit $?
  grep -h '^{' "$OUT/d$d.log" >> "$OUT/host_cost.jsonl"
done
