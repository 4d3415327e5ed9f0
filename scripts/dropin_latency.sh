#!/bin/bash
# Build tests/cpp/dropin_test.cpp (as tests/test_cpp_dropin.py does) and run it on the GPU box: its output
# has the host single-ray vs GPU batch-of-one latencies per call.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
OUT="$R/gpurun_out/${RUN:-.}"; mkdir -p "$OUT"
P="$R/cuda-bezier-triangle-raytracer_amd"
g++ -O2 -std=c++17 -ffp-contract=off tests/cpp/dropin_test.cpp -Iinclude/bzr -Iinclude -Ioracle -L"$P/lib" -lbzr \
  -Loracle -loracle -Wl,-rpath,"$P/lib" -Wl,-rpath,"$R/oracle" -o "$OUT/dropin_test" && timeout -k 10 300 "$OUT/dropin_test"
