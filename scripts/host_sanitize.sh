#!/bin/bash
# Host-code sanitizers (CPU only -- GPU ASan / XNACK runs are not available): libbzr's host C++ and the host halves
# of its HIP translation units built with clang's ASan + UBSan (make asan -> lib/asan/libbzr.so), then
#   1. tests/cpp/dropin_test.cpp's CPU part (preprocessing, BezierMesh, the single-ray methods vs the oracle),
#   2. the host-side Python tests (BVH proofs and replays, preprocessing parity, the C ABI's argument checks)
#      with the sanitizer runtime preloaded into python.
# Any report stops the run (halt_on_error) and is left in /tmp/{asan,ubsan}log.*.  Leaks are checked in (1) only
# (python itself leaks by design).  ~10 minutes on 8 cores.
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
make -C cuda-bezier-triangle-raytracer_amd -j8 asan > /tmp/host_sanitize_build.log 2>&1
make -C oracle > /dev/null
CXX=/opt/rocm/lib/llvm/bin/clang++
$CXX -g -O1 -std=c++17 -ffp-contract=off -pthread -fsanitize=address,undefined -fno-omit-frame-pointer \
  tests/cpp/dropin_test.cpp -Iinclude/bzr -Iinclude -Ioracle -Lcuda-bezier-triangle-raytracer_amd/lib/asan -lbzr \
  -Loracle -loracle -Wl,-rpath,"$R/cuda-bezier-triangle-raytracer_amd/lib/asan" -Wl,-rpath,"$R/oracle" \
  -o /tmp/dropin_asan 2> /dev/null
rm -f /tmp/asanlog.* /tmp/ubsanlog.*
ASAN_OPTIONS=detect_leaks=1:halt_on_error=1:log_path=/tmp/asanlog \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=/tmp/ubsanlog /tmp/dropin_asan
LD_PRELOAD="$($CXX -print-file-name=libclang_rt.asan-x86_64.so)" \
  ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:log_path=/tmp/asanlog \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=/tmp/ubsanlog \
  BZR_LIBRARY="$R/cuda-bezier-triangle-raytracer_amd/lib/asan/libbzr.so" BZR_NO_TORCH_PRELOAD=1 \
  python -m pytest tests/test_culling_conservative.py tests/test_host_parity.py tests/test_capi.py -x -q -m "not gpu" \
  -p no:cacheprovider
if ls /tmp/asanlog.* /tmp/ubsanlog.* > /dev/null 2>&1; then echo "sanitizer reports:"; ls /tmp/asanlog.* /tmp/ubsanlog.* 2>/dev/null; exit 1; fi
echo "host sanitizers: clean"
