#!/bin/bash
# Per-kernel register/occupancy summary of trace.hip (our kernels only).
cd "$(dirname "$0")/../cuda-bezier-triangle-raytracer_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize -I../include \
  -fPIC -c csrc/device/trace.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep "^csrc/device/trace.hip" | sed -E 's/ \[-Rpass-analysis=kernel-resource-usage\]//; s/^csrc[^ ]* remark: +//' \
  | awk '/^Function Name:/{name=$3} /^VGPRs:/{v=$2} /^TotalSGPRs:/{s=$2} /^SGPRs Spill/{ss=$3} /^VGPRs Spill/{vs=$3} /^Occupancy/{o=$3}
         /^LDS Size/{printf "%-64s vgpr %4s sgpr %4s spill s%s/v%s occ %s\n", substr(name,1,64), v, s, ss, vs, o}'
