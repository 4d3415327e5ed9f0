#!/bin/bash
# round-3 profiles: rocprofv3 kernel trace + PMC passes (prof_run.sh) for cfg4 fused, cfg5 staged, cfg2 fused
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
for spec in "r03_cfg4_fused_v1|--config cfg4 --pipeline fused|cfg4/fused/parity/4096" \
            "r03_cfg5_staged_v1|--config cfg5 --pipeline staged|cfg5/staged/parity/8192" \
            "r03_cfg2_fused_v1|--config cfg2 --pipeline fused|cfg2/fused/parity/1024"; do
  IFS="|" read -r tag bench wl <<< "$spec"
  TAG=$tag BENCH="$bench" WORKLOAD=$wl bash scripts/prof_run.sh || exit $?
done
exit 0
