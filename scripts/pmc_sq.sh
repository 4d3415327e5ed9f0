#!/bin/bash
# SQ / SQC counters (issue, stall and scalar-cache breakdown) over a short bench run; PMC passes with --kernel-trace only.
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --cpu-baseline off ${PROF_ARGS:-}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
  --kernel-trace -d "$OUT/pmc_sq1" -o run -- python3 $B > "$OUT/pmc_sq1.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM SQ_INSTS_LDS SQ_LEVEL_WAVES \
  --kernel-trace -d "$OUT/pmc_sq2" -o run -- python3 $B > "$OUT/pmc_sq2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_TC_STALL SQC_DCACHE_BUSY_CYCLES SQC_TC_DATA_READ_REQ \
  --kernel-trace -d "$OUT/pmc_sq3" -o run -- python3 $B > "$OUT/pmc_sq3.log" 2>&1 || exit $?
