#!/bin/bash
# GPU box: in-process A/B of variant builds (scripts/ab.py); AB_ARGS = variants + flags
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab.py $AB_ARGS > gpurun_out/ab.log 2>&1
