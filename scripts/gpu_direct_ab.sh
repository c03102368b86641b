#!/bin/bash
# GPU tests (one process), then in-process A/Bs of a per-call env knob on the C2 and C5 calls.
# Usage: gpu_direct_ab.sh TAG "A-env" "B-env"
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-ab}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_$TAG.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/gt_$TAG.log; exit 1; }
tail -2 gpurun_out/gt_$TAG.log
timeout -k 10 150 python scripts/diag/ab_call.py "$2" "$3" 30 > gpurun_out/ab_$TAG.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_$TAG.log; exit 1; }
timeout -k 10 250 python scripts/diag/ab_call.py "$2" "$3" 8 pooled >> gpurun_out/ab_$TAG.log 2>&1 || { echo AB_POOLED_FAIL; tail -20 gpurun_out/ab_$TAG.log; exit 1; }
grep -E '^(A|B) ' gpurun_out/ab_$TAG.log
