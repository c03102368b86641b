#!/bin/bash
# Round-6 A/B of call knobs: GPU parity tests under setting B first (a subset: the ops call, every-read
# parity), then in-process alternating A/B calls (scripts/diag/ab_call.py).
# Usage: gpu_r06_ab.sh <tag> "<A env>" "<B env>" [rounds] [mode]
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; A=$2; B=$3; N=${4:-30}; MODE=${5:-}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
( IFS=','; for kv in $B; do export "$kv"; done
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_full_parity.py tests/test_gpu_indel.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests_B.log 2>&1 ) || { tail -40 $O/tests_B.log; exit 1; }
tail -1 $O/tests_B.log
timeout -k 10 600 python3 -u scripts/diag/ab_call.py "$A" "$B" $N $MODE > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
tail -8 $O/ab.log
