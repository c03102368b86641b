#!/bin/bash
# Round-6 A/Bs of two env settings on several workloads (scripts/diag/ab_call.py: alternating
# in-process calls, outputs compared): usage gpu_r06_ab2.sh <tag> "<A env>" "<B env>" [rounds] [modes...]
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; A=$2; B=$3; N=${4:-20}; shift 4; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for mode in "$@"; do
  m=$mode; [ "$m" = c2 ] && m=""
  timeout -k 10 300 python3 -u scripts/diag/ab_call.py "$A" "$B" $N $m > $O/ab_$mode.log 2>&1 || { echo "ab $mode failed"; tail -20 $O/ab_$mode.log; exit 1; }
  echo "== $mode"; tail -2 $O/ab_$mode.log
done
