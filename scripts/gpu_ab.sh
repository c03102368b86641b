#!/bin/bash
# A/B of library knobs on one MI355X after a test subset: bash scripts/gpu_ab.sh <tag> <tests> "<A>" "<B>" [rounds] [workloads]
# tests: pytest paths ("-" = none); A / B: env settings ("VAR=v,VAR2=w"); workloads: space-separated ab_call.py modes ("c2 pooled c3 c4")
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
if [ "$2" != "-" ]; then
  timeout -k 10 400 python -u -m pytest $2 -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for w in ${6:-c2}; do
  m=$w; [ "$w" = "c2" ] && m=""
  timeout -k 10 300 python scripts/diag/ab_call.py "$3" "$4" ${5:-24} $m > $OUT/ab_$w.log 2>&1 || { tail -20 $OUT/ab_$w.log; exit 1; }
  echo "== $w"; tail -3 $OUT/ab_$w.log
done
