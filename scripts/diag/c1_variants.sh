#!/bin/bash
# C1-shape call under each library variant (default, and those named): rocprofv3 kernel stats of
# c1_ab.py, the classify / wide / exact lines, and the call's median time.
# Usage (through gpurun): bash scripts/diag/c1_variants.sh noseed nosub1 ...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  lib=libcrispr_nw.so; [ "$v" != default ] && lib=libcrispr_nw_$v.so
  CRISPR_NW_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c1var_$v -o c1 --output-format csv -- python3 $R/scripts/diag/c1_ab.py "" "" 1 > $R/gpurun_out/c1var_$v.log 2>&1 || { tail -5 $R/gpurun_out/c1var_$v.log; exit 1; }
  echo "== $v: $(grep -h '^A ' $R/gpurun_out/c1var_$v.log | cut -c1-160)"
  grep -h "classify\|fill<128\|walk<128\|align_kernel\|segsort" $R/gpurun_out/c1var_$v/c1_kernel_stats.csv | cut -d, -f1-4 | cut -c1-110
done
