#!/bin/bash
# one-wave exact kernel latency by phase (debug modes 0 / 1 / 2) on 8 reads
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in 0 1 2; do
  CRISPR_NW_DEBUG_MODE=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/exlat_$m -o run --output-format csv -- python3 $R/scripts/diag/exact_latency.py ${1:-8} > $R/gpurun_out/exlat_$m.log 2>&1 || { tail -20 $R/gpurun_out/exlat_$m.log; exit 1; }
  f=$(find $R/gpurun_out/exlat_$m -name "*kernel_stats.csv" | head -1)
  echo "mode $m"; grep -E "nw_align_kernel|nw_exact" "$f" | cut -c1-160
done
