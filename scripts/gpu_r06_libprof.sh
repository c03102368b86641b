#!/bin/bash
# Per-library kernel stats of the resident pass: rocprofv3 --kernel-trace --stats over bench.py --kernel-only
# for each variant library.  Usage (through gpurun): bash scripts/gpu_r06_libprof.sh <tag> "<lib1> <lib2> ..."
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
for l in $2; do
  CRISPR_NW_LIB=$l timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/p_$l -o run --output-format csv -- python3 bench.py --kernel-only --steps 20 --warmup 5 > $OUT/k_$l.json 2> $OUT/k_$l.err || { tail -20 $OUT/k_$l.err; exit 1; }
  f=$(ls $OUT/p_$l/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find $OUT/p_$l -name '*kernel_stats.csv' | head -1)
  echo "== $l"; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('kernel_ms', round(d['kernel_ms'],4), {k: round(v,4) for k,v in (d.get('phases_ms') or {}).items()})" $OUT/k_$l.json
  cut -d, -f1-4 "$f" | head -10
done
