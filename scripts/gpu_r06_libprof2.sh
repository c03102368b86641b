#!/bin/bash
# Per-library kernel stats of the resident pass (bench.py --kernel-only) and of the headline call
# (bench.py call legs only), rocprofv3 --kernel-trace --stats.  Usage (through gpurun):
# bash scripts/gpu_r06_libprof2.sh <tag> "<lib1> <lib2> ..." [kernel-name filter regex]
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp; F=${3:-cert|classify}
cd $R
for l in $2; do
  CRISPR_NW_LIB=$l timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/k_$l -o run --output-format csv -- python3 bench.py --kernel-only --steps 20 --warmup 5 > $OUT/k_$l.json 2> $OUT/k_$l.err || { tail -20 $OUT/k_$l.err; exit 1; }
  CRISPR_NW_LIB=$l timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/c_$l -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-quant --no-legs --no-multi --no-check --skip-kernel-pass > $OUT/c_$l.json 2> $OUT/c_$l.err || { tail -20 $OUT/c_$l.err; exit 1; }
  echo "== $l"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('kernel_ms', round(d['kernel_ms'],4))" $OUT/k_$l.json
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('call_ms', round(d['ms_per_step'],4))" $OUT/c_$l.json
  for m in k c; do f=$(find $OUT/${m}_$l -name '*kernel_stats.csv' | head -1); echo "[$m]"; cut -d, -f1-4 "$f" | grep -E "$F" || true; done
done
