#!/bin/bash
# Variant-library A/B on one MI355X: kernel-resident pass and headline call per library build
# (CRISPR_NW_LIB=<name> under crispresso_amd/lib), libraries interleaved over rounds.
# Usage (through gpurun): bash scripts/gpu_libab.sh <tag> "<lib1> <lib2> ..." [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
for r in $(seq ${3:-2}); do
  for l in $2; do
    CRISPR_NW_LIB=$l timeout -k 10 200 python bench.py --kernel-only --steps 20 --warmup 5 > $OUT/k_${l}_$r.json 2> $OUT/k_${l}_$r.err || { tail -20 $OUT/k_${l}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'kernel_ms', round(d['kernel_ms'],4), {k: round(v,4) for k,v in (d.get('phases_ms') or {}).items()})" $OUT/k_${l}_$r.json $l
    CRISPR_NW_LIB=$l timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu --no-quant --no-legs --no-multi --no-check --skip-kernel-pass > $OUT/c_${l}_$r.json 2> $OUT/c_${l}_$r.err || { tail -20 $OUT/c_${l}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'call_ms', round(d['ms_per_step'],4))" $OUT/c_${l}_$r.json $l
  done
done
