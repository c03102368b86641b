set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03m; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_TAIL=0" 10 c3 > $OUT/ab_c3_tail.log 2>&1 || { tail -20 $OUT/ab_c3_tail.log; exit 1; }
tail -2 $OUT/ab_c3_tail.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 10 c3 > $OUT/ab_c3_diag.log 2>&1 || { tail -20 $OUT/ab_c3_diag.log; exit 1; }
tail -2 $OUT/ab_c3_diag.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kprof -o run --output-format csv -- python3 $R/bench.py --kernel-only --steps 10 --warmup 3 > $OUT/kprof.log 2>&1 || { tail -20 $OUT/kprof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/cprof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-quant --no-legs --no-multi --no-check --skip-kernel-pass > $OUT/cprof.log 2>&1 || { tail -20 $OUT/cprof.log; exit 1; }
cd $R && bash scripts/gpu_pmc.sh r03 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
tail -25 $OUT/pmc.log
