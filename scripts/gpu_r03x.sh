set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03x; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_RAMP_TAIL=2:4:16" 20 > $OUT/ab1.log 2>&1 || { tail -20 $OUT/ab1.log; exit 1; }
tail -2 $OUT/ab1.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_RAMP_HEAD=8:4:2,CRISPR_NW_RAMP_TAIL=2:4" 20 > $OUT/ab2.log 2>&1 || { tail -20 $OUT/ab2.log; exit 1; }
tail -2 $OUT/ab2.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_RAMP_HEAD=8:4:2,CRISPR_NW_RAMP_TAIL=2:4:8" 20 > $OUT/ab3.log 2>&1 || { tail -20 $OUT/ab3.log; exit 1; }
tail -2 $OUT/ab3.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_CHUNK=196608" 20 > $OUT/ab4.log 2>&1 || { tail -20 $OUT/ab4.log; exit 1; }
tail -2 $OUT/ab4.log
