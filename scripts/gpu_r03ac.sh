set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03ac; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
for q in 4 8 4 8; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_TAIL=0" 12 > $OUT/ab_q$q.log 2>&1 || { tail -20 $OUT/ab_q$q.log; exit 1; }
echo "queues $q"; tail -2 $OUT/ab_q$q.log
done
