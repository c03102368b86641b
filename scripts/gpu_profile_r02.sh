#!/bin/bash
# rocprofv3 kernel-trace stats of the bench command, then PMC counter passes (one group per
# run, never combined with tracing).  Output: gpurun_out/prof_<tag>/, gpurun_out/pmc_<tag>/summary.json
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
mkdir -p $R/gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --kernel-only > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
f=$(find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
head -14 "$f"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INST_CYCLES_VALU" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_$TAG/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --kernel-only > $R/gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; tail -5 $R/gpurun_out/pmc_$TAG/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_$TAG $R/gpurun_out/pmc_$TAG/summary.json > /dev/null && echo PMC_OK
# the call-level trace (chunked kernels + copies of the pipelined nw_align_ops call)
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof_call_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-quant --no-legs --no-check > $R/gpurun_out/prof_call_$TAG.log 2>&1 || { echo PROF_CALL_FAIL; tail -20 $R/gpurun_out/prof_call_$TAG.log; exit 1; }
echo CALL_TRACE_OK
