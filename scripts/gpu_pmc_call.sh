#!/bin/bash
# PMC counters of the resident pass bench.py times for value (bench.py --kernel-only: warmup + steps
# passes, one launch of each kernel per pass), of the call_pcie calls' kernels (bench.py --skip-kernel-pass: warmup + steps pipelined
# nw_align_ops_packed calls, each kernel once per chunk) and of the quantification leg
# (bench.py --quant-only), one counter group per rocprofv3 pass (never with tracing domains).
# Summaries: gpurun_out/pmc_<tag>/summary_resident.json (bytes per pass), summary_call.json (bytes per
# call) and summary_quant.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CALLS=4   # --warmup 1 --steps 3
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $O/call_p$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --skip-kernel-pass --no-cpu --no-quant --no-legs --no-multi --no-check > $O/call_p$i.log 2>&1 || { echo "call PMC pass $i ($grp) failed"; tail -5 $O/call_p$i.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $O/res_p$i -o run -- python3 $R/bench.py --kernel-only --steps 3 --warmup 1 > $O/res_p$i.log 2>&1 || { echo "resident PMC pass $i ($grp) failed"; tail -5 $O/res_p$i.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $O/quant_p$i -o run -- python3 $R/bench.py --quant-only --steps 3 --warmup 1 --no-cpu > $O/quant_p$i.log 2>&1 || { echo "quant PMC pass $i ($grp) failed"; tail -5 $O/quant_p$i.log; exit 1; }
done
mkdir -p $O/call $O/quant $O/res
mv $O/call_p* $O/call/ && mv $O/quant_p* $O/quant/ && mv $O/res_p* $O/res/
python3 $R/scripts/pmc_summary.py $O/res $O/summary_resident.json 4 > $O/summary_resident.txt
python3 $R/scripts/pmc_summary.py $O/call $O/summary_call.json $CALLS > $O/summary_call.txt
python3 $R/scripts/pmc_summary.py $O/quant $O/summary_quant.json 4 > $O/summary_quant.txt
tail -20 $O/summary_resident.txt
