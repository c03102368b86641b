#!/bin/bash
# Quantification leg: gpu_r06_quant.sh (tests, timing, kernel stats) then its PMC passes
# (bench.py --quant-only, one counter group per rocprofv3 pass) -> gpurun_out/<tag>/summary_quant.*
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r06_quantpmc}; O=$R/gpurun_out/$TAG; mkdir -p $O
bash $R/scripts/gpu_r06_quant.sh $TAG || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $O/quant/quant_p$i -o run -- python3 $R/bench.py --quant-only --steps 3 --warmup 1 --no-cpu > $O/quant_p$i.log 2>&1 || { echo "quant PMC pass $i ($grp) failed"; tail -5 $O/quant_p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/quant $O/summary_quant.json 4 > $O/summary_quant.txt
cat $O/summary_quant.txt | cut -c1-250
