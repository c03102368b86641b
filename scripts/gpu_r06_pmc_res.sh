#!/bin/bash
# PMC counters of the kernel-resident pass (bench.py --kernel-only), one counter group per rocprofv3
# pass -> gpurun_out/<tag>/summary_resident.{json,txt}
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r06_pmcres}; O=$R/gpurun_out/$TAG; mkdir -p $O/res
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $O/res/res_p$i -o run -- python3 $R/bench.py --kernel-only --steps 3 --warmup 1 --no-cpu > $O/res_p$i.log 2>&1 || { echo "resident PMC pass $i ($grp) failed"; tail -5 $O/res_p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/res $O/summary_resident.json 4 > $O/summary_resident.txt
cut -c1-400 $O/summary_resident.txt
