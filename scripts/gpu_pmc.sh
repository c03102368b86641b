#!/bin/bash
# PMC counters of one kernel-resident aligner pass over the C2 batch (bench.py --kernel-only:
# every kernel launched once over the 1M reads, so per-dispatch = per-pass), one counter
# group per rocprofv3 pass (never combined with tracing domains).  Output under
# gpurun_out/pmc_<tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
mkdir -p $R/gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc_list_$TAG.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INST_CYCLES_VALU" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_$TAG/p$i -o run -- python3 $R/bench.py --kernel-only --steps 1 --warmup 0 > $R/gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "PMC pass $i ($grp) failed"; tail -5 $R/gpurun_out/pmc_$TAG/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_$TAG $R/gpurun_out/pmc_$TAG/summary.json
