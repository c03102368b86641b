#!/bin/bash
# build + run the microbenchmarks on the GPU box; results -> gpurun_out/ubench_*.txt
# The issue-rate kernels are also timed by PMC (SQ_INSTS_VALU over GRBM_GUI_ACTIVE / 8, the
# guide's in-kernel clock: MI355X_MICROARCH.md "DVFS give-back"), not only by HIP events.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out
cd $GRAFT_REPO_ROOT/scripts/ubench && mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 pcie_h2d.hip -o /tmp/pcie_h2d && timeout -k 10 120 /tmp/pcie_h2d | tee $OUT/ubench_pcie_h2d.txt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 issue_rate.hip -o /tmp/issue_rate && timeout -k 10 120 /tmp/issue_rate | tee $OUT/ubench_issue_rate.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES -d $OUT/ubench_issue_pmc -o pmc --output-format csv -- /tmp/issue_rate > $OUT/ubench_issue_pmc.log 2>&1
echo pmc rc=$?
