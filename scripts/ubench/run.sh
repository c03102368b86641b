#!/bin/bash
# build + run the microbenchmarks on the GPU box; results -> gpurun_out/ubench_*.txt
set -o pipefail
cd $GRAFT_REPO_ROOT/scripts/ubench && mkdir -p $GRAFT_REPO_ROOT/gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 fill_chain.hip -o /tmp/fill_chain 2>/dev/null && timeout -k 10 120 /tmp/fill_chain | tee $GRAFT_REPO_ROOT/gpurun_out/ubench_fill_chain.txt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 issue_rate.hip -o /tmp/issue_rate 2>/dev/null && timeout -k 10 120 /tmp/issue_rate | tee $GRAFT_REPO_ROOT/gpurun_out/ubench_issue_rate.txt
