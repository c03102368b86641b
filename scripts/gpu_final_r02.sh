#!/bin/bash
# Final check of the round: GPU tests + smoke + bench line, ramp-shape A/Bs, then the rocprof profile.
# Usage: gpu_final_r02.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r02v5}
cd $R && mkdir -p gpurun_out
[ -z "$SKIP_CHECK" ] && { bash scripts/gpu_check_r02.sh $TAG || exit 1; }
for t in "CRISPR_NW_RAMP_TAIL=2:8" "CRISPR_NW_RAMP_TAIL=4:8" "CRISPR_NW_RAMP_HEAD=8:4:2"; do
  timeout -k 10 120 python scripts/diag/ab_call.py "" "$t" 30 > gpurun_out/ab_ramp.log 2>&1 || { echo AB_FAIL; exit 1; }
  grep -E "^(A|B) " gpurun_out/ab_ramp.log
done
bash scripts/gpu_profile_r02.sh $TAG || exit 1
