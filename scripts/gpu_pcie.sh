#!/bin/bash
# PCIe placement probes: copy rates per host placement, then the headline call per placement.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_pcie}
mkdir -p $O
cd $R
numactl -H > $O/numa.txt 2>&1 || true
cat $O/numa.txt | head -5
timeout -k 10 300 python3 scripts/diag/pcie_probe.py > $O/pcie.log 2>&1 || { tail -20 $O/pcie.log; exit 1; }
cat $O/pcie.log
for m in free local remote local; do
  timeout -k 10 120 python3 scripts/diag/h2d_probe.py $m 20 >> $O/call.log 2>&1 || { tail -20 $O/call.log; exit 1; }
done
cat $O/call.log
