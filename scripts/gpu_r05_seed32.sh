#!/bin/bash
# The seeded list through the second level: window / C1-shape parity tests, the C1 call's path
# counts, A/B against the seeded list straight to the wide level (CRISPR_NW_SEED32=0), kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_seed32}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_windows.py \
  "tests/test_gpu_full_parity.py::test_c1_shape_every_read" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AB_COUNTS=1 timeout -k 10 200 python3 scripts/diag/ab_call.py "CRISPR_NW_SEED32=0" "" 8 c1 > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
cat $O/c1.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 $R/scripts/diag/ab_call.py "" "" 2 c1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo prof done
