#!/bin/bash
# The dual call: its parity tests (C3 every read, small one-chunk batch), the C3 parity tests of the
# two-call form, then the C3 step A/B (dual call vs the two calls) and a per-chunk trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_dual}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_full_parity.py::test_dual_call_small_and_odd_reads" "tests/test_gpu_full_parity.py::test_c3_dual_call_every_read" \
  "tests/test_gpu_full_parity.py::test_c3_both_passes_every_read" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 10 dual > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
CRISPR_NW_HOST_TIMING=1 timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 1 dualonly > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -v "^nw host" $O/trace.log | tail -30
