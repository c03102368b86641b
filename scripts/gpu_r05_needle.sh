#!/bin/bash
# align_reads on the GPU (golden DataFrames: forward + HDR passes through the dual call) and the
# end-to-end pin.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_needle}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_golden.py tests/test_e2e_pin.py tests/test_gpu_quant.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
