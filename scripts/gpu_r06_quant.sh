#!/bin/bash
# Round-6 quantification probe: its GPU tests (reference fixtures), then the bench's quantification
# leg alone (bench.py --quant-only) and its rocprofv3 kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r06_quant}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_quant.py tests/test_e2e_pin.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py --quant-only --steps 20 --warmup 5 --no-cpu > $OUT/quant.json 2> $OUT/quant.err || { tail -30 $OUT/quant.err; exit 1; }
tail -c 1500 $OUT/quant.json; echo
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/qprof -o q --output-format csv -- python3 $R/bench.py --quant-only --steps 10 --warmup 3 --no-cpu > $OUT/qprof.log 2>&1 || { tail -20 $OUT/qprof.log; exit 1; }
f=$(find $OUT/qprof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv; cut -d, -f1-4 $OUT/kernel_stats.csv | head -12
