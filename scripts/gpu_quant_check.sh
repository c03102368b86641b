#!/bin/bash
# Quantification kernel: GPU parity tests, then the bench (aligner + quant leg) with a rocprofv3 kernel summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_quant.py -q > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/${TAG}_bench.err || { echo BENCH_FAIL; tail -20 $R/gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json,sys; d=json.load(open('$R/gpurun_out/${TAG}_bench.json')); q=d['downstream_quantification']
print('align', round(d['value']/1e6,2), 'M/s; quant', round(q['value']/1e6,1), 'M/s kernel', round(q['kernel_ms_avg'],4), 'ms', round(q['roofline']['achieved'],1), 'GB/s')"
grep -E "quant|Name" $R/gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -d, -f1-4
