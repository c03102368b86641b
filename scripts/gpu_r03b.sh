set -o pipefail
OUT=gpurun_out/r03_check2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo tests failed; tail -50 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/diag/pooled_probe.py pooled c4 pooled timing > $OUT/pooled_probe.log 2>&1 || { echo probe failed; tail -30 $OUT/pooled_probe.log; exit 1; }
cat $OUT/pooled_probe.log | tail -40
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-quant > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['kernel_rate']['kernel_ms'], d['kernel_rate']['phases_ms'], d['path_counts'], d['sample_check']['sample_mismatches'])
print('c4', d['c4_shard']['ms_per_pass'], 'pooled', d['pooled']['ms_per_step'], 'dual', d['dual_alignment']['ms_per_step'], 'e2e', d['e2e']['seconds'])
"
