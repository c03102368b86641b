#!/bin/bash
# Round-6 quick perf probe: the kernel-resident pass (bench.py --kernel-only: value + per-phase
# HIP-event times) and its rocprofv3 kernel stats; optional extra bench args after the tag.
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-r06_perf}; shift; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 300 python bench.py --kernel-only --steps 20 --warmup 5 --no-cpu "$@" > $OUT/kernel_only.json 2> $OUT/kernel_only.err || { tail -30 $OUT/kernel_only.err; exit 1; }
python3 - "$OUT/kernel_only.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"])
kr = d.get("kernel_rate") or {}
print("kernel_rate", json.dumps(kr)[:1500])
PY
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kprof -o kern --output-format csv -- python3 $R/bench.py --kernel-only --steps 10 --warmup 3 --no-cpu "$@" > $OUT/kprof.log 2>&1 || { tail -20 $OUT/kprof.log; exit 1; }
f=$(find $OUT/kprof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv; cut -d, -f1-4 $OUT/kernel_stats.csv | head -20
