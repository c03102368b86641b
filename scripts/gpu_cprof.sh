#!/bin/bash
# rocprofv3 kernel + copy stats of the headline call (bench.py call legs only) and the
# kernel-resident pass: bash scripts/gpu_cprof.sh <tag>; output under gpurun_out/<tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-cprof}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/cprof -o call --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-quant --no-legs --no-multi --no-check --skip-kernel-pass > $OUT/cprof.log 2>&1 || { tail -20 $OUT/cprof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kprof -o kern --output-format csv -- python3 $R/bench.py --kernel-only --steps 10 --warmup 3 > $OUT/kprof.log 2>&1 || { tail -20 $OUT/kprof.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
for pat in ("cprof/**/*kernel_stats.csv", "kprof/**/*kernel_stats.csv"):
    for p in glob.glob(sys.argv[1] + "/" + pat, recursive=True):
        print("==", p.split("/")[-1])
        for r in list(csv.DictReader(open(p)))[:16]:
            print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):6.2f}%')
PY
