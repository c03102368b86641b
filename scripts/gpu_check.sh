#!/bin/bash
# Full check of the tree on one MI355X: GPU tests, smoke, the bench line, rocprofv3 kernel
# and call stats; with "pmc" as the second argument also the PMC passes (gpu_pmc.sh).
# Usage (through gpurun): bash scripts/gpu_check.sh <tag> [pmc]; output under gpurun_out/<tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-check}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/gpu_tests.log | head -30; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "resident_check", (d.get("resident_check") or {}).get("same_as_call"))
print("call_pcie", {x: (d.get("call_pcie") or {}).get(x) for x in ("value", "ms_per_step")})
for k in ("c4_shard", "pooled", "dual_alignment", "c1_shape", "e2e", "downstream_quantification", "upstream_merge"):
    v = d.get(k) or {}
    print(k, {x: v.get(x) for x in ("value", "ms_per_step", "error") if x in v},
          (v.get("sample_check") or {}).get("sample_mismatches") if isinstance(v.get("sample_check"), dict) else "")
print("roofline", {k: d["roofline"].get(k) for k in ("achieved", "frac", "call_frac", "traffic")})
print("kernel_rate", d.get("kernel_rate", {}).get("kernel_ms"), d.get("sample_check", {}).get("sample_mismatches"))
PY
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kprof -o kern --output-format csv -- python3 $R/bench.py --kernel-only --steps 10 --warmup 3 > $OUT/kprof.log 2>&1 || { tail -20 $OUT/kprof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/cprof -o call --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-quant --no-legs --no-multi --no-check --skip-kernel-pass > $OUT/cprof.log 2>&1 || { tail -20 $OUT/cprof.log; exit 1; }
echo prof done
if [ "$2" = "pmc" ]; then
  cd $R && bash scripts/gpu_pmc.sh $TAG > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
  echo pmc done
fi
