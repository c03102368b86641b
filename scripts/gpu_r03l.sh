set -o pipefail
OUT=gpurun_out/r03l; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open("gpurun_out/r03l/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"])
for k in ("c4_shard","pooled","dual_alignment","e2e","downstream_quantification"):
    v=d.get(k) or {}
    print(k, {x: v.get(x) for x in ("value","ms_per_step","align_s","total_s") if x in v})
print("roofline", {k: d["roofline"].get(k) for k in ("achieved","frac","call_frac","traffic")})
print("kernel_rate", d.get("kernel_rate",{}).get("ms"), d.get("sample_check"))
PY
