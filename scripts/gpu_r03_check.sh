#!/bin/bash
# Round 3 check on the GPU box: GPU tests, smoke, default bench line (each step time-limited).
set -o pipefail
OUT=gpurun_out/${1:-r03_check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "call_frac", d["roofline"]["call_frac"])
for k in ("c4_shard", "pooled", "e2e", "dual_alignment", "sample_check", "cpu_baseline"):
    v = d.get(k)
    if isinstance(v, dict):
        print(k, {kk: vv for kk, vv in v.items() if not isinstance(vv, (dict, list)) or kk in ("seconds",)})
PY
