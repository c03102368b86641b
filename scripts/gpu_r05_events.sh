#!/bin/bash
# (libcrispr_nw_r5base.so: the parent commit's build, copied aside before rebuilding)
# A/B of the timing events: the resident pass with / without its phase events (bench value, wall clock),
# and the C2 / C1 calls with the previous library (every chunk's ev_cs, ev_fill, ev_walk, timing uploads'
# events) against this one; then the GPU tests of the phase / ops-times paths.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_events}
mkdir -p $O
cd $R
for r in 1 2 3; do
  for f in "" "--phase-events"; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-quant --no-legs --no-multi --no-check $f > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('phase_events' if sys.argv[2] else 'no_events', 'value_ms', round(d['ms_per_step'],4), 'call_ms', round(d['call_pcie']['ms_per_step'],4), 'kernel_ms', round(d['kernel_rate']['kernel_ms'],4), d['resident_check']['same_as_call'])" $O/b.json "$f"
  done
done
for r in 1 2; do
  for l in libcrispr_nw_r5base.so libcrispr_nw.so; do
    CRISPR_NW_LIB=$l timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 15 > $O/c_$l.log 2>&1 || { tail -20 $O/c_$l.log; exit 1; }
    echo "$l C2 $(grep '^A ' $O/c_$l.log)"
    CRISPR_NW_LIB=$l timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 10 c1 > $O/c1_$l.log 2>&1 || { tail -20 $O/c1_$l.log; exit 1; }
    echo "$l C1 $(grep '^A ' $O/c1_$l.log)"
  done
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
