#!/bin/bash
# Round-6 GPU tests: the named test files first (-x), then the whole GPU suite; one process each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06_tests}
shift
mkdir -p $O
cd $R
if [ $# -gt 0 ]; then
  timeout -k 10 600 python3 -u -m pytest "$@" -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/first.log 2>&1 || { tail -60 $O/first.log; exit 1; }
  tail -3 $O/first.log
fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
