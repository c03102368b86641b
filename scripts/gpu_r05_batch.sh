#!/bin/bash
# Several round-5 GPU steps in one box lease, stopping at the first failure: usage
# gpu_r05_batch.sh script1.sh [script2.sh ...] (each a scripts/ file taking its default output dir)
set -o pipefail
cd $GRAFT_REPO_ROOT
for s in "$@"; do
  echo "=== $s"
  bash scripts/$s || { echo "FAILED: $s"; exit 1; }
done
