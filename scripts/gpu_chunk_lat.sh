#!/bin/bash
# Chain latency of single-chunk calls by size (chunk_latency.py), host-timed, then a rocprofv3
# kernel trace of the 16k-read call (timeline of its chain).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_lat}
mkdir -p $O
cd $R
timeout -k 10 200 python3 scripts/diag/chunk_latency.py 4096,16384,32768,65536,131072,262144 30 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
CRISPR_NW_HOST_TIMING=1 timeout -k 10 200 python3 scripts/diag/chunk_latency.py 16384,65536 3 > $O/lat_host.log 2>&1 || { tail -20 $O/lat_host.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace16k -o run --output-format csv -- python3 $R/scripts/diag/chunk_latency.py 16384 4 > $O/trace16k.log 2>&1 || { tail -20 $O/trace16k.log; exit 1; }
python3 $R/scripts/diag/call_timeline.py $O/trace16k > $O/timeline16k.txt
cat $O/lat.log
tail -32 $O/timeline16k.txt
