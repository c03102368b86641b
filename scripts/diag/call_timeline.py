"""Timeline of one pipelined nw_align_ops_packed call from a rocprofv3 kernel + memory-copy trace:
per chunk, the kernels and copies with start offsets and durations (microseconds).
Usage: call_timeline.py <trace dir>"""
import csv
import glob
import os
import sys

d = sys.argv[1]
rows = []
for name, kind in (("kernel_trace", "K"), ("memory_copy_trace", "C")):
    for path in glob.glob(os.path.join(d, "**", f"*{name}.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                label = r.get("Kernel_Name") or (r.get("Direction") or r.get("Operation") or "copy")
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, label[:60],
                             r.get("Stream_Id", r.get("Queue_Id", ""))))
rows.sort()
# the last call: from the last H2D burst that precedes the final kernels; print the final 150 events
tail = rows[-160:]
t0 = tail[0][0]
for s, e, k, lab, q in tail:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {k} q{q} {lab}")
