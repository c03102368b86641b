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
# the last call: from the last H2D burst that precedes the final kernels; print the final 200 events
tail = rows[-200:]
t0 = tail[0][0]
for s, e, k, lab, q in tail:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {k} q{q} {lab}")

# summary of the last call: the events after the last idle gap > 100 us
def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + ((cur_e - cur_s) if cur_e is not None else 0)


start = 0
end_so_far = rows[0][1]
for i in range(1, len(rows)):
    if rows[i][0] - end_so_far > 100_000:
        start = i
    end_so_far = max(end_so_far, rows[i][1])
call = rows[start:]
c0, c1 = call[0][0], max(r[1] for r in call)
kern = [(s, e) for s, e, k, lab, q in call if k == "K"]
h2d = [(s, e) for s, e, k, lab, q in call if k == "C" and "HOST_TO_DEVICE" in lab]
d2h = [(s, e) for s, e, k, lab, q in call if k == "C" and "DEVICE_TO_HOST" in lab]
print(f"\nlast call: span {(c1 - c0) / 1e3:.1f} us, kernels busy {union(kern) / 1e3:.1f} us, "
      f"H2D busy {union(h2d) / 1e3:.1f} us, D2H busy {union(d2h) / 1e3:.1f} us, events {len(call)}")
gaps, busy_end = [], c0
for s, e in sorted(kern):
    if s - busy_end > 10_000:
        gaps.append(((busy_end - c0) / 1e3, (s - busy_end) / 1e3))
    busy_end = max(busy_end, e)
print("kernel idle gaps > 10 us (offset, length):", [(round(a, 1), round(b, 1)) for a, b in gaps])
