"""Per-dispatch view of a rocprofv3 kernel trace (kernel_trace.csv): for the general
path's pass kernels, duration per pass and the idle gaps between dispatches, so that
launch/round-trip overheads show next to kernel time.  usage: passtrace.py DIR [first_kernel_regex]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def short(n):
    return n.replace("(anonymous namespace)::", "").split("(")[0][-28:]
# the last tr_classify .. the end: one chunk of the last call
idx = [k for k, r in enumerate(rows) if "tr_classify" in r["Kernel_Name"]]
if not idx:
    sys.exit("no tr_classify")
a = idx[-2] if len(idx) > 1 else idx[-1]
b = idx[-1]
busy = gap = 0
prev_end = None
agg = {}
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev_end) if prev_end else 0
    prev_end = e
    n = short(r["Kernel_Name"])
    busy += e - s
    gap += max(g, 0)
    agg.setdefault(n, [0, 0])
    agg[n][0] += 1
    agg[n][1] += e - s
    print(f"{n:30s} {(e - s) / 1e3:8.2f} us  gap {g / 1e3:8.2f}")
print(f"chunk: busy {busy / 1e3:.1f} us, gaps {gap / 1e3:.1f} us")
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {n:30s} x{c:3d} {t / 1e3:8.1f} us")
