"""Summarize a profiles/collect.sh output directory: per-kernel average duration
(kernel trace) and per-dispatch average of every PMC counter collected."""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "kt", "**", "*kernel_stats.csv"), recursive=True)):
    print("== kernel stats", f)
    for r in list(csv.DictReader(open(f)))[:12]:
        print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
agg = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]
        agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
print("== counters (mean per dispatch)")
for (k, c), v in sorted(agg.items()):
    if sum(v) == 0:
        continue
    print(f"{k:40s} {c:24s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
