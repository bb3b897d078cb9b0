"""A config-3 chunk's timeline from a rocprofv3 kernel trace (profiles/run.sh pmc:3's
kt/kt_kernel_trace.csv): per chunk, the setup kernels, then each pass's balance scan
and evaluation (duration and the gap before it), then the epilogue.
    python3 profiles/chunk_timeline.py TRACE.csv [chunk index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def name(r):
    return r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]


# chunks start at tr_prep
starts = [k for k, r in enumerate(rows) if name(r) == "tr_prep"]
want = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) - 1
k0 = starts[want]
k1 = starts[want + 1] if want + 1 < len(starts) else len(rows)
t0 = int(rows[k0]["Start_Timestamp"])
prev = t0
tot = {}
p = 0
for r in rows[k0:k1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = name(r)
    tag = ""
    if n == "bs_fused_narrow":
        tag = f"pass {p}"
    if n == "tr_eval_lists":
        p += 1
    print(f"{(s - t0) / 1e3:8.1f} {n[:28]:28s} gap={(s - prev) / 1e3:6.1f} dur={(e - s) / 1e3:6.1f} {tag}")
    tot[n] = tot.get(n, 0) + (e - s)
    prev = e
print(f"chunk {want}: {(prev - t0) / 1e3:.1f} us, {p} passes")
for n, v in sorted(tot.items(), key=lambda x: -x[1])[:12]:
    print(f"  {n:28s} {v / 1e3:8.1f} us")
