"""Summarize a profiles/collect.sh output directory: per-kernel average duration
(kernel trace) and per-dispatch average of every PMC counter collected."""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]
avg_ns = {}
for f in sorted(glob.glob(os.path.join(out, "kt", "**", "*kernel_stats.csv"), recursive=True)):
    print("== kernel stats", f)
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        avg_ns[r["Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]] = float(r["AverageNs"])
    for r in rows[:12]:
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
# LDS bank conflicts (extra cycles over all LDS cycles) and mean resident waves per
# busy CU cycle, per kernel that ran the LDS / occupancy pass.
for k in sorted({k for k, _ in agg}):
    bc, ia = agg.get((k, "SQ_LDS_BANK_CONFLICT")), agg.get((k, "SQ_LDS_IDX_ACTIVE"))
    wc = agg.get((k, "SQ_WAVE_CYCLES"))
    if bc and ia and sum(ia):
        print(f"{k:40s} lds_bank_conflict_frac={sum(bc)/sum(ia):.4f}")
    if wc and k in avg_ns and avg_ns[k] > 0:
        # SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md): resident waves per CU
        # = 4 x wave-cycles / (kernel duration x 2.4 GHz x 256 CUs), max 32 (8 per SIMD)
        occ = 4 * sum(wc) / len(wc) / (avg_ns[k] * 1e-9 * 2.4e9 * 256)
        print(f"{k:40s} mean_resident_waves_per_cu={occ:.1f} (of 32; {avg_ns[k] / 1e3:.1f} us/dispatch)")
# Per-event HBM bytes of the fast-path kernels: FETCH_SIZE / WRITE_SIZE are in KiB;
# on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads
# (MI355X_MICROARCH.md, HBM section), so both the raw and the x2 figure are shown.
ev = float(sys.argv[2]) if len(sys.argv) > 2 else 0
if ev:
    print(f"== bytes per event ({ev:.0f} events per launch)")
    for k in sorted({k for k, _ in agg}):
        f, w = agg.get((k, "FETCH_SIZE")), agg.get((k, "WRITE_SIZE"))
        if not f or not w or k.startswith("__amd"):
            continue
        fm, wm = sum(f) / len(f) * 1024, sum(w) / len(w) * 1024
        if fm + wm < ev:  # kernels that do not scale with the call
            continue
        print(f"{k:40s} fetch={fm/ev:7.1f} B (x2: {2*fm/ev:7.1f})  write={wm/ev:7.1f} B")
    # Per-launch HBM traffic of every kernel that scales with the call, for bench.py's
    # roofline.traffic: 2 x FETCH_SIZE (gfx950 half-count of wide reads) + WRITE_SIZE.
    # Random 8/16/32-B accesses are uncalibrated (MI355X_MICROARCH.md), and Infinity-Cache
    # hits are counted as fabric traffic, so this is an upper-bound estimate of HBM bytes.
    import json
    res = {}
    for k in sorted({k for k, _ in agg}):
        f, w = agg.get((k, "FETCH_SIZE")), agg.get((k, "WRITE_SIZE"))
        if not f or not w or k.startswith("__amd"):
            continue
        fm, wm = sum(f) / len(f) * 1024, sum(w) / len(w) * 1024
        res[k] = {"fetch_bytes_raw": fm, "write_bytes": wm, "traffic_bytes": 2 * fm + wm,
                  "events_per_launch": ev}
    # Whole-step traffic of the commit path (the general path's roofline unit): every
    # commit kernel's dispatches summed, over the profiled calls (warmup + steps), the
    # account setup (ac_*, k_*) and queries (q_*) excluded.
    tot = 0.0
    for k in sorted({k for k, _ in agg}):
        if k.startswith(("__amd", "ac_", "k_", "q_", "lg_")):
            continue
        f, w = agg.get((k, "FETCH_SIZE")), agg.get((k, "WRITE_SIZE"))
        if f and w:
            tot += 2 * sum(f) * 1024 + sum(w) * 1024 * len(f) / len(w)
    res["_meta"] = {"config": int(os.environ.get("TB_CONFIG", "2")), "accounts": int(os.environ.get("TB_ACCOUNTS", "1000000")),
                    "id_order": os.environ.get("TB_ID_ORDER", "sequential"),
                    "routed": bool(os.environ.get("TB_ROUTED")),
                    "steps": int(os.environ.get("TB_CALLS", "3")), "events_per_step": ev,
                    "commit_traffic_bytes": tot}
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)
