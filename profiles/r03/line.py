"""Print the headline numbers of a bench.py JSON line: python3 profiles/r03/line.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError) as e:
        print(f, "unreadable:", e)
        continue
    r = d.get("roofline") or {}
    out = {"value_G": round(d["value"] / 1e9, 4), "frac": r.get("frac"), "kernel": r.get("kernel"),
           "dominant_ms": r.get("dominant_ms_per_step"), "device_ms": r.get("device_ms_per_step"),
           "non_ok": d.get("non_ok_results"), "passes": d.get("fixed_point_passes")}
    if d.get("cpu_baseline"):
        out["cpu"] = d["cpu_baseline"]["value"]
    if d.get("host_path"):
        out["single_us"] = d["host_path"]["single"]["latency_us"]
    if d.get("create_accounts"):
        out["accounts"] = {k: d["create_accounts"].get(k) for k in ("accounts_per_s", "device_ms")}
        out["accounts"]["frac"] = d["create_accounts"]["roofline"]["frac"]
    if d.get("routed"):
        out["routed"] = d["routed"]["phase_ms_one_unpipelined_step_max_over_ranks"]
    if d.get("verify"):
        out["verify"] = d["verify"]
    print(f, json.dumps(out))
