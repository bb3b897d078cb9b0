"""Timing-only ablation of the fast-path kernel (cdna_hip_programming.md §7, step 2).

Builds one variant library per ablation mask (compile-time FP_ABLATE: the product
library has no ablation switch), runs the bench workload once per variant in a fresh
process (TBGPU_LIB) and prints the per-phase device time; results of ablated runs are
wrong by construction.  Build the variants on the CPU host first:
    python profiles/ablate.py --build
"""
import json
import os
import subprocess
import sys

MASKS = {"full": 0, "no-balances": 2, "no-rows": 4, "no-balances+rows": 6, "no-probes": 32,
         "no-probes+balances+rows": 38, "no-event-load": 16, "no-event+probes+balances+rows": 54}
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1:] == ["--build"]:
    sys.path.insert(0, ROOT)
    from tigerbeetle_amd.build import build_variant
    for name, m in MASKS.items():
        print(build_variant(f"ablate{m}", [f"FP_ABLATE={m}"]))
    sys.exit(0)
args = sys.argv[1:] or ["--steps", "3", "--warmup", "1", "--no-cpu", "--no-queries"]
for name, m in MASKS.items():
    lib = os.path.join(ROOT, "tigerbeetle_amd", "build", f"var_ablate{m}", "libtbgpu.so")
    env = dict(os.environ, TBGPU_LIB=lib)
    r = subprocess.run([sys.executable, "bench.py", *args], env=env, capture_output=True, text=True)
    try:
        line = json.loads(r.stdout.strip().splitlines()[-1])
        ph = line["roofline"]["phase_ms_per_step"]
        print(f"{name:22s} value={line['value']/1e9:6.3f} G/s  commit={ph['classify']:.4f} ms  "
              f"index={ph['index']:.4f} ms  step={line['ms_per_step']:.4f} ms", flush=True)
    except Exception:
        print(name, "failed", r.stderr[-500:], flush=True)
