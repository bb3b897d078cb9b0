"""Compare timing variants of the engine library (build.build_variant) on the
bench workload: each variant runs in fresh processes with TBGPU_LIB pointing at
its library.  Usage (GPU box, repo root):
    python3 profiles/variants.py NAME[=DEFINE+DEFINE..] ... [-- bench args]
'base' is the product library; any other NAME is tigerbeetle_amd/build/var_NAME/libtbgpu.so,
built here from its DEFINEs when missing (the variant builds stay off the pushed tree:
.gpurunignore)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
argv = sys.argv[1:]
bench_args = ["--steps", "5", "--warmup", "1", "--no-cpu"]
if "--" in argv:
    k = argv.index("--")
    argv, bench_args = argv[:k], argv[k + 1:]
reps = int(os.environ.get("REPS", "3"))
for spec in argv:
    name, _, defs = spec.partition("=")
    lib = os.path.join(ROOT, "tigerbeetle_amd", "build", "var_" + name, "libtbgpu.so")
    env = dict(os.environ)
    if name != "base":
        if not os.path.exists(lib):
            if not defs:
                print(name, "missing", lib, "(give NAME=DEFINE+DEFINE to build it)", flush=True)
                continue
            sys.path.insert(0, ROOT)
            from tigerbeetle_amd.build import build_variant
            build_variant(name, defs.split("+"))
        env["TBGPU_LIB"] = lib
    vals, commits, idx, app = [], [], [], []
    for _ in range(reps):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *bench_args], env=env,
                           capture_output=True, text=True, cwd=ROOT)
        try:
            line = json.loads(r.stdout.strip().splitlines()[-1])
        except Exception:
            print(name, "failed", r.stderr[-800:], flush=True)
            break
        ph = line["roofline"]["phase_ms_per_step"]
        vals.append(line["value"] / 1e9)
        commits.append(ph["classify"])
        idx.append(ph["index"])
        app.append(ph["apply"])
    if vals:
        print(f"{name:12s} value max={max(vals):.3f} G/s  commit min={min(commits):.4f} ms  "
              f"apply min={min(app):.4f} ms  index min={min(idx):.4f} ms  all={[round(v, 3) for v in vals]}", flush=True)
