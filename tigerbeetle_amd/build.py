"""Build libtbgpu.so (HIP for gfx950) in-tree, and the test oracle.

    python -m tigerbeetle_amd.build
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "libtbgpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("TBGPU_ARCH", "gfx950")
CXXFLAGS = ["-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
            "-Wno-unused-result", "-munsafe-fp-atomics"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_stamp(sources, headers, defines) -> str:
    """sha256 of every source and header the library is built from, the compiler
    flags and the defines: the library is rebuilt whenever its stamp differs, whatever
    the files' modification times say (a copied tree keeps mtimes that need not order
    sources before the library)."""
    h = hashlib.sha256()
    for f in list(sources) + list(headers):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join([HIPCC, *CXXFLAGS, *defines]).encode())
    return h.hexdigest()


def build_lib(verbose: bool = False, force: bool = False, defines=(), build_dir: str = BUILD,
              lib: str = LIB) -> str:
    """Compile csrc/*.hip and link `lib`.  `defines` (e.g. ["FP_WAVES_PER_EU=8"]) and
    a separate `build_dir`/`lib` build timing variants for experiments; the product
    library is the default one, and it never takes TBGPU_TIMING_VARIANTS (which admits
    the results-changing ablations, csrc/fast.h)."""
    if os.path.abspath(lib) == LIB and any(d.split("=")[0] == "TBGPU_TIMING_VARIANTS" for d in defines):
        raise ValueError("the product library is never built with TBGPU_TIMING_VARIANTS")
    os.makedirs(build_dir, exist_ok=True)
    sources = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "tbgpu.h")]
    stamp = build_stamp(sources, headers, defines)
    stamp_file = lib + ".stamp"
    try:
        with open(stamp_file) as fh:
            force = force or fh.read().strip() != stamp
    except OSError:
        force = True
    objs = []
    jobs = []
    for src in sources:
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + headers):
            jobs.append([HIPCC, *CXXFLAGS, *[f"-D{d}" for d in defines], "-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for cmd, r in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
            if verbose or r.returncode != 0:
                sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for {cmd[-3]}")
    if force or jobs or _stale(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("link failed")
        with open(stamp_file, "w") as fh:
            fh.write(stamp + "\n")
    return lib


def build_variant(name: str, defines) -> str:
    """build/var_<name>/libtbgpu.so, loaded instead of the product library when
    TBGPU_LIB points at it (profiles/variants.py)."""
    d = os.path.join(BUILD, "var_" + name)
    return build_lib(defines=["TBGPU_TIMING_VARIANTS", *defines], build_dir=d, lib=os.path.join(d, "libtbgpu.so"),
                     force=True)


def build_oracle() -> str:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return os.path.join(ROOT, "oracle", "liboracle.so")


def build_all(verbose: bool = False) -> None:
    build_lib(verbose=verbose)
    build_oracle()


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv)
    print(LIB)
