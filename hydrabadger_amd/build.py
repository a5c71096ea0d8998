"""Build libhbgpu.so (the C-ABI engine) in-tree with hipcc for gfx950.

    python -m hydrabadger_amd.build          # incremental
    python -m hydrabadger_amd.build --force  # rebuild everything

Objects go to hydrabadger_amd/build/, the library to hydrabadger_amd/libhbgpu.so
(both git-ignored; the .so travels to the GPU box with gpurun).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "libhbgpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HBG_ARCH", "gfx950")
CFLAGS = ["-O3", "-std=c++20", "-fPIC", f"--offload-arch={ARCH}", "-fconstexpr-steps=100000000",
          "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


def _local_includes(path: str, seen: set) -> set:
    """Every quoted #include reachable from `path` (a translation unit may
    include another .hip: tdec_kernels_lat.hip)."""
    for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', open(path).read(), flags=re.M):
        dep = os.path.normpath(os.path.join(os.path.dirname(path), m.group(1)))
        if os.path.exists(dep) and dep not in seen:
            seen.add(dep)
            _local_includes(dep, seen)
    return seen


def _deps_mtime(src: str) -> float:
    return max(os.path.getmtime(f) for f in _local_includes(src, {src}))


def _compile(src: str, force: bool) -> tuple:
    """(object path, whether it was compiled now)."""
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    deps = _deps_mtime(src)
    fresh = not force and os.path.exists(obj) and os.path.getmtime(obj) >= deps
    if not fresh:
        cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
        # stamp the object with its inputs' time: an edit made while hipcc ran
        # still marks it stale
        os.utime(obj, (deps, deps))
    return obj, not fresh


def source_digest() -> str:
    """16 hex digits of SHA-256 over every csrc/ file (name + bytes, sorted):
    the identity of the kernels a profile was measured on.  Profiles under
    profiles/ carry it as `csrc_sha16`; bench.py compares it with the tree it
    runs from and reports `measured_at_head`."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted(os.listdir(CSRC)):
        path = os.path.join(CSRC, f)
        if os.path.isfile(path):
            h.update(f.encode() + b"\0" + open(path, "rb").read())
    return h.hexdigest()[:16]


def build(force: bool = False, jobs: int | None = None) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        res = list(ex.map(lambda s: _compile(s, force), srcs))
    objs = [o for o, _ in res]
    # objects carry their inputs' time, which can predate the library linked
    # from their previous version: relink whenever one was compiled now
    if (force or any(new for _, new in res) or not os.path.exists(LIB)
            or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs)):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force))
    sys.exit(0)
