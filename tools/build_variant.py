#!/usr/bin/env python3
"""Build an instrumented / diagnostic variant of libhbgpu (tool builds only,
never the product library): every csrc/*.hip compiled with extra -D flags
into tools/build_<name>/, linked to tools/libhbgpu_<name>.so.  Load it with
HBG_LIB_PATH.

    python tools/build_variant.py fpcount -DHBG_FP_COUNT
    python tools/build_variant.py debug -DHBG_DEBUG_CHECKS
    HBG_VARIANT_ONLY=rbc_kernels.hip python tools/build_variant.py ring2 -DHBG_FUSED_DATA_SRC=2

HBG_VARIANT_ONLY=<file.hip>: recompile only that source with the flags and
link it with the product objects of the others (hydrabadger_amd/build/).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(name: str, defines: list) -> str:
    sys.path.insert(0, ROOT)
    from hydrabadger_amd import build as hb
    obj_dir = os.path.join(ROOT, "tools", f"build_{name}")
    lib = os.path.join(ROOT, "tools", f"libhbgpu_{name}.so")
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(hb.CSRC, "*.hip")))

    only = os.environ.get("HBG_VARIANT_ONLY")

    def one(src):
        if only and os.path.basename(src) != only:
            return os.path.join(hb.OBJ, os.path.basename(src) + ".o")
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        r = subprocess.run([hb.HIPCC, *hb.CFLAGS, *defines, "-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr[-4000:])
        return obj
    with cf.ThreadPoolExecutor(max_workers=len(srcs)) as ex:
        objs = list(ex.map(one, srcs))
    subprocess.run([hb.HIPCC, f"--offload-arch={hb.ARCH}", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    return lib


if __name__ == "__main__":
    print(build(sys.argv[1], sys.argv[2:]))
