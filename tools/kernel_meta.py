#!/usr/bin/env python3
"""Kernel resource metadata of libhbgpu's gfx950 code objects (occupancy
evidence for the bench's rooflines).

For every object in hydrabadger_amd/build/ the .hip_fatbin section (a clang
offload bundle) is unpacked, the gfx950 code object's AMDGPU metadata note is
read with llvm-readelf, and per kernel we record VGPR/AGPR/SGPR counts,
scratch (spill) bytes, LDS bytes and the waves per SIMD the register file
allows (gfx950: 512 unified registers per lane per SIMD, allocation granule
8, at most 8 waves; /opt/skills/guides/MI355X_MICROARCH.md "Register files").

    python tools/kernel_meta.py [--out profiles/kernel_meta.json]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import struct
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def bundle_entries(blob: bytes):
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    assert blob.startswith(magic), "not an offload bundle"
    (n,) = struct.unpack_from("<Q", blob, len(magic))
    pos = len(magic) + 8
    for _ in range(n):
        off, size, tlen = struct.unpack_from("<QQQ", blob, pos)
        pos += 24
        triple = blob[pos:pos + tlen].decode()
        pos += tlen
        yield triple, blob[off:off + size]


def waves_per_simd(vgpr: int, agpr: int) -> int:
    regs = vgpr + agpr
    alloc = max(8, (regs + 7) // 8 * 8)
    return min(8, 512 // alloc)


def kernels_of(code_object: bytes):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code_object)
        f.flush()
        txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True,
                             check=True).stdout
    out = {}
    for blk in re.split(r"\n\s+- \.", txt):
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name or ".vgpr_count" not in blk:
            continue
        def g(key, default=0):
            m = re.search(rf"\.{key}:\s+(\d+)", blk)
            return int(m.group(1)) if m else default
        k = {"vgpr": g("vgpr_count"), "agpr": g("agpr_count"), "sgpr": g("sgpr_count"),
             "scratch_bytes": g("private_segment_fixed_size"), "lds_bytes": g("group_segment_fixed_size"),
             "max_flat_workgroup_size": g("max_flat_workgroup_size")}
        k["waves_per_simd_by_regs"] = waves_per_simd(k["vgpr"], k["agpr"])
        out[name.group(1)] = k
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "kernel_meta.json"))
    a = ap.parse_args()
    result = {}
    for obj in sorted(glob.glob(os.path.join(ROOT, "hydrabadger_amd", "build", "*.o"))):
        with tempfile.TemporaryDirectory() as d:
            fat = os.path.join(d, "fat.bin")
            r = subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj,
                                os.path.join(d, "x.o")], capture_output=True)
            if r.returncode != 0 or not os.path.exists(fat):
                continue  # host-only object (api.hip)
            blob = open(fat, "rb").read()
        for triple, co in bundle_entries(blob):
            if "gfx950" in triple and co[:4] == b"\x7fELF":
                for name, k in kernels_of(co).items():
                    if not name.startswith("_ZN3hbg"):
                        continue  # library kernels (hipcub / rocprim sort and scan)
                    k["object"] = os.path.basename(obj)
                    result[name] = k
    json.dump({"source": "tools/kernel_meta.py (llvm-readelf --notes of the gfx950 code objects)",
               "kernels": result}, open(a.out, "w"), indent=1, sort_keys=True)
    print(a.out, len(result), "kernels")


if __name__ == "__main__":
    main()
