#!/usr/bin/env python3
"""Measured Fp-multiplication counts of the ThresholdDecrypt kernels (the
algorithmic unit of the TDec roofline: one Fp multiplication = 288
v_mad_u64_u32).

    python tools/fpcount.py build                 # CPU: instrumented library
    python tools/fpcount.py run --n-ct 2048       # GPU: counts -> profiles/fpcount.json

`build` compiles every csrc/*.hip with -DHBG_FP_COUNT (bls.h: each fp_mul /
fp_sqr call adds 1 per active lane to a device counter; tdec_kernels.hip:
every launcher closes the previous launch's count) into
tools/libhbgpu_fpcount.so — a tool build, never the product library.
`run` loads it (HBG_LIB_PATH), generates the bench's TDec epoch
(hydrabadger_amd/tdec_workload.py: N=64, t=21, 1 % bad shares, 256-B
contributions) at a smaller ciphertext count, runs hbg_tdec_threshold_decrypt
and hbg_tdec_verify_shares once each, and writes per-kernel and per-share
counts.  Counts per share are shape-stable (the group-testing rounds depend on
the bad-share rate, not on the batch size).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "libhbgpu_fpcount.so")


def build():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from build_variant import build as bv
    # no divergent branch next to the products (bls.h fp_count): each lane adds 1, and the compiler's
    # wave-aggregating atomic optimizer (which would put the branch back) is off
    print(bv("fpcount", ["-DHBG_FP_COUNT", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]))
    # the sources this instrumented library was built from: `run` stamps this
    # digest (not the tree's), so a stale library never reads as measured at HEAD
    sys.path.insert(0, ROOT)
    from hydrabadger_amd.build import source_digest
    with open(LIB + ".sha16", "w") as f:
        f.write(source_digest() + "\n")


def _report(lib) -> dict:
    buf = C.create_string_buffer(1 << 16)
    assert lib.hbg_fp_count_report(buf, len(buf)) == 0
    return json.loads(buf.value.decode())


def run(n_ct: int, out: str, bad_rate: float = 0.01):
    os.environ["HBG_LIB_PATH"] = LIB
    sys.path.insert(0, ROOT)
    import torch
    from hydrabadger_amd import _lib, tdec_workload as tw, threshold as th
    lib = _lib.lib()
    lib.hbg_fp_count_report.argtypes = [C.c_char_p, C.c_uint64]
    lib.hbg_fp_count_report.restype = C.c_int
    dev = torch.device("cuda:0")
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    # the batched schedule at every size (the bench's configs[3] size uses it;
    # below 393,216 shares the default would check every share alone)
    _lib.check(lib.hbg_test_set_tdec_batched(ctx.h, 3))
    ep = tw.make_epoch(ctx, dev, n_ct, 64, 256, bad_rate, seed=1)
    N, t, n = ep.n_nodes, ep.t, n_ct * ep.n_nodes
    ctx.sync()
    _report(lib)  # drop the generator's counts
    pt = torch.zeros(n_ct * ep.msg_len, dtype=torch.uint8, device=dev)
    st = torch.zeros(n_ct, dtype=torch.int32, device=dev)
    oc = torch.zeros((n_ct, N), dtype=torch.uint8, device=dev)
    th.threshold_decrypt_arrays(t, N, ep.U, ep.V, ep.V_off, ep.W, ep.pk48, ep.share48, None, pt, st, oc, ctx=ctx,
                                device=True)
    drv = _report(lib)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    sct = torch.arange(n_ct, dtype=torch.int32, device=dev).repeat_interleave(N)
    spk = torch.arange(N, dtype=torch.int32, device=dev).repeat(n_ct)
    _lib.check(lib.hbg_tdec_verify_shares(ctx.h, n_ct, ep.U.data_ptr(), ep.V.data_ptr(), ep.V_off.data_ptr(),
                                          ep.W.data_ptr(), N, ep.pk48.data_ptr(), n, ep.share48.data_ptr(),
                                          sct.data_ptr(), spk.data_ptr(), ok.data_ptr(), _lib.HBG_DEVICE), "verify")
    ver = _report(lib)
    good = bool((st == 0).all().item()) and bool(torch.equal(pt, ep.msgs))

    def table(rep):
        k = {name: {"fp_mul": v[0], "fp_sqr": v[1], "launches": v[2], "per_share": (v[0] + v[1]) / n}
             for name, v in rep.items() if v[0] + v[1] > 0}
        return k, sum(v["per_share"] for v in k.values())
    dk, dtot = table(drv)
    vk, vtot = table(ver)
    try:
        built_from = open(LIB + ".sha16").read().strip()
    except OSError:
        built_from = None  # unknown sources: never matches HEAD
    res = {"source": f"tools/fpcount.py run --n-ct {n_ct} (instrumented build, HBG_FP_COUNT)",
           "csrc_sha16": built_from,
           "shape": {"n_nodes": N, "t": t, "bad_rate": bad_rate, "n_ct": n_ct, "msg_len": ep.msg_len},
           "unit": "Fp multiplications + squarings (each 288 v_mad_u64_u32)",
           "per_share_total": dtot, "per_share_verify_total": vtot, "kernels": dk, "verify_kernels": vk,
           "outputs_ok": good}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["build", "run"])
    ap.add_argument("--n-ct", type=int, default=2048)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "fpcount.json"))
    ap.add_argument("--bad-rate", type=float, default=0.01,
                    help="fraction of replaced shares (0: the schedule's minimum, no group testing or fallback)")
    a = ap.parse_args()
    build() if a.what == "build" else run(a.n_ct, a.out, a.bad_rate)


if __name__ == "__main__":
    main()
