#!/usr/bin/env python3
"""Diagnostic: one hbg_tdec_threshold_decrypt of the bench's generator at
--n-ct ciphertexts with every launch on the throughput build
(hbg_test_set_latency_lanes(0)) — the dispatch the instrumented tool build
(tools/fpcount.py) uses — and the batched schedule; prints whether every
plaintext matches."""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-ct", type=int, default=2048)
    ap.add_argument("--lat-lanes", type=int, default=0)
    a = ap.parse_args()
    import torch
    from hydrabadger_amd import _lib, tdec_workload as tw, threshold as th
    lib = _lib.lib()
    lib.hbg_test_set_latency_lanes.argtypes = [C.c_uint64]
    lib.hbg_test_set_latency_lanes.restype = C.c_uint64
    dev = torch.device("cuda:0")
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(lib.hbg_test_set_tdec_batched(ctx.h, 3))
    ep = tw.make_epoch(ctx, dev, a.n_ct, 64, 256, 0.01, seed=1)
    ctx.sync()
    lib.hbg_test_set_latency_lanes(a.lat_lanes)
    n_ct, N, t = a.n_ct, ep.n_nodes, ep.t
    pt = torch.zeros(n_ct * ep.msg_len, dtype=torch.uint8, device=dev)
    st = torch.zeros(n_ct, dtype=torch.int32, device=dev)
    oc = torch.zeros((n_ct, N), dtype=torch.uint8, device=dev)
    th.threshold_decrypt_arrays(t, N, ep.U, ep.V, ep.V_off, ep.W, ep.pk48, ep.share48, None, pt, st, oc, ctx=ctx,
                                device=True)
    ctx.sync()
    print(json.dumps({"n_ct": n_ct, "lat_lanes": a.lat_lanes, "status_ok": bool((st == 0).all().item()),
                      "plaintexts_match": bool(torch.equal(pt, ep.msgs))}))


if __name__ == "__main__":
    main()
