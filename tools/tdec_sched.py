#!/usr/bin/env python3
"""Batched vs per-share verify_decryption_share schedule by batch size (the
crossover behind api.hip kBatchMinShares).  Device-generated N=64 t=21 epochs
(1 % bad shares), hbg_tdec_verify_shares timed with HIP events per mode:

    python tools/tdec_sched.py --n-ct 256,1024,4096,8192,16384 --reps 2

One JSON line per size: ms per call for mode 3 (batched at every size) and
mode 0 (one pairing check per share), bits checked against construction.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-ct", default="256,1024,4096,8192")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=64)
    a = ap.parse_args()
    import numpy as np
    import torch
    from hydrabadger_amd import _lib, tdec_workload as tw
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx = _lib.Context(0)
    ctx.set_stream(st.cuda_stream)
    L = _lib.lib()
    N = a.nodes
    for n_ct in [int(x) for x in a.n_ct.split(",")]:
        ep = tw.make_epoch(ctx, dev, n_ct, N, 256, 0.01, 5)
        n = n_ct * N
        sct = torch.arange(n_ct, dtype=torch.int32, device=dev).repeat_interleave(N)
        spk = torch.arange(N, dtype=torch.int32, device=dev).repeat(n_ct)
        ok = torch.zeros(n, dtype=torch.uint8, device=dev)

        def call():
            _lib.check(L.hbg_tdec_verify_shares(ctx.h, n_ct, ep.U.data_ptr(), ep.V.data_ptr(), ep.V_off.data_ptr(),
                                                ep.W.data_ptr(), N, ep.pk48.data_ptr(), n, ep.share48.data_ptr(),
                                                sct.data_ptr(), spk.data_ptr(), ok.data_ptr(),
                                                _lib.HBG_DEVICE | _lib.HBG_ASYNC), "verify")
        res = {"n_ct": n_ct, "shares": n}
        for mode in (3, 0):
            _lib.check(L.hbg_test_set_tdec_batched(ctx.h, mode))
            call()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                call()
            e.record()
            e.synchronize()
            res[f"mode{mode}_ms"] = s.elapsed_time(e) / a.reps
            res[f"mode{mode}_bits_ok"] = bool(np.array_equal(ok.cpu().numpy().reshape(n_ct, N).astype(bool),
                                                            ~ep.bad))
        _lib.check(L.hbg_test_set_tdec_batched(ctx.h, 1))
        print(json.dumps(res), flush=True)
        del ep
    ctx.close()


if __name__ == "__main__":
    main()
