#!/usr/bin/env python3
"""Kernel micro-benchmarks through the C ABI (device-resident batches).

    python tools/kbench.py --what merkle,encode,rs,decode --instances 2048,4096 --reps 5

Prints one JSON line per (what, instances) with the average ms per launch
(HIP events on the engine's stream).  Used for occupancy sweeps and as the
target of rocprofv3 --pmc passes (tools/pmc.sh).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="merkle,encode,rs,decode")
    ap.add_argument("--instances", default="2048")
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--payload", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dec-fused", default="-1",
                    help="decode schedules to time (hbg_test_set_rbc_decode_fused): 0 three launches, 1 fused")
    ap.add_argument("--splits", default="0,1",
                    help="decode schedules to time (hbg_test_set_rs_split): 0 one-pass, 1 data rows + constant "
                         "parity encoder, -1 the library default")
    ap.add_argument("--pairs", default="-1",
                    help="merkle_build leaf schedules to time (hbg_test_set_merkle_pairs): 0 one lane a leaf, "
                         "1 a lane pair a leaf, -1 the library default (pairs for a partial last generation)")
    a = ap.parse_args()
    from hydrabadger_amd import _lib, workload
    from hydrabadger_amd import broadcast as bc

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx = _lib.Context(0)
    ctx.set_stream(st.cuda_stream)
    N, P = a.nodes, a.payload
    L = _lib.shard_len(N, P)
    S = (L + 15) // 16 * 16
    nodes = _lib.merkle_nodes(N)
    D, Q = bc.shard_counts(N)
    whats = a.what.split(",")
    for B in [int(x) for x in a.instances.split(",")]:
        pay = torch.empty((B, (P + 15) // 16 * 16), dtype=torch.uint8, device=dev)
        bc.synth_bytes(1, 0, P, pay, ctx=ctx, device=True)
        plen = torch.full((B,), P, dtype=torch.int64, device=dev)
        shards = torch.empty((B, N, S), dtype=torch.uint8, device=dev)
        levels = torch.empty((B, nodes, 32), dtype=torch.uint8, device=dev)
        bc.rbc_encode_merkle_batch(N, pay, plen, L, shards, levels, ctx=ctx, device=True)

        def t(fn):
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                fn()
            e.record()
            e.synchronize()
            return s.elapsed_time(e) / a.reps

        res = {"instances": B, "N": N, "P": P, "L": L}
        if "merkle" in whats:
            for pm in [int(x) for x in a.pairs.split(",")]:
                _lib.check(_lib.lib().hbg_test_set_merkle_pairs(ctx.h, pm))
                key = "merkle_ms" if pm == -1 else f"merkle_pairs{pm}_ms"
                res[key] = t(lambda: bc.merkle_build_batch(N, L, shards, levels, ctx=ctx, device=True,
                                                           asynchronous=True))
            _lib.check(_lib.lib().hbg_test_set_merkle_pairs(ctx.h, -1))
        if "encode" in whats:  # the two-launch schedule (rs_encode_const -> merkle_build)
            _lib.check(_lib.lib().hbg_test_set_rbc_fused(ctx.h, 0))
            res["encode_merkle_ms"] = t(lambda: bc.rbc_encode_merkle_batch(N, pay, plen, L, shards, levels, ctx=ctx,
                                                                          device=True, asynchronous=True))
            _lib.check(_lib.lib().hbg_test_set_rbc_fused(ctx.h, -1))
        if "fused" in whats:  # the single-launch schedule (hbg_test_set_rbc_fused)
            _lib.check(_lib.lib().hbg_test_set_rbc_fused(ctx.h, 1))
            res["encode_merkle_fused_ms"] = t(lambda: bc.rbc_encode_merkle_batch(N, pay, plen, L, shards, levels,
                                                                                ctx=ctx, device=True,
                                                                                asynchronous=True))
            _lib.check(_lib.lib().hbg_test_set_rbc_fused(ctx.h, -1))
        if "rs" in whats:
            def rs():
                _lib.check(_lib.lib().hbg_rs_encode(ctx.h, D, Q, L, shards.data_ptr(), S, B,
                                                    _lib.HBG_DEVICE | _lib.HBG_ASYNC))
            res["rs_encode_ms"] = t(rs)
        if "decode" in whats:
            present = torch.tensor([workload.erasure_mask(k, N, Q) for k in range(B)], dtype=torch.uint8,
                                   device=dev)
            roots = levels[:, nodes - 1, :].contiguous()
            OS = (D * L + 15) // 16 * 16
            out = torch.empty((B, OS), dtype=torch.uint8, device=dev)
            dpl = torch.empty(B, dtype=torch.int64, device=dev)
            dst = torch.empty(B, dtype=torch.uint8, device=dev)
            for fz in [int(x) for x in a.dec_fused.split(",")]:  # hbg_test_set_rbc_decode_fused
                _lib.check(_lib.lib().hbg_test_set_rbc_decode_fused(ctx.h, fz))
                for split in [int(x) for x in a.splits.split(",")]:  # hbg_test_set_rs_split
                    if fz != 0 and split != -1:
                        continue  # the fused decoder has one schedule
                    _lib.check(_lib.lib().hbg_test_set_rs_split(ctx.h, split))
                    res[f"decode_fused{fz}_split{split}_ms"] = t(lambda: bc.rbc_decode_batch(
                        N, L, shards, present, roots, out, dpl, dst, ctx=ctx, device=True, asynchronous=True))
                    res[f"decode_fused{fz}_split{split}_ok"] = bool((dst == 1).all().item()) and bool(
                        torch.equal(out[:, :P], pay[:, :P]))
            _lib.check(_lib.lib().hbg_test_set_rs_split(ctx.h, -1))
            _lib.check(_lib.lib().hbg_test_set_rbc_decode_fused(ctx.h, -1))
        print(json.dumps(res), flush=True)
        del pay, shards, levels
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
