#!/usr/bin/env python3
"""Benchmark: hbbft RBC encode+Merkle (send_shards) at N=64 f=21, 1 MiB proposals.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--instances B]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

A step = one `hbg_rbc_encode_merkle` pass (BE length prefix + pad + chunk +
RS(22,42) encode + SHA3 Merkle tree) over B resident 1 MiB payloads per GPU
(BASELINE.json configs[2]).  Instances are sharded across ranks with no
data-path collective (weak scaling); only the timing max uses a collective.
`value` = payload bytes of all ranks / max-over-ranks wall time.

Also reported: per-kernel averages (HIP events on the engine's stream),
the roofline of the dominant kernel (the fused rbc_encode_merkle<22,42>, the
whole step: integer-VALU bound) with the two-launch schedule
beside it, the decode path (reconstruct 2f erasures + Merkle + glue), and the
CPU baseline (oracle C port, all host threads, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

N_NODES, PAYLOAD = 64, 1 << 20
BASE = json.load(open(os.path.join(ROOT, "BASELINE.json")))

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md: 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz; HBM 8 TB/s)
VALU_PEAK = 256 * 4 * 32 * 2.4e9   # int32 lane-ops/s
HBM_PEAK = 8.0e12                  # B/s
# Algorithmic VALU lane-ops: one Keccak-f[1600] on gfx950
# with 3-input bitop3 + alignbit = 24 rounds x 180; absorbing one 136-B block = 34 xors.
KECCAK_F_OPS = 24 * 180
ABSORB_OPS = 34


def merkle_counts(N: int, L: int):
    leaf_perms = N * (L // 136 + 1)
    pair = 0
    n = N
    while n > 1:
        pair += n // 2
        n = (n + 1) // 2
    return leaf_perms, pair


def encoder_alg_ops(D: int, Q: int, L: int) -> int:
    """Algorithmic lane-ops of Coding::encode for one instance: one v_bitop3
    split-nibble MAC per (parity row, data row, 4-byte word) — the GF(2^8)
    products of Q x D x L bytes, four per 32-bit lane-op."""
    return Q * D * ((L + 3) // 4)


def merkle_alg(N: int, L: int):
    leaf_perms, pair = merkle_counts(N, L)
    ops = leaf_perms * (KECCAK_F_OPS + ABSORB_OPS) + pair * KECCAK_F_OPS
    nodes = 2 * N - 1
    bytes_ = N * L + nodes * 32  # read every shard once, write the flat tree
    return ops, bytes_


LEGS = ("rbc", "decode", "cfg1", "n128", "bwire", "epoch", "tdec", "wire", "f1", "coin")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--instances", type=int, default=8192, help="1 MiB proposals per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=1024, help="instances in the CPU-baseline sample")
    ap.add_argument("--tdec-cts", type=int, default=100000,
                    help="ciphertexts per TDec step (BASELINE.json configs[3]: 100k x 64 shares, N=64 t=21); "
                         "0 disables the TDec leg")
    ap.add_argument("--epoch-nodes", type=int, default=128,
                    help="configs[4]: one N-node HoneyBadger epoch spanning all ranks (RCCL all-gather); 0 disables")
    ap.add_argument("--epoch-contrib", type=int, default=1 << 20,
                    help="contribution bytes per node in the configs[4] epoch (threshold-encrypted, then broadcast; "
                         "SURVEY.md §8(d) cfg 5: 1 MiB proposals)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend for N>1 (nccl = RCCL over xGMI; gloo: CPU rehearsal)")
    ap.add_argument("--wire-msgs", type=int, default=65536,
                    help="SURVEY.md §8(f2): wire messages signed + verified (0 disables)")
    ap.add_argument("--f1-cts", type=int, default=16384,
                    help="SURVEY.md §8(f1): ciphertexts encrypted + x64 decryption shares (0 disables)")
    ap.add_argument("--coins", type=int, default=16384,
                    help="SURVEY.md §8(f3): common coins (x64 signature shares) signed, verified, combined (0 disables)")
    ap.add_argument("--wire-instances", type=int, default=1024,
                    help="SURVEY.md §8(f4): instances whose N Value messages are written/parsed/validated (0 disables)")
    ap.add_argument("--cfg1-instances", type=int, default=10000,
                    help="configs[1] leg: N=16 f=5 64 KiB instances (encode+Merkle+decode); 0 disables")
    ap.add_argument("--n128-instances", type=int, default=2048,
                    help="N=128 (RS 44+84) 1 MiB encode+Merkle+decode instances; 0 disables")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--legs", default="all",
                    help="comma list of legs besides the timed step: " + ",".join(LEGS) + " (default all)")
    return ap.parse_args()


def head_digest() -> str:
    """The kernels this tree builds (hydrabadger_amd.build.source_digest)."""
    from hydrabadger_amd.build import source_digest
    return source_digest()


def measured_at_head(d: dict) -> bool | None:
    """Whether a committed profile was measured on the kernels of this tree
    (its csrc_sha16 stamp, tools/pack_profiles.py / tools/fpcount.py); None
    for a profile older than the stamp."""
    sha = d.get("csrc_sha16") or (d.get("_meta") or {}).get("csrc_sha16")
    return None if sha is None else sha == head_digest()


def newest(*rel: str) -> str:
    """The first of the candidate profile paths that exists (newest first)."""
    for r in rel:
        p = os.path.join(ROOT, *r.split("/"))
        if os.path.exists(p):
            return p
    return os.path.join(ROOT, *rel[-1].split("/"))


def pmc_traffic(instances: int) -> dict:
    """HBM bytes per launch measured by rocprofv3 PMC passes (FETCH_SIZE x2 +
    WRITE_SIZE, separate runs: tools/pmc.sh) at this launch shape, from
    profiles/pmc_traffic.json; empty when the shape differs."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return {}
    out = {"source": d.get("source", "") + f" ({os.path.relpath(path, ROOT)})"}
    for k in ("merkle_build", "rs_encode_const_22_42", "rbc_encode_merkle_22_42"):
        if d.get(k, {}).get("instances") == instances:
            out[k] = d[k]["hbm_bytes_per_launch"]
            # a kernel measured in a later pass names its own summary
            out[k + "_source"] = d[k].get("summary", d.get("summary", ""))
            out[k + "_measured_at_head"] = measured_at_head(d[k])
            if d[k].get("valu_insts_per_wave"):
                out[k + "_valu_insts_per_wave"] = d[k]["valu_insts_per_wave"]
    return out


# Kernels of one hbg_rbc_decode call at N = 64 (PMC passes: tools/gpu_r04d.sh /
# gpu_r04g.sh on the default fused schedule, profiles/r04/pmc_decode_fused_8192.json;
# FETCH_SIZE x2 + WRITE_SIZE per kernel; the three-launch schedule's passes are
# profiles/r04/pmc_decode_8192.json).
DECODE_KERNELS = ("rs_plan", "rs_code_movrel", "rs_encode_missing", "merkle_build", "rbc_glue_status",
                  "rbc_glue_copy", "rbc_decode_merkle")


def decode_pmc_traffic(instances: int) -> dict:
    path = newest("profiles/r06/pmc_decode_fused_8192.json", "profiles/r04/pmc_decode_fused_8192.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return {}
    if instances != 8192:
        return {}
    by = {}
    for name, v in d.items():
        short = name.split("<")[0]
        if short in DECODE_KERNELS and "hbm_read_bytes_corrected" in v:
            by[short] = v["hbm_read_bytes_corrected"] + v.get("hbm_write_bytes", 0.0)
    if not by:
        return {}
    vw = {name.split("<")[0]: v.get("valu_insts_per_wave") for name, v in d.items()
          if isinstance(v, dict) and name.split("<")[0] == "rbc_decode_merkle"}
    return {"bytes_per_call": sum(by.values()), "by_kernel": by, "source": os.path.relpath(path, ROOT),
            "valu_insts_per_wave": vw.get("rbc_decode_merkle"), "measured_at_head": measured_at_head(d)}


def timed(fn, reps: int):
    """Average ms per call of fn over reps (events on the current stream)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def cpu_baseline(n_sample: int):
    from oracle import corc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    threads = max(1, min(threads, os.cpu_count() or 1, 64))
    L = corc.shard_len(N_NODES, PAYLOAD)
    pay = np.empty((n_sample, PAYLOAD), np.uint8)
    for k in range(n_sample):
        pay[k] = corc.synth_bytes(1, k, PAYLOAD)
    corc.rbc_encode_merkle_batch(N_NODES, pay[:threads], L, threads)  # warm
    t0 = time.perf_counter()
    corc.rbc_encode_merkle_batch(N_NODES, pay, L, threads)
    dt = time.perf_counter() - t0
    return {"value": n_sample * PAYLOAD / dt / 1e9, "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{n_sample} x 1 MiB send_shards (RS 22+42 AVX2 split-nibble + SHA3 Merkle), "
                      f"oracle/c/rbc_oracle.c -O3, one instance per thread, {dt:.2f} s wall",
            "simd": bool(corc.lib().orc_simd_enabled())}


# TDec roofline constants.  Every Fp multiplication / squaring the kernels run
# is a generated 12x12-limb Montgomery CIOS body of 288 v_mad_u64_u32
# (tools/gen_bls_fp_sub.py: the hbg_fpmul1/2/3 subroutines; counted in the gfx950 asm).  The peak is the measured
# v_mad_u64_u32 issue rate — 4.44 cycles per wave-instruction per SIMD at 8
# waves/SIMD (profiles/r01/valu_issue_rates_ubench2.txt) — at the 2.4 GHz
# nominal clock on 1,024 SIMDs: 35.4 T lane-MADs/s.
REALTIME_HZ = 100e6  # s_memrealtime: the constant 100 MHz clock of CDNA3/4
MADS_PER_FP_MUL = 288
MAD_PEAK = 256 * 4 * 64 / 4.44 * 2.4e9
# The issue bound of a whole Fp multiplication: 288 v_mad_u64_u32 + 288
# v_addc_co_u32_e64 (both half rate on gfx950: 4.34 / 4.33 cycles per
# wave-instruction per SIMD at 8 waves/SIMD, profiles/r03/ubench5_fp_mul_issue.txt)
# + ~100 full-rate VALU (2.25): 2,720 cycles per wave-multiplication, so
# 1,024 SIMDs x 64 lanes x 2.4 GHz / 2,720 = 57.8 G Fp mul/s chip-wide.
FP_MUL_ISSUE_CYCLES = 288 * 4.34 + 288 * 4.33 + 100 * 2.25
FP_MUL_PEAK = 256 * 4 * 64 * 2.4e9 / FP_MUL_ISSUE_CYCLES


def fp_count_profile(n_nodes: int, t: int, bad_rate: float) -> dict:
    """Per-share Fp-multiplication counts of the ThresholdDecrypt driver's
    kernels, measured by the instrumented build (tools/fpcount.py ->
    profiles/fpcount.json) on the same generator at a smaller ciphertext
    count; empty when the committed profile is for another shape."""
    path = os.path.join(ROOT, "profiles", "fpcount.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return {}
    sh = d.get("shape", {})
    if (sh.get("n_nodes"), sh.get("t"), sh.get("bad_rate")) != (n_nodes, t, bad_rate):
        return {}
    d["path"] = os.path.relpath(path, ROOT)
    d["measured_at_head"] = measured_at_head(d)
    return d


# Kernels whose Fp work is per call (the N public-key shares), not per share:
# their profiled count is re-spread over this run's share count.
FP_FIXED_PER_CALL = ("tdec_pk_table", "tdec_pk_prepare")


def fp_per_share(prof: dict, key: str, n_shares: int) -> float:
    """Fp multiplications per share at n_shares from the profile's per-kernel
    counts (per-share and per-ciphertext kernels scale with the shares; the
    per-call key-table work is divided by this run's share count)."""
    total = 0.0
    for name, v in prof[key].items():
        total += (v["fp_mul"] + v["fp_sqr"]) / n_shares if name in FP_FIXED_PER_CALL else v["per_share"]
    return total


# Kernels of one hbg_tdec_threshold_decrypt call (the epoch generator's
# encrypt / decrypt_share kernels in the same profile are not part of it).
TDEC_DRIVER_KERNELS = ("tdec_pk_prepare", "tdec_ct_decode", "tdec_ct_prepare", "tdec_ct_prepare_w", "tdec_ct_prepare_hw", "tdec_v_digest",
                       "tdec_ct_verify", "tdec_pair_index", "tdec_pk_table", "tdec_iota", "tdec_group_marks",
                       "tdec_batch_heads", "tdec_batch_desc", "tdec_batch_leaves", "tdec_bin_root", "tdec_bin_step",
                       "tdec_verify_shares", "tdec_select", "tdec_combine_msm", "tdec_combine_seed",
                       "tdec_keystream_xor", "tdec_status_merge", "tdec_index_sanitize")


def tdec_pmc_traffic(n_shares: int) -> dict:
    """HBM bytes of one ThresholdDecrypt call at the bench shape (100k x 64,
    1 % bad), from the committed rocprofv3 PMC passes (FETCH_SIZE x2 +
    WRITE_SIZE per dispatch, profiles/r05/pmc_tdec_100k.json over
    tools/tdec_kbench.py --cts 100000: the LDS Miller accumulator and the
    binary check rounds); per-dispatch averages times the dispatches per call."""
    path = newest("profiles/r06/pmc_tdec_100k.json", "profiles/r05/pmc_tdec_100k.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return {}
    per_call = {"tdec_bin_step": 6}
    per_kernel = {}
    for name, v in d.items():
        short = name.split("::")[-1].split("<")[0]
        if "bls_lat" in name or short not in TDEC_DRIVER_KERNELS or not isinstance(v, dict):
            continue
        if "hbm_read_bytes_corrected" in v:
            per_kernel[short] = (v["hbm_read_bytes_corrected"] + v["hbm_write_bytes"]) * per_call.get(short, 1)
    if not per_kernel or n_shares != 6_400_000:
        return {}
    total = sum(per_kernel.values())
    return {"bytes_per_call": total, "bytes_per_share": total / n_shares,
            "per_kernel_bytes_per_share": {k: v / n_shares for k, v in sorted(per_kernel.items(), key=lambda x: -x[1])},
            "source": os.path.relpath(path, ROOT) + " (tools/pmc_tdec.sh, KB_ARGS='--cts 100000 --reps 1', "
                      "EXTRA_GROUPS='FETCH_SIZE WRITE_SIZE')",
            "kernels_measured": sorted(per_kernel), "measured_at_head": measured_at_head(d)}


def fp_count_floor() -> dict:
    """The batched verifier's executed Fp count with no bad share (no group
    testing, no per-share fallback): profiles/r06/ (or r05/) fpcount_batched_0pct.json."""
    path = newest("profiles/r06/fpcount_batched_0pct.json", "profiles/r05/fpcount_batched_0pct.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return {}
    return {"per_share_total": d["per_share_total"], "per_share_verify_total": d["per_share_verify_total"],
            "source": os.path.relpath(path, ROOT), "measured_at_head": measured_at_head(d)}


def kernel_meta(names) -> dict:
    """VGPR / scratch / waves-per-SIMD of the named kernels (tools/kernel_meta.py)."""
    try:
        k = json.load(open(os.path.join(ROOT, "profiles", "kernel_meta.json")))["kernels"]
    except (OSError, ValueError, KeyError):
        return {}
    out = {}
    for mangled, v in k.items():
        if "bls_lat" in mangled:  # the one-wave latency build of the same kernels
            continue
        for n in names:
            if f"{len(n)}{n}E" in mangled or f"{len(n)}{n}I" in mangled:
                out[n] = {x: v[x] for x in ("vgpr", "agpr", "sgpr", "scratch_bytes", "lds_bytes",
                                            "waves_per_simd_by_regs")}
    return out


def cpu_baseline_tdec(ep, n_ct: int = 512):
    """The C restatement of threshold_crypto's per-share algorithm
    (oracle/c/bls_oracle.c: share decode with the crate's [r]P subgroup check,
    hash_g1_g2 recomputed per call, two full pairings per
    verify_decryption_share) on the first n_ct ciphertexts of the SAME
    device-generated epoch the GPU leg runs: verify all N shares of each,
    then PublicKeySet::decrypt of the first t+1 valid ones (node order), one
    contiguous block of shares per host thread.  512 ciphertexts: ~15 s of
    CPU work on 16 threads (64 in rounds 1-4: under 2 s)."""
    from hydrabadger_amd import tdec_workload as tw
    from oracle import corb
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    threads = max(1, min(threads, os.cpu_count() or 1, 64))
    N, t, L = ep.n_nodes, ep.t, ep.msg_len
    U = ep.U[:n_ct].cpu().numpy().reshape(-1).copy()
    W = ep.W[:n_ct].cpu().numpy().reshape(-1).copy()
    V = np.concatenate([ep.V[:n_ct * L].cpu().numpy(), np.zeros(1, np.uint8)])
    off = (np.arange(n_ct + 1, dtype=np.uint64) * L)
    pk = ep.pk48.cpu().numpy().reshape(-1).copy()
    sh = ep.share48[:n_ct].cpu().numpy().reshape(-1).copy()
    sct = np.repeat(np.arange(n_ct, dtype=np.uint32), N)
    spk = np.tile(np.arange(N, dtype=np.uint32), n_ct)
    t0 = time.perf_counter()
    ok = corb.verify_shares_arrays(threads, U, V, off, W, pk, sh, sct, spk)
    tv = time.perf_counter() - t0
    acc = tw.expected_outcomes(ep.bad[:n_ct], t) == 1
    ix = np.stack([np.nonzero(acc[k])[0][: t + 1] for k in range(n_ct)]).astype(np.uint32)
    csh = ep.share48[:n_ct].cpu().numpy()[np.arange(n_ct)[:, None], ix].reshape(-1).copy()
    t0 = time.perf_counter()
    out, st = corb.decrypt_arrays(threads, t, csh, ix.reshape(-1).copy(), V, off)
    tc = time.perf_counter() - t0
    ref = ep.msgs[:n_ct * L].cpu().numpy().tobytes()
    return {"value": n_ct * N / (tv + tc), "unit": "shares/s", "cores": threads, "kind": "port",
            "verify_shares_per_s": n_ct * N / tv, "combine_cts_per_s": n_ct / tc,
            "sample": f"{n_ct} ciphertexts x {N} shares of the bench's device-generated epoch: {n_ct * N} "
                      f"verify_decryption_share in {tv:.2f} s + {n_ct} PublicKeySet::decrypt (t={t}) in {tc:.2f} s, "
                      f"oracle/c/bls_oracle.c -O3 (64-bit limbs, the crate's per-share algorithm), {threads} threads",
            "bits_match": bool(np.array_equal(ok.astype(bool), ~ep.bad[:n_ct].reshape(-1))),
            "plaintexts_match": bool((st == 0).all()) and out[:len(ref)].tobytes() == ref}


def tdec_leg(ctx, dev, n_ct: int, reps: int, seed: int = 1, bad_rate: float = 0.01, per_share: bool = True):
    """BASELINE.json configs[3]: one node's ThresholdDecrypt for an epoch of
    n_ct DISTINCT ciphertexts (N=64, t=21), device-generated
    (hydrabadger_amd/tdec_workload.py: encrypt_with_rng + every node's
    decrypt_share_no_verify, 1 % of the shares replaced by three kinds of bad
    share), through hbg_tdec_threshold_decrypt: Ciphertext::verify, all 64
    shares verified, first t+1 valid selected (faults / ignored late shares),
    PublicKeySet::decrypt.  Inputs HBM-resident; the verify call alone is
    timed beside it.  per_share=False leaves out the HBG_VERIFY_PER_SHARE
    pass (tools/tdec_kbench.py under the PMC passes, whose per-kernel
    averages must hold the batched call's launches only)."""
    from hydrabadger_amd import _lib
    from hydrabadger_amd import tdec_workload as tw
    from hydrabadger_amd import threshold as th
    t_gen = time.perf_counter()
    ep = tw.make_epoch(ctx, dev, n_ct, N_NODES, 256, bad_rate, seed)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen
    N, t = ep.n_nodes, ep.t
    n = n_ct * N
    pt = torch.zeros(n_ct * ep.msg_len, dtype=torch.uint8, device=dev)
    st = torch.zeros(n_ct, dtype=torch.int32, device=dev)
    oc = torch.zeros((n_ct, N), dtype=torch.uint8, device=dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    sct = torch.arange(n_ct, dtype=torch.int32, device=dev).repeat_interleave(N)
    spk = torch.arange(N, dtype=torch.int32, device=dev).repeat(n_ct)
    A = _lib.HBG_DEVICE | _lib.HBG_ASYNC

    def run():
        th.threshold_decrypt_arrays(t, N, ep.U, ep.V, ep.V_off, ep.W, ep.pk48, ep.share48, None, pt, st, oc,
                                    ctx=ctx, device=True, asynchronous=True)

    def verify():
        _lib.check(_lib.lib().hbg_tdec_verify_shares(ctx.h, n_ct, ep.U.data_ptr(), ep.V.data_ptr(),
                                                     ep.V_off.data_ptr(), ep.W.data_ptr(), N, ep.pk48.data_ptr(), n,
                                                     ep.share48.data_ptr(), sct.data_ptr(), spk.data_ptr(),
                                                     ok.data_ptr(), A), "verify")
    run()
    verify()
    ctx.sync()
    outcomes_ok = bool(np.array_equal(oc.cpu().numpy(), tw.expected_outcomes(ep.bad, t)))
    bits_ok = bool(np.array_equal(ok.cpu().numpy().astype(bool), ~ep.bad.reshape(-1)))
    pts_ok = bool((st == 0).all().item()) and bool(torch.equal(pt, ep.msgs))
    ms = timed(run, reps)
    ms_v = timed(verify, reps)
    # the deterministic schedule (hbg_set_share_verify(HBG_VERIFY_PER_SHARE): the
    # crate's pairing equation per share) on the same shares: its time and bits
    ms_ps, ps_bits_ok = None, None
    if per_share:
        ctx.set_share_verify(_lib.HBG_VERIFY_PER_SHARE)
        try:
            ok.zero_()
            ms_ps = timed(verify, 1)
            ps_bits_ok = bool(np.array_equal(ok.cpu().numpy().astype(bool), ~ep.bad.reshape(-1)))
        finally:
            ctx.set_share_verify(_lib.HBG_VERIFY_BATCHED)
    kinds = {tw.BAD_KINDS[k]: int((ep.kind == k).sum()) for k in range(3)}
    out = {"metric": "TDec shares/s (ThresholdDecrypt: ct verify + verify_decryption_share + select + decrypt) "
                     "at N=64 t=21", "unit": "shares/s",
           "value": n / (ms * 1e-3), "threshold_decrypt_ms": ms, "verify_ms": ms_v,
           "verify_shares_per_s": n / (ms_v * 1e-3), "decrypt_cts_per_s": n_ct / (ms * 1e-3),
           "n_ct": n_ct, "shares": n, "corrupted": int(ep.bad.sum()), "corrupted_by_kind": kinds,
           "faults_reported": int((oc == _lib.HBG_SHARE_FAULTY).sum().item()),
           "ok_bits_match": bits_ok, "outcomes_match": outcomes_ok, "plaintexts_match": pts_ok,
           "batch_weights": {"bits": 127, "form": "a + b|x| + c x^2 + d|x|^3, a odd, a..d the four 32-bit "
                                                  "words of SHA3(K || batch digest || lane)",
                             "key": "32 secret bytes from getrandom(2) at hbg_init",
                             "soundness": "a (sub)batch check holding an invalid share passes with "
                                          "probability <= 2^-127",
                             "round5_threshold_decrypt_ms": 824.3,
                             "round5_note": "32-bit public Fiat-Shamir halves (2^-63, grindable), BENCH_r05.json"},
           "per_share_schedule": {"verify_ms": ms_ps, "verify_shares_per_s": n / (ms_ps * 1e-3) if ms_ps else None,
                                  "bits_match": ps_bits_ok,
                                  "note": "hbg_set_share_verify(HBG_VERIFY_PER_SHARE): every bit the crate's own "
                                          "pairing equation, deterministic"},
           "inputs": f"distinct: {n_ct} ciphertexts of 256-B contributions encrypted on the device under a seeded "
                     f"degree-{t} key set, all {N} decryption shares per ciphertext made on the device, "
                     f"{bad_rate:.0%} replaced (three kinds); generated in {t_gen:.1f} s, HBM-resident"}
    prof = fp_count_profile(N, t, bad_rate)
    if prof:
        per_share = fp_per_share(prof, "kernels", n)
        achieved = per_share * MADS_PER_FP_MUL * n / (ms * 1e-3)
        per_share_v = fp_per_share(prof, "verify_kernels", n)
        achieved_v = per_share_v * MADS_PER_FP_MUL * n / (ms_v * 1e-3)
        out["roofline"] = {
            "kernel": "hbg_tdec_threshold_decrypt (all its kernels; per-kernel counts in the profile)",
            "bound": "valu", "unit": "T v_mad_u64_u32/s",
            "achieved": achieved / 1e12, "peak": MAD_PEAK / 1e12, "frac": achieved / MAD_PEAK,
            "fp_mul_per_share": per_share, "mads_per_fp_mul": MADS_PER_FP_MUL,
            "fp_mul_issue_bound": {
                "achieved_G_fp_mul_per_s": per_share * n / (ms * 1e-3) / 1e9,
                "peak_G_fp_mul_per_s": FP_MUL_PEAK / 1e9,
                "frac": per_share * n / (ms * 1e-3) / FP_MUL_PEAK,
                "note": "peak = whole-multiplication issue rate (288 mad + 288 addc, both half rate, + ~100 "
                        "full-rate VALU) measured on gfx950 (profiles/r03/ubench5_fp_mul_issue.txt)"},
            "verify_only": {"achieved": achieved_v / 1e12, "frac": achieved_v / MAD_PEAK,
                            "fp_mul_per_share": per_share_v},
            "traffic": None, "count_source": prof["path"] + " (" + prof.get("source", "") + ")",
            "count_measured_at_head": prof.get("measured_at_head"),
            "count_note": "counted at this round's kernels by the branch-free instrumented build (one atomic add per "
                          "active lane per Fp product; DESIGN.md §4 'The HBG_FP_COUNT fault'), outputs checked "
                          "against the product's",
            "peak_source": "v_mad_u64_u32 4.44 cyc/wave-instr/SIMD (profiles/r01/valu_issue_rates_ubench2.txt) "
                           "x 1024 SIMDs x 64 lanes x 2.4 GHz",
            "note": "each Fp mul also issues 288 v_addc (carry) + ~95 other VALU: frac <= ~0.5 by construction",
            "occupancy": kernel_meta(["tdec_batch_leaves", "tdec_bin_step", "tdec_verify_shares",
                                      "tdec_ct_prepare", "tdec_ct_verify", "tdec_combine_msm"]),
        }
        floor = fp_count_floor()
        if floor:
            # executed count at this bad-share rate vs the same algorithm with no bad share
            out["roofline"]["fp_mul_per_share_no_bad_shares"] = floor["per_share_total"]
            out["roofline"]["executed_vs_no_bad_shares"] = per_share / floor["per_share_total"]
            out["roofline"]["verify_only"]["executed_vs_no_bad_shares"] = per_share_v / floor["per_share_verify_total"]
            out["roofline"]["floor_source"] = floor["source"]
            out["roofline"]["floor_measured_at_head"] = floor["measured_at_head"]
        tr = tdec_pmc_traffic(n)
        if tr:
            out["roofline"]["traffic"] = tr["bytes_per_call"]
            out["roofline"]["traffic_unit"] = "HBM bytes per hbg_tdec_threshold_decrypt call (PMC)"
            out["roofline"]["traffic_per_share"] = tr["bytes_per_share"]
            out["roofline"]["traffic_per_share_by_kernel"] = tr["per_kernel_bytes_per_share"]
            out["roofline"]["traffic_source"] = tr["source"]
            out["roofline"]["traffic_kernels_measured"] = tr["kernels_measured"]
            out["roofline"]["traffic_measured_at_head"] = tr["measured_at_head"]
    return out, ep


def _dev_scalars(n: int, dev, seed: int):
    """n 32-byte little-endian scalars < 2^254 (< r), device-resident, seeded."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    r = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g)
    r[:, 31] &= 0x3F
    return r.to(dev)


def wire_leg(ctx, dev, n_msgs: int, msg_len: int, reps: int):
    """SecretKey::sign + PublicKey::verify of n_msgs wire
    messages (64 signing nodes, msg_len-byte messages), device-resident."""
    from hydrabadger_amd import _lib
    L = _lib.lib()
    flags = _lib.HBG_DEVICE | _lib.HBG_ASYNC
    g = torch.Generator(device="cpu").manual_seed(0x5167)
    msgs = torch.randint(0, 256, (n_msgs, msg_len), dtype=torch.uint8, generator=g)
    msgs[:, :4] = torch.tensor([7, 0, 0, 0], dtype=torch.uint8)  # WireMessageKind::Message: poll verifies it
    msgs[:, 4:12] = torch.tensor([16, 0, 0, 0, 0, 0, 0, 0], dtype=torch.uint8)  # its Uid: a 16-byte uuid
    msgs = msgs.reshape(-1).to(dev)
    off = (torch.arange(n_msgs + 1, dtype=torch.int64) * msg_len).to(dev)
    flen = 4 + 8 + msg_len + 96
    foff = (torch.arange(n_msgs + 1, dtype=torch.int64) * flen).to(dev)
    frames = torch.empty(n_msgs * flen + 16, dtype=torch.uint8, device=dev)
    fst = torch.empty(n_msgs, dtype=torch.int32, device=dev)
    n_keys = 64
    sk = _dev_scalars(n_keys, dev, 17)
    from oracle import bls12_381 as B  # checker only: public keys of the 64 signers
    sk_host = sk.cpu().numpy()
    pk = torch.from_numpy(np.frombuffer(b"".join(
        B.g1_compress(B.g1_mul(B.G1, int.from_bytes(sk_host[i].tobytes(), "little"))) for i in range(n_keys)),
        np.uint8).copy()).to(dev)
    who = (torch.arange(n_msgs, dtype=torch.int32) % n_keys).to(dev)
    sig = torch.empty((n_msgs, 96), dtype=torch.uint8, device=dev)
    ok = torch.empty(n_msgs, dtype=torch.uint8, device=dev)

    def sign():
        _lib.check(L.hbg_bls_sign(ctx.h, n_keys, sk.data_ptr(), n_msgs, who.data_ptr(), msgs.data_ptr(),
                                  off.data_ptr(), sig.data_ptr(), flags), "sign")

    def verify():
        _lib.check(L.hbg_bls_verify(ctx.h, n_keys, pk.data_ptr(), n_msgs, who.data_ptr(), msgs.data_ptr(),
                                    off.data_ptr(), sig.data_ptr(), ok.data_ptr(), flags), "verify")
    def sign_frames():  # §8(f4): WireMessages::start_send (sign + SignedWireMessage + codec frame)
        _lib.check(L.hbg_wire_sign_frames(ctx.h, n_keys, sk.data_ptr(), n_msgs, who.data_ptr(), msgs.data_ptr(),
                                          off.data_ptr(), frames.data_ptr(), foff.data_ptr(), flags), "sign_frames")

    def poll_frames():  # WireMessages::poll (frame + bincode checks, kind, PublicKey::verify)
        _lib.check(L.hbg_wire_verify_frames(ctx.h, n_keys, pk.data_ptr(), n_msgs, who.data_ptr(), frames.data_ptr(),
                                            foff.data_ptr(), fst.data_ptr(), flags), "poll_frames")
    sign()
    verify()
    sign_frames()
    poll_frames()
    torch.cuda.synchronize()
    all_ok = bool(ok.all().item())
    frames_ok = bool((fst == 0).all().item()) and bool(torch.equal(
        frames[:n_msgs * flen].reshape(n_msgs, flen)[:, flen - 96:], sig))
    ms_s = timed(sign, reps)
    ms_v = timed(verify, reps)
    ms_sf = timed(sign_frames, reps)
    ms_pf = timed(poll_frames, reps)
    return {"workload": f"{n_msgs} wire messages x {msg_len} B, 64 signers (SecretKey::sign / PublicKey::verify)",
            "sign_per_s": n_msgs / (ms_s * 1e-3), "verify_per_s": n_msgs / (ms_v * 1e-3), "sign_ms": ms_s,
            "verify_ms": ms_v, "all_verified": all_ok,
            "frames": {"workload": "WireMessages::start_send / poll: SignedWireMessage in LengthDelimitedCodec frames",
                       "sign_frames_per_s": n_msgs / (ms_sf * 1e-3), "poll_frames_per_s": n_msgs / (ms_pf * 1e-3),
                       "sign_frames_ms": ms_sf, "poll_frames_ms": ms_pf, "all_accepted": frames_ok}}


def tdec_inputs_leg(ctx, dev, n_ct: int, n_nodes: int, reps: int):
    """PublicKey::encrypt_with_rng of n_ct 256-B contributions
    and every node's SecretKeyShare::decrypt_share_no_verify (n_ct x n_nodes)."""
    from hydrabadger_amd import _lib
    L = _lib.lib()
    flags = _lib.HBG_DEVICE | _lib.HBG_ASYNC
    from hydrabadger_amd import tdec_workload as tw
    pk48 = torch.from_numpy(np.frombuffer(tw.G1_GENERATOR, np.uint8).copy()).to(dev)  # any G1 point
    msg_len = 256
    gen = torch.Generator(device="cpu").manual_seed(0x48424247)
    msgs = torch.randint(0, 256, (n_ct * msg_len,), dtype=torch.uint8, generator=gen).to(dev)
    off = (torch.arange(n_ct + 1, dtype=torch.int64) * msg_len).to(dev)
    r = _dev_scalars(n_ct, dev, 23)
    U = torch.empty((n_ct, 48), dtype=torch.uint8, device=dev)
    V = torch.empty(n_ct * msg_len, dtype=torch.uint8, device=dev)
    W = torch.empty((n_ct, 96), dtype=torch.uint8, device=dev)
    sk = _dev_scalars(n_nodes, dev, 29)
    n = n_ct * n_nodes
    sc = torch.arange(n_ct, dtype=torch.int32, device=dev).repeat_interleave(n_nodes)
    ss = torch.arange(n_nodes, dtype=torch.int32, device=dev).repeat(n_ct)
    sh = torch.empty((n, 48), dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)

    def enc():
        _lib.check(L.hbg_tdec_encrypt(ctx.h, pk48.data_ptr(), n_ct, r.data_ptr(), msgs.data_ptr(), off.data_ptr(),
                                      U.data_ptr(), V.data_ptr(), W.data_ptr(), flags), "encrypt")

    def shares():
        _lib.check(L.hbg_tdec_decrypt_shares(ctx.h, n_ct, U.data_ptr(), n_nodes, sk.data_ptr(), n, sc.data_ptr(),
                                             ss.data_ptr(), sh.data_ptr(), st.data_ptr(), flags), "decrypt_share")
    enc()
    shares()
    torch.cuda.synchronize()
    ok = bool((st == 0).all().item())
    ms_e = timed(enc, reps)
    ms_d = timed(shares, reps)
    return {"workload": f"{n_ct} x 256-B contributions encrypted, {n_ct} x {n_nodes} decryption shares",
            "encrypt_per_s": n_ct / (ms_e * 1e-3), "decrypt_shares_per_s": n / (ms_d * 1e-3),
            "encrypt_ms": ms_e, "decrypt_shares_ms": ms_d, "status_ok": ok}


def coin_leg(ctx, dev, n_coins: int, n_nodes: int, reps: int):
    """threshold_sign common coin at N=n_nodes, t=(N-1)/3 —
    every node signs every coin's nonce (hbg_bls_sign with key shares), all
    shares verified with 1 % of them replaced by another node's share
    (hbg_sig_verify_shares: hash_g2 once per coin, weighted batches; the
    per-share hbg_bls_verify timed beside it), first t+1 combined + parity
    (hbg_sig_combine).  Device-resident."""
    from hydrabadger_amd import _lib
    from oracle import bls12_381 as B  # checker only: key material of a seeded degree-t polynomial
    L = _lib.lib()
    flags = _lib.HBG_DEVICE | _lib.HBG_ASYNC
    t = (n_nodes - 1) // 3
    rng = np.random.default_rng(0x5167)
    coeffs = [int.from_bytes(rng.bytes(31), "little") for _ in range(t + 1)]
    sks = [sum(c * pow(i + 1, j, B.R) for j, c in enumerate(coeffs)) % B.R for i in range(n_nodes)]
    pk_shares = b"".join(B.g1_compress(B.g1_mul(B.G1, k)) for k in sks)
    master_pk = B.g1_compress(B.g1_mul(B.G1, coeffs[0]))
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    sk = d(np.frombuffer(b"".join(k.to_bytes(32, "little") for k in sks), np.uint8).copy())
    pk = d(np.frombuffer(pk_shares, np.uint8).copy())
    mpk = d(np.frombuffer(master_pk, np.uint8).copy())
    n = n_coins * n_nodes
    nonce_len = 32
    docs = torch.from_numpy(np.frombuffer(rng.bytes(n_coins * nonce_len), np.uint8).copy()).to(dev)
    # message k = coin k // N's nonce, signed by node k % N
    msgs = docs.view(n_coins, nonce_len).repeat_interleave(n_nodes, dim=0).reshape(-1).contiguous()
    off = (torch.arange(n + 1, dtype=torch.int64, device=dev) * nonce_len)
    who = (torch.arange(n, dtype=torch.int32, device=dev) % n_nodes)
    sig = torch.empty((n, 96), dtype=torch.uint8, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    ix = torch.arange(t + 1, dtype=torch.int32, device=dev).repeat(n_coins)
    comb_sh = torch.empty((n_coins, t + 1, 96), dtype=torch.uint8, device=dev)
    out = torch.empty((n_coins, 96), dtype=torch.uint8, device=dev)
    par = torch.empty(n_coins, dtype=torch.uint8, device=dev)
    st = torch.empty(n_coins, dtype=torch.int32, device=dev)

    def sign():
        _lib.check(L.hbg_bls_sign(ctx.h, n_nodes, sk.data_ptr(), n, who.data_ptr(), msgs.data_ptr(), off.data_ptr(),
                                  sig.data_ptr(), flags), "coin sign")

    # 1 % of the verified shares claim another node's share of the same coin
    bad = torch.from_numpy(rng.random(n) < 0.01).to(dev)
    sig_v = torch.empty_like(sig)
    share_doc = (torch.arange(n, dtype=torch.int32, device=dev) // n_nodes)
    off_c = torch.arange(n_coins + 1, dtype=torch.int64, device=dev) * nonce_len
    ok1 = torch.empty(n, dtype=torch.uint8, device=dev)

    def verify():
        _lib.check(L.hbg_sig_verify_shares(ctx.h, n_coins, docs.data_ptr(), off_c.data_ptr(), n_nodes, pk.data_ptr(),
                                           n, sig_v.data_ptr(), share_doc.data_ptr(), who.data_ptr(), ok.data_ptr(),
                                           flags), "coin verify")

    def verify_per_share():
        _lib.check(L.hbg_bls_verify(ctx.h, n_nodes, pk.data_ptr(), n, who.data_ptr(), msgs.data_ptr(), off.data_ptr(),
                                    sig_v.data_ptr(), ok1.data_ptr(), flags), "coin verify per share")

    def combine():
        comb_sh.copy_(sig.view(n_coins, n_nodes, 96)[:, : t + 1])
        _lib.check(L.hbg_sig_combine(ctx.h, t, n_coins, comb_sh.data_ptr(), ix.data_ptr(), out.data_ptr(),
                                     par.data_ptr(), st.data_ptr(), flags), "coin combine")
    sign()
    sh = sig.view(n_coins, n_nodes, 96)
    sig_v.copy_(torch.where(bad.view(n_coins, n_nodes, 1), sh.roll(1, dims=1), sh).view(n, 96))
    verify()
    verify_per_share()
    combine()
    # the combined signatures verify under the master key
    ok_m = torch.empty(n_coins, dtype=torch.uint8, device=dev)
    zeros = torch.zeros(n_coins, dtype=torch.int32, device=dev)
    _lib.check(L.hbg_bls_verify(ctx.h, 1, mpk.data_ptr(), n_coins, zeros.data_ptr(), docs.data_ptr(), off_c.data_ptr(),
                                out.data_ptr(), ok_m.data_ptr(), flags), "master verify")
    torch.cuda.synchronize()
    good = (bool(torch.equal(ok, (~bad).to(torch.uint8))) and bool(torch.equal(ok1, ok))
            and bool((st == 0).all().item()) and bool(ok_m.all().item()))
    ms_s, ms_v, ms_c = timed(sign, reps), timed(verify, reps), timed(combine, reps)
    ms_v1 = timed(verify_per_share, 1)
    return {"workload": f"{n_coins} coins x {n_nodes} signature shares (t={t}), 1 % of the verified shares wrong",
            "share_sign_per_s": n / (ms_s * 1e-3), "share_verify_per_s": n / (ms_v * 1e-3),
            "share_verify_per_share_path_per_s": n / (ms_v1 * 1e-3), "wrong_shares": int(bad.sum().item()),
            "combine_coins_per_s": n_coins / (ms_c * 1e-3), "coins_per_s": n_coins / ((ms_s + ms_v + ms_c) * 1e-3),
            "heads_fraction": float(par.float().mean().item()), "all_ok": good}


def rbc_config_leg(ctx, dev, n_nodes: int, payload: int, n_inst: int, reps: int, config: str):
    """encode+Merkle (send_shards) and decode (2f erasures) throughput of one
    RBC configuration at batch size, with the VALU fraction of its
    merkle_build launch (the same algorithmic count as the headline) and the
    decode round trip checked."""
    from hydrabadger_amd import _lib, workload
    from hydrabadger_amd import broadcast as bc
    L = _lib.shard_len(n_nodes, payload)
    S = (L + 15) // 16 * 16
    nodes = _lib.merkle_nodes(n_nodes)
    data, parity = bc.shard_counts(n_nodes)
    PS = (payload + 15) // 16 * 16
    pay = torch.zeros((n_inst, PS), dtype=torch.uint8, device=dev)
    bc.synth_bytes(1, 0x10000000, payload, pay, ctx=ctx, device=True)
    plen = torch.full((n_inst,), payload, dtype=torch.int64, device=dev)
    shards = torch.empty((n_inst, n_nodes, S), dtype=torch.uint8, device=dev)
    levels = torch.empty((n_inst, nodes, 32), dtype=torch.uint8, device=dev)

    def enc():
        bc.rbc_encode_merkle_batch(n_nodes, pay, plen, L, shards, levels, ctx=ctx, device=True, asynchronous=True)

    def mk():
        bc.merkle_build_batch(n_nodes, L, shards, levels, ctx=ctx, device=True, asynchronous=True)
    enc()
    ms_step = timed(enc, reps)
    ms_merkle = timed(mk, reps)
    present = torch.tensor([workload.erasure_mask(0x10000000 + k, n_nodes, parity) for k in range(n_inst)],
                           dtype=torch.uint8, device=dev)
    roots = levels[:, nodes - 1, :].contiguous()
    OS = (data * L + 15) // 16 * 16
    out = torch.empty((n_inst, OS), dtype=torch.uint8, device=dev)
    dplen = torch.empty(n_inst, dtype=torch.int64, device=dev)
    st = torch.empty(n_inst, dtype=torch.uint8, device=dev)
    work = shards.clone()

    def dec():
        bc.rbc_decode_batch(n_nodes, L, work, present, roots, out, dplen, st, ctx=ctx, device=True,
                            asynchronous=True)
    dec()
    torch.cuda.synchronize()
    ok = bool((st == 1).all().item()) and bool(torch.equal(out[:, :payload], pay[:, :payload]))
    ms_dec = timed(dec, reps)
    ops, _ = merkle_alg(n_nodes, L)
    achieved = ops * n_inst / (ms_merkle * 1e-3)
    return {"config": config, "n_nodes": n_nodes, "f": (n_nodes - 1) // 3, "rs": f"{data}+{parity}",
            "payload_bytes": payload, "shard_len": L, "instances": n_inst,
            "encode_merkle_GBps": n_inst * payload / (ms_step * 1e-3) / 1e9, "encode_merkle_ms": ms_step,
            "merkle_build_ms": ms_merkle, "rs_encode_ms": max(ms_step - ms_merkle, 0.0),
            "merkle_valu": {"achieved": achieved / 1e12, "peak": VALU_PEAK / 1e12, "frac": achieved / VALU_PEAK,
                            "unit": "T int32 lane-ops/s", "alg_ops_per_instance": ops},
            "decode_GBps": n_inst * payload / (ms_dec * 1e-3) / 1e9, "decode_ms": ms_dec,
            "erased_per_instance": parity, "roundtrip_ok": ok}


def broadcast_wire_leg(ctx, dev, shards, levels, L: int, n_inst: int, reps: int):
    """every Value message (bincode Message::Value(proof(i)))
    of n_inst encoded N=64 instances written from the shard batch + levels,
    parsed back into the validate table, and validated (Proof::validate)."""
    from hydrabadger_amd import _lib
    from hydrabadger_amd import broadcast as bc
    N = shards.shape[1]
    S = shards.shape[2]
    m = n_inst * N
    idx = np.tile(np.arange(N, dtype=np.uint32), n_inst)
    off = bc.proof_msg_offsets(N, L, idx)
    total = int(off[-1])
    d_inst = torch.from_numpy(np.repeat(np.arange(n_inst, dtype=np.int64), N)).to(dev)
    d_idx = torch.from_numpy(idx.astype(np.int32)).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    depth = _lib.merkle_depth(N)
    tag = torch.empty(m, dtype=torch.int32, device=dev)
    vals = torch.empty((m, S), dtype=torch.uint8, device=dev)
    rindex = torch.empty(m, dtype=torch.int32, device=dev)
    dig = torch.empty((m, depth, 32), dtype=torch.uint8, device=dev)
    nd = torch.empty(m, dtype=torch.int32, device=dev)
    roots = torch.empty((m, 32), dtype=torch.uint8, device=dev)
    st = torch.empty(m, dtype=torch.int32, device=dev)
    ok = torch.empty(m, dtype=torch.uint8, device=dev)
    A = _lib.HBG_DEVICE | _lib.HBG_ASYNC

    def write():
        bc.write_proof_msgs_batch(N, L, shards, levels, bc.Message.VALUE, d_inst, d_idx, out, d_off, ctx=ctx,
                                  device=True, asynchronous=True)

    def read():
        bc.read_msgs_batch(N, L, out, d_off, tag, vals, rindex, dig, nd, roots, st, ctx=ctx, device=True,
                           asynchronous=True)

    def validate():
        _lib.check(_lib.lib().hbg_merkle_validate(ctx.h, N, L, _lib.ptr(vals), S, _lib.ptr(rindex), _lib.ptr(dig),
                                                  _lib.ptr(nd), _lib.ptr(roots), _lib.ptr(ok), m, A), "validate")
    write()
    read()
    validate()
    torch.cuda.synchronize()
    good = (bool((st == 0).all().item()) and bool((ok == 1).all().item())
            and bool(torch.equal(vals[:, :L].reshape(n_inst, N, L), shards[:n_inst, :, :L])))
    ms_w, ms_r, ms_v = timed(write, reps), timed(read, reps), timed(validate, reps)
    value_bytes = m * L
    return {"workload": f"{m} Message::Value(proof) of {n_inst} N={N} instances (1 MiB proposals)",
            "msg_bytes": total, "write_ms": ms_w, "read_ms": ms_r, "validate_ms": ms_v,
            "write_hbm_GBps": (value_bytes + total) / (ms_w * 1e-3) / 1e9,
            "read_hbm_GBps": (total + value_bytes) / (ms_r * 1e-3) / 1e9,
            "hbm_frac_write": (value_bytes + total) / (ms_w * 1e-3) / HBM_PEAK,
            "hbm_frac_read": (total + value_bytes) / (ms_r * 1e-3) / HBM_PEAK,
            "validate_proofs_per_s": m / (ms_v * 1e-3), "roundtrip_ok": good}


def epoch_leg(ctx, dev, n_nodes: int, contrib: int, reps: int, agg_dev):
    """configs[4]: one HoneyBadger epoch of ONE n_nodes-node network whose
    nodes are split over all ranks (hydrabadger_amd/epoch.py): threshold-
    encrypt every contribution, the Broadcast Value -> Echo -> Ready rounds as
    bincode wire messages (Values by one all-to-all to their recipients,
    Echoes / Readys / decryption shares by all-gathers: RCCL over xGMI),
    decode, and ThresholdDecrypt of every accepted ciphertext.  The headline
    epoch is per-node faithful: every node validates the Values addressed to
    it and every echo, decodes every instance and runs its own
    ThresholdDecrypt of every accepted ciphertext with its own arrival order
    (the network's whole crypto work, spread over the ranks); the shared view
    (one check / decode / TDec instance per rank for all its nodes) is timed
    beside it, labelled as such.  Timed per phase on every rank, max over
    ranks; every contribution must come out of every node's ThresholdDecrypt
    byte-exact."""
    from hydrabadger_amd import epoch as hbe
    from hydrabadger_amd import network, shard
    eng = network.DeviceEngine(dev, ctx)
    ep = hbe.HoneyBadgerEpoch(n_nodes, contrib, eng, seed=1)

    def check(res, e):
        want = eng.synth(hbe.TAG_CONTRIB, hbe.instance_id(e, 0), n_nodes, contrib)
        return (bool(res.delivered.all()) and res.accepted == list(range(n_nodes))
                and bool((res.ct_status == 0).all())
                and all(bool(torch.equal(res.plaintexts[v], want)) for v in range(len(res.views))))

    def timed_epochs(per_node: bool):
        ok = check(ep.run(epoch=0, per_node=per_node), 0)  # warm
        phases = {}
        for r in range(reps):
            if torch.distributed.is_initialized():
                torch.distributed.barrier()
            res = ep.run(epoch=1 + r, per_node=per_node)
            ok = ok and check(res, 1 + r)
            for k, v in res.times_ms.items():
                phases[k] = phases.get(k, 0.0) + v / reps
        return {k: shard.max_over_ranks(v, agg_dev) for k, v in phases.items()}, res, ok
    phases, res, ok = timed_epochs(True)
    torch.cuda.empty_cache()
    sphases, sres, sok = timed_epochs(False)
    f = (n_nodes - 1) // 3
    work = {k: int(shard.sum_over_ranks(float(v), agg_dev)) for k, v in res.work.items()}
    return {"workload": f"one {n_nodes}-node HoneyBadger epoch (RS {n_nodes - 2 * f}+{2 * f}, t={f}), "
                        f"{contrib}-B contributions threshold-encrypted and broadcast, nodes split over "
                        f"{ep.world} rank(s); per-node faithful (every node's own validations, decodes and "
                        f"ThresholdDecrypt)",
            "nodes_per_rank": ep.m, "epoch_ms": phases["epoch"], "phases_ms": phases,
            "contributions_per_s": n_nodes / (phases["epoch"] * 1e-3),
            "contribution_GBps": n_nodes * contrib / (phases["epoch"] * 1e-3) / 1e9,
            "network_work_per_epoch": work,
            "share_verifications_per_s": work.get("tdec_shares", 0) / (phases["tdec"] * 1e-3),
            "collective_recv_bytes_per_rank": res.exchange_bytes,
            "messages_per_epoch": {"value": n_nodes * n_nodes, "echo": n_nodes * n_nodes,
                                   "ready": n_nodes * n_nodes, "decryption_shares": n_nodes * n_nodes},
            "all_decrypted_ok": ok,
            "shared_view": {"note": "one check / decode / ThresholdDecrypt instance per rank on behalf of all its "
                                    "nodes (round 3's epoch): not the network's work",
                            "epoch_ms": sphases["epoch"], "phases_ms": sphases,
                            "work": {k: int(shard.sum_over_ranks(float(v), agg_dev)) for k, v in sres.work.items()},
                            "all_decrypted_ok": sok}}


def init_distributed(backend: str, local: int):
    """One process per GPU: RANK / WORLD_SIZE / MASTER_* from the launcher."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        torch.distributed.init_process_group(backend, **kw)
    return world, rank


def dist_info(dist: bool) -> dict:
    """What the process group actually saw (not what was asked for): backend,
    ranks in the group, and the RCCL version when the backend is nccl."""
    if not dist:
        return {"backend": None, "world_size_seen": 1, "rccl_version": None}
    backend = torch.distributed.get_backend()
    ver = None
    if backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            ver = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception as e:  # report, never fail the line on it
            ver = f"unavailable: {e}"
    return {"backend": backend, "world_size_seen": torch.distributed.get_world_size(), "rccl_version": ver}


def run_timed(step, steps: int, warmup: int, sync, agg_dev) -> float:
    """W untimed steps, then exactly K steps bracketed by a barrier and a
    device sync on both sides; the max over ranks of the wall time (s)."""
    from hydrabadger_amd import shard
    dist_on = torch.distributed.is_initialized()
    for _ in range(warmup):
        step()
    sync()
    if dist_on:
        torch.distributed.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist_on:
        torch.distributed.barrier()
    return shard.max_over_ranks(time.perf_counter() - t0, agg_dev)


class Legs:
    """Runs the optional legs after the headline; a failing leg is recorded in
    the line (leg_errors) and the others still run (after a device fault they
    fail fast with their own HIP errors, which are recorded too)."""

    def __init__(self):
        self.errors = {}

    def __call__(self, name, fn):
        try:
            return fn()
        except Exception as ex:  # reported in the JSON line, never silently dropped
            self.errors[name] = f"{type(ex).__name__}: {ex}"
            return None


def checks(decode, tdec, cfg1, n128, epoch, bwire, coin, wire) -> dict:
    """Every correctness verdict the legs computed, first in the line (the
    driver keeps only the head of a long line)."""
    def g(d, *path):
        for k in path:
            if not isinstance(d, dict):
                return None
            d = d.get(k)
        return d
    c = {"decode_oracle_match": g(decode, "oracle_match"), "encode_oracle_match": g(decode, "oracle_sample",
                                                                                   "encode_oracle_match"),
         "decode_roundtrip_ok": g(decode, "roundtrip_ok"),
         "tdec_bits_match": g(tdec, "cpu_baseline", "bits_match"),
         "tdec_plaintexts_match": g(tdec, "cpu_baseline", "plaintexts_match"),
         "tdec_driver_outcomes_match": g(tdec, "outcomes_match"), "tdec_driver_bits_match": g(tdec, "ok_bits_match"),
         "tdec_driver_plaintexts_match": g(tdec, "plaintexts_match"),
         "tdec_per_share_bits_match": g(tdec, "per_share_schedule", "bits_match"),
         "config1_roundtrip_ok": g(cfg1, "roundtrip_ok"), "n128_roundtrip_ok": g(n128, "roundtrip_ok"),
         "epoch_all_decrypted_ok": g(epoch, "all_decrypted_ok"), "broadcast_wire_roundtrip_ok": g(bwire, "roundtrip_ok"),
         "coin_all_ok": g(coin, "all_ok"), "wire_all_verified": g(wire, "all_verified")}
    vals = [v for v in c.values() if v is not None]
    c["all_ok"] = bool(vals) and all(bool(v) for v in vals)
    return c


def clock_probe(ctx, step, n_wg: int, dev) -> dict:
    """Core clock the fused kernel ran at: one extra (untimed) launch with the
    in-kernel stamps on (hbg_test_set_clock_probe: s_memtime = shader clock,
    s_memrealtime = 100 MHz constant clock, at every workgroup's entry and
    exit).  clock = sum of shader-clock ticks / sum of real time over all
    workgroups, i.e. the average clock a workgroup saw while resident."""
    from hydrabadger_amd import _lib
    buf = torch.zeros(n_wg * 4, dtype=torch.int64, device=dev)
    _lib.check(_lib.lib().hbg_test_set_clock_probe(ctx.h, buf.data_ptr(), n_wg), "clock probe")
    try:
        step()
        torch.cuda.synchronize()
    finally:
        _lib.check(_lib.lib().hbg_test_set_clock_probe(ctx.h, None, 0), "clock probe off")
    c = buf.view(n_wg, 4).cpu().numpy().astype(np.int64)
    ticks = int((c[:, 1] - c[:, 0]).sum())
    real = int((c[:, 3] - c[:, 2]).sum())
    if real <= 0 or ticks <= 0:
        return {"clock_GHz": None, "note": "no stamps"}
    span_ms = (int(c[:, 3].max()) - int(c[:, 2].min())) / REALTIME_HZ * 1e3
    return {"clock_GHz": ticks / (real / REALTIME_HZ) / 1e9, "workgroups": n_wg, "span_ms": span_ms,
            "mean_workgroup_us": real / n_wg / REALTIME_HZ * 1e6,
            "source": "s_memtime / s_memrealtime (100 MHz) stamps per workgroup of one untimed launch"}


def rbc_oracle_sample(N: int, L: int, shards, levels, pay, present, out, idx) -> dict:
    """Checker (not the product path, outside every timed region): the C
    oracle's send_shards and decode_from_shards on sampled instances of the
    device batch — shards + tree bit-exact, and the 2f-erased decode payload
    equal to the device's decode output and to the original payload."""
    from oracle import corc
    enc_ok = dec_ok = True
    for k in idx:
        p = pay[k].cpu().numpy()
        rs, rl = corc.rbc_encode_merkle(N, p)
        enc_ok &= bool(np.array_equal(shards[k, :, :L].cpu().numpy(), rs[:, :L]) and
                       np.array_equal(levels[k].cpu().numpy(), rl))
        pm = present[k].cpu().numpy()
        dmg = rs[:, :L].copy()
        dmg[pm == 0] = 0
        got = corc.rbc_decode(N, L, dmg, pm, rl[-1].tobytes())
        dec_ok &= got is not None and got == p.tobytes() and got == out[k, :len(got)].cpu().numpy().tobytes()
    return {"instances": [int(k) for k in idx], "encode_oracle_match": enc_ok, "decode_oracle_match": dec_ok}


def main():
    a = parse()
    legs = set(LEGS) if a.legs == "all" else set(a.legs.split(","))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    world, rank = init_distributed(a.backend, local)
    dist = world > 1
    agg_dev = torch.device("cuda", local) if a.backend == "nccl" else torch.device("cpu")

    from hydrabadger_amd import _lib, shard
    from hydrabadger_amd import broadcast as bc
    if os.environ.get("HBG_LAT_LANES"):  # A/B knob of the BLS latency build (hbgpu_testing.h); default untouched
        _lib.lib().hbg_test_set_latency_lanes(int(os.environ["HBG_LAT_LANES"]))

    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(dev)  # one dedicated stream: events and engine launches share it
    torch.cuda.set_stream(stream)
    ctx = _lib.Context(local)
    ctx.set_stream(stream.cuda_stream)

    B = a.instances
    L = _lib.shard_len(N_NODES, PAYLOAD)
    S = (L + 15) // 16 * 16
    nodes = _lib.merkle_nodes(N_NODES)
    data, parity = bc.shard_counts(N_NODES)
    first = shard.instance_block(rank, world, B).start
    pay = torch.empty((B, PAYLOAD), dtype=torch.uint8, device=dev)
    bc.synth_bytes(1, first, PAYLOAD, pay, ctx=ctx, device=True)
    plen = torch.full((B,), PAYLOAD, dtype=torch.int64, device=dev)
    shards = torch.empty((B, N_NODES, S), dtype=torch.uint8, device=dev)
    levels = torch.empty((B, nodes, 32), dtype=torch.uint8, device=dev)

    def step():
        bc.rbc_encode_merkle_batch(N_NODES, pay, plen, L, shards, levels, ctx=ctx, device=True, asynchronous=True)

    dt = run_timed(step, a.steps, a.warmup, torch.cuda.synchronize, agg_dev)
    total_bytes = world * B * PAYLOAD * a.steps
    value = total_bytes / dt / 1e9

    # ---- per-kernel breakdown (rank-local, same stream as the kernels) ----
    # The step is ONE rbc_encode_merkle<22,42> launch (+ the tiny payload
    # length check): the fused schedule, hbg_rbc_encode_merkle's default at
    # N = 64.  The two-launch schedule (rs_encode_const -> merkle_build) is
    # timed beside it for reference.
    reps = max(3, min(a.steps, 10))
    ms_step = timed(step, reps)
    _lib.check(_lib.lib().hbg_test_set_rbc_fused(ctx.h, 0))
    ms_two = timed(step, reps)
    _lib.check(_lib.lib().hbg_test_set_rbc_fused(ctx.h, -1))
    ms_merkle = timed(lambda: bc.merkle_build_batch(N_NODES, L, shards, levels, ctx=ctx, device=True,
                                                     asynchronous=True), reps)
    ms_encode = max(ms_two - ms_merkle, 0.0)
    ops, mbytes = merkle_alg(N_NODES, L)
    enc_ops = encoder_alg_ops(data, parity, L)
    traffic = pmc_traffic(B)
    achieved_ops = (ops + enc_ops) * B / (ms_step * 1e-3)
    fused_bytes = PAYLOAD + N_NODES * L + (2 * N_NODES - 1) * 32  # read payload, write shards + tree once
    enc_bytes = B * (PAYLOAD + N_NODES * L)  # read payload, write N shards
    roofline = {
        "kernel": "rbc_encode_merkle<22,42> (send_shards in one launch: encode + LDS transpose + SHA3-256 leaves "
                  "+ pair tree)",
        "bound": "valu", "unit": "Tops/s",
        "achieved": achieved_ops / 1e12, "peak": VALU_PEAK / 1e12, "frac": achieved_ops / VALU_PEAK,
        "traffic": traffic.get("rbc_encode_merkle_22_42"), "traffic_unit": "HBM bytes per launch (PMC)",
        "traffic_source": traffic.get("rbc_encode_merkle_22_42_source") or traffic.get("source"),
        "traffic_measured_at_head": traffic.get("rbc_encode_merkle_22_42_measured_at_head"),
        "valu_insts_per_wave_pmc": traffic.get("rbc_encode_merkle_22_42_valu_insts_per_wave"),
        "traffic_vs_alg_bytes": (traffic["rbc_encode_merkle_22_42"] / (fused_bytes * B)
                                 if traffic.get("rbc_encode_merkle_22_42") else None),
        "alg_ops_per_instance": ops + enc_ops, "keccak_ops_per_instance": ops, "encoder_ops_per_instance": enc_ops,
        "keccak_f_ops": KECCAK_F_OPS,
        "hbm": {"achieved_GBps": fused_bytes * B / (ms_step * 1e-3) / 1e9, "peak_GBps": HBM_PEAK / 1e9,
                "frac": fused_bytes * B / (ms_step * 1e-3) / HBM_PEAK, "alg_bytes_per_instance": fused_bytes},
        "avg_ms": ms_step, "instances_per_launch": B,
    }
    clk = None
    try:
        clk = clock_probe(ctx, step, B, dev)
        if clk.get("clock_GHz"):
            roofline["clock_GHz"] = clk["clock_GHz"]
            roofline["frac_at_measured_clock"] = achieved_ops / (VALU_PEAK * clk["clock_GHz"] / 2.4)
            roofline["clock"] = clk
    except Exception as e:  # noqa: BLE001 - the probe is a report, never the line
        roofline["clock"] = {"error": repr(e)[:200]}
    kernels = {"rbc_encode_merkle_22_42_ms": ms_step,
               "two_launch": {"ms": ms_two, "merkle_build_ms": ms_merkle, "rs_encode_const_22_42_ms": ms_encode,
                              "merkle_build_valu_frac": ops * B / (ms_merkle * 1e-3) / VALU_PEAK,
                              "merkle_build_traffic_bytes_per_launch": traffic.get("merkle_build"),
                              "rs_encode_traffic_bytes_per_launch": traffic.get("rs_encode_const_22_42"),
                              "rs_encode_hbm_GBps": enc_bytes / (ms_encode * 1e-3) / 1e9 if ms_encode > 0 else None}}

    run_leg = Legs()

    # ---- decode path: reconstruct exactly 2f erasures + tree + glue ----
    def decode_leg():
        from hydrabadger_amd import workload
        nd = B  # the headline batch (reconstruct + tree + glue of every instance the step encoded)
        present = torch.tensor([workload.erasure_mask(first + k, N_NODES, parity) for k in range(nd)],
                               dtype=torch.uint8, device=dev)
        roots = levels[:nd, nodes - 1, :].contiguous()
        OS = (data * L + 15) // 16 * 16
        out = torch.empty((nd, OS), dtype=torch.uint8, device=dev)
        dplen = torch.empty(nd, dtype=torch.int64, device=dev)
        st = torch.empty(nd, dtype=torch.uint8, device=dev)
        work = shards[:nd]

        def dec():
            bc.rbc_decode_batch(N_NODES, L, work, present, roots, out, dplen, st, ctx=ctx, device=True,
                                asynchronous=True)
        dec()
        torch.cuda.synchronize()
        ok = bool((st == 1).all().item()) and bool(torch.equal(out[:, :PAYLOAD], pay[:nd]))
        sample = rbc_oracle_sample(N_NODES, L, work, levels, pay, present, out, sorted({0, nd // 2, nd - 1}))
        ms_dec = timed(dec, reps)
        # Roofline (DESIGN.md §4 "decode"): exactly Q = 2f rows are rebuilt from
        # the first D present rows, so the coding work is Q x D x L/4 MAC-words,
        # the encoder's, and the Merkle rebuild hashes all N rows: the same
        # 109.1 M lane-ops per instance as send_shards.  Algorithmic bytes: read
        # the D present rows, write the Q rebuilt rows, the tree and the payload.
        d_ops = ops + enc_ops
        d_bytes = data * L + parity * L + (2 * N_NODES - 1) * 32 + PAYLOAD
        achieved = d_ops * nd / (ms_dec * 1e-3)
        tr = decode_pmc_traffic(nd)
        return {"GBps": nd * PAYLOAD / (ms_dec * 1e-3) / 1e9, "ms": ms_dec, "instances": nd,
                "erased_per_instance": parity, "roundtrip_ok": ok, "oracle_match": sample["decode_oracle_match"],
                "oracle_sample": sample,
                "roofline": {"bound": "valu", "unit": "Tops/s", "achieved": achieved / 1e12,
                             "peak": VALU_PEAK / 1e12, "frac": achieved / VALU_PEAK,
                             "alg_ops_per_instance": d_ops, "alg_bytes_per_instance": d_bytes,
                             "hbm": {"achieved_GBps": d_bytes * nd / (ms_dec * 1e-3) / 1e9,
                                     "frac": d_bytes * nd / (ms_dec * 1e-3) / HBM_PEAK},
                             "traffic": tr.get("bytes_per_call"), "traffic_unit": "HBM bytes per decode call (PMC)",
                             "traffic_vs_alg_bytes": (tr["bytes_per_call"] / (d_bytes * nd)
                                                      if tr.get("bytes_per_call") else None),
                             "traffic_by_kernel": tr.get("by_kernel"), "traffic_source": tr.get("source"),
                             "traffic_measured_at_head": tr.get("measured_at_head"),
                             "valu_insts_per_wave_pmc": tr.get("valu_insts_per_wave")}}

    decode = run_leg("decode", decode_leg) if not a.no_decode and "decode" in legs else None
    bwire = (run_leg("bwire", lambda: broadcast_wire_leg(ctx, dev, shards, levels, L, min(a.wire_instances, B), reps))
             if a.wire_instances > 0 and "bwire" in legs else None)
    wire = run_leg("wire", lambda: wire_leg(ctx, dev, a.wire_msgs, 256, 2)) if a.wire_msgs > 0 and "wire" in legs \
        else None
    tdec_in = (run_leg("f1", lambda: tdec_inputs_leg(ctx, dev, a.f1_cts, N_NODES, 2))
               if a.f1_cts > 0 and "f1" in legs else None)
    coin = run_leg("coin", lambda: coin_leg(ctx, dev, a.coins, N_NODES, 2)) if a.coins > 0 and "coin" in legs else None

    # the legs added this round run last (the full epoch last of all): a failure there cannot cost the others
    cfg1 = (run_leg("cfg1", lambda: rbc_config_leg(ctx, dev, 16, 1 << 16, a.cfg1_instances, reps,
                                                   "BASELINE.json configs[1]: N=16 f=5, 64 KiB proposals"))
            if a.cfg1_instances > 0 and "cfg1" in legs else None)
    n128 = (run_leg("n128", lambda: rbc_config_leg(ctx, dev, 128, PAYLOAD, a.n128_instances, reps,
                                                   "BASELINE.json configs[4] coding: N=128 f=42, 1 MiB proposals"))
            if a.n128_instances > 0 and "n128" in legs else None)
    tdec = tdec_ep = None
    if a.tdec_cts > 0 and "tdec" in legs:
        r = run_leg("tdec", lambda: tdec_leg(ctx, dev, a.tdec_cts, 2, seed=1 + rank))
        if r is not None:
            tdec, tdec_ep = r
        # every rank joins both reductions, whether or not its leg ran (a rank
        # that skipped a collective would leave the others waiting in it)
        total = shard.sum_over_ranks(tdec["value"] if tdec else 0.0, agg_dev)  # whole-job shares/s
        ranks_ok = int(round(shard.sum_over_ranks(1.0 if tdec else 0.0, agg_dev)))
        if tdec is not None:
            tdec["value"] = total if ranks_ok == world else None
            if ranks_ok != world:
                run_leg.errors["tdec_ranks"] = f"TDec leg failed on {world - ranks_ok} of {world} ranks"

    epoch = (run_leg("epoch", lambda: epoch_leg(ctx, dev, a.epoch_nodes, a.epoch_contrib, max(2, min(a.steps, 5)),
                                                agg_dev))
             if a.epoch_nodes > 0 and a.epoch_nodes % world == 0 and "epoch" in legs else None)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        if "rbc" in legs:
            cpu = cpu_baseline(a.cpu_sample)
        if tdec is not None:
            tdec["cpu_baseline"] = run_leg("tdec_cpu_baseline", lambda: cpu_baseline_tdec(tdec_ep))

    if rank == 0:
        line = {
            "metric": BASE["metric"], "value": value, "unit": "GB/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "checks": checks(decode, tdec, cfg1, n128, epoch, bwire, coin, wire),
            "dtype": "u8", "data": "synthetic (device SplitMix64, seed 0x48424247)",
            "config": {"workload": "rbc_encode_merkle: send_shards N=64 f=21 (RS 22+42) 1 MiB payloads",
                       "n_nodes": N_NODES, "f": (N_NODES - 1) // 3, "payload_bytes": PAYLOAD, "shard_len": L,
                       "instances_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"instances sharded over {world} GPU(s), no data-path collective"},
            "roofline": roofline, "kernels": kernels, "decode": decode, "cpu_baseline": cpu,
            "shard_bytes_GBps": value * N_NODES * L / PAYLOAD,
            "tdec": tdec,
            "config1_n16": cfg1,
            "n128_encode_merkle": n128,
            "network_epoch": epoch,
            "broadcast_wire": bwire,
            "wire_signatures": wire,
            "tdec_inputs": tdec_in,
            "coin": coin,
            "leg_errors": run_leg.errors or None,
            "distributed": dist_info(dist),
        }
        line["checks_final"] = checks_final(line)  # last key: survives a driver that keeps the line's tail
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        torch.distributed.destroy_process_group()
    if rank == 0:
        sys.exit(exit_status(line))


def checks_final(line: dict) -> dict:
    """The compact verdicts repeated as the line's LAST key: every check
    that ran (None = the leg did not run), the failed legs' names, all_ok."""
    c = {k: v for k, v in line["checks"].items() if v is not None and k != "all_ok"}
    c["leg_errors"] = sorted(line.get("leg_errors") or {})
    c["all_ok"] = all(bool(v) for k, v in c.items() if k != "leg_errors") and not c["leg_errors"]
    return c


def exit_status(line: dict) -> int:
    """0 only when every check that ran is true and no leg failed: a wrong
    result or a crashed leg makes the run fail loudly (the line is still
    printed first)."""
    return 0 if line["checks_final"]["all_ok"] else 1


if __name__ == "__main__":
    main()
