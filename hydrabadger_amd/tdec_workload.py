"""Device-generated ThresholdDecrypt epochs (SURVEY.md §8(d) cfg 4, BASELINE.json configs[3]).

One epoch of an N-node network as one node's ThresholdDecrypt sees it: a
seeded degree-t key set (SyncKeyGen's output, out of scope, so its scalars
are drawn here), n_ct DISTINCT ciphertexts of msg_len-byte contributions
(PublicKey::encrypt_with_rng on the device), every node's decryption share of
every ciphertext (SecretKeyShare::decrypt_share_no_verify on the device), and
a seeded fraction of the shares replaced by one of three kinds of bad share:

  0  another node's share of the same ciphertext (claimed under the wrong key),
  1  the same node's share of another ciphertext,
  2  a random valid G1 point.

Only the Fr key scalars (N + 1 of them) are computed on the host; every point
and byte string is produced by libhbgpu kernels, so inputs of 100k
ciphertexts x 64 shares never cross PCIe.  The expected verdicts follow from
construction (a replaced share is invalid; the probability that one verifies
is negligible) and are checked against the engine's outputs by the callers.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from . import broadcast as bc
from .workload import SplitMix64, TAG_TDEC

# BLS12-381 scalar field order and the compressed G1 generator (zcash encoding)
FR_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
G1_GENERATOR = bytes.fromhex(
    "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
BAD_KINDS = ("wrong key", "another ciphertext's share", "random valid point")


def fr_scalar(rng: SplitMix64) -> int:
    v = 0
    for _ in range(4):
        v = (v << 64) | rng.next()
    return v % FR_ORDER


def keyset(n_nodes: int, t: int, seed: int):
    """SecretKeySet of degree t: (coefficients, secret key shares sk_i = p(i+1))."""
    rng = SplitMix64(TAG_TDEC, 0xC0EF ^ seed)
    coeffs = [fr_scalar(rng) for _ in range(t + 1)]
    shares = []
    for i in range(n_nodes):
        acc = 0
        for c in reversed(coeffs):
            acc = (acc * (i + 1) + c) % FR_ORDER
        shares.append(acc)
    return coeffs, shares


def _scalars_le(vals) -> np.ndarray:
    return np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in vals), np.uint8).copy()


@dataclass
class TdecEpoch:
    t: int
    n_nodes: int
    n_ct: int
    msg_len: int
    U: torch.Tensor          # [n_ct][48]
    V: torch.Tensor          # [n_ct * msg_len]
    V_off: torch.Tensor      # [n_ct + 1] int64
    W: torch.Tensor          # [n_ct][96]
    pk48: torch.Tensor       # [N][48] public key shares
    master_pk48: torch.Tensor
    share48: torch.Tensor    # [n_ct][N][48], sender i's share of ct k at [k][i]
    msgs: torch.Tensor       # [n_ct * msg_len] the plaintexts
    bad: np.ndarray          # [n_ct][N] bool: replaced shares
    kind: np.ndarray         # [n_ct][N] int8: kind of replacement (-1: none)


def _decrypt_shares(ctx, dev, U48, sk32, pairs_ct, pairs_sk, n_ct: int, n_sk: int):
    n = pairs_ct.numel()
    out = torch.empty((n, 48), dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().hbg_tdec_decrypt_shares(ctx.h, n_ct, U48.data_ptr(), n_sk, sk32.data_ptr(), n,
                                                  pairs_ct.data_ptr(), pairs_sk.data_ptr(), out.data_ptr(),
                                                  st.data_ptr(), _lib.HBG_DEVICE), "decrypt_share_no_verify")
    return out, st


def make_epoch(ctx: _lib.Context, dev: torch.device, n_ct: int, n_nodes: int = 64, msg_len: int = 256,
               bad_rate: float = 0.01, seed: int = 1) -> TdecEpoch:
    """Builds the epoch on `dev` with the engine (ctx must be bound to torch's
    current stream of `dev`)."""
    t = (n_nodes - 1) // 3
    coeffs, sks = keyset(n_nodes, t, seed)
    i32 = dict(dtype=torch.int32, device=dev)
    # public key shares and the master key: [s] G1 through decrypt_share_no_verify with U = G1
    g1 = torch.from_numpy(np.frombuffer(G1_GENERATOR, np.uint8).copy()).to(dev)
    sk_all = torch.from_numpy(_scalars_le([coeffs[0]] + sks)).to(dev)
    pts, st = _decrypt_shares(ctx, dev, g1, sk_all, torch.zeros(n_nodes + 1, **i32),
                              torch.arange(n_nodes + 1, **i32), 1, n_nodes + 1)
    if not bool((st == 0).all()):
        raise _lib.HbgError(_lib.HBG_E_INVALID_POINT, "key shares")
    master_pk48, pk48 = pts[0].contiguous(), pts[1:].contiguous()
    # contributions and encryption randomness (device SplitMix64 streams)
    msgs = torch.empty((n_ct, msg_len), dtype=torch.uint8, device=dev)
    bc.synth_bytes(TAG_TDEC, seed << 24, msg_len, msgs, ctx=ctx, device=True)
    r32 = torch.empty((n_ct, 32), dtype=torch.uint8, device=dev)
    bc.synth_bytes(TAG_TDEC ^ 0x10, seed << 24, 32, r32, ctx=ctx, device=True)
    r32[:, 31] &= 0x3F                                   # < 2^254 < r
    V_off = torch.arange(n_ct + 1, dtype=torch.int64, device=dev) * msg_len
    U = torch.empty((n_ct, 48), dtype=torch.uint8, device=dev)
    V = torch.empty(n_ct * msg_len, dtype=torch.uint8, device=dev)
    W = torch.empty((n_ct, 96), dtype=torch.uint8, device=dev)
    msgs = msgs.reshape(-1)
    _lib.check(_lib.lib().hbg_tdec_encrypt(ctx.h, master_pk48.data_ptr(), n_ct, r32.data_ptr(), msgs.data_ptr(),
                                           V_off.data_ptr(), U.data_ptr(), V.data_ptr(), W.data_ptr(),
                                           _lib.HBG_DEVICE), "encrypt_with_rng")
    # every node's share of every ciphertext
    sk_dev = torch.from_numpy(_scalars_le(sks)).to(dev)
    n = n_ct * n_nodes
    pc = torch.arange(n_ct, **i32).repeat_interleave(n_nodes)
    ps = torch.arange(n_nodes, **i32).repeat(n_ct)
    share, st = _decrypt_shares(ctx, dev, U, sk_dev, pc, ps, n_ct, n_nodes)
    if not bool((st == 0).all()):
        raise _lib.HbgError(_lib.HBG_E_INVALID_POINT, "decryption shares")
    share = share.view(n_ct, n_nodes, 48)
    # seeded corruption, three kinds
    rng = np.random.default_rng(0x48424247 ^ seed)
    bad = rng.random((n_ct, n_nodes)) < bad_rate
    kind = np.where(bad, rng.integers(0, 3, size=(n_ct, n_nodes)), -1).astype(np.int8)
    orig = share.clone()
    for kd in (0, 1):
        kk, ii = np.nonzero(kind == kd)
        if len(kk) == 0:
            continue
        k_t = torch.from_numpy(kk).to(dev)
        i_t = torch.from_numpy(ii).to(dev)
        if kd == 0:
            share[k_t, i_t] = orig[k_t, (i_t + 1) % n_nodes]
        else:
            share[k_t, i_t] = orig[(k_t + 1) % n_ct, i_t]
    kk, ii = np.nonzero(kind == 2)
    if len(kk):
        rnd = [fr_scalar(SplitMix64(TAG_TDEC, 0xBAD0000 + q)) for q in range(len(kk))]
        pts, st = _decrypt_shares(ctx, dev, g1, torch.from_numpy(_scalars_le(rnd)).to(dev),
                                  torch.zeros(len(kk), **i32), torch.arange(len(kk), **i32), 1, len(kk))
        share[torch.from_numpy(kk).to(dev), torch.from_numpy(ii).to(dev)] = pts
    del orig
    return TdecEpoch(t, n_nodes, n_ct, msg_len, U, V, V_off, W, pk48, master_pk48, share.contiguous(), msgs, bad,
                     kind)


def expected_outcomes(bad: np.ndarray, t: int) -> np.ndarray:
    """ThresholdDecrypt's per-(ct, sender) outcome for arrivals in node order:
    the first t+1 valid shares are accepted, invalid ones before that point
    are faults, everything after it is ignored (hbbft try_output /
    terminated); assumes every row has t+1 valid shares."""
    valid = ~bad
    pos = np.cumsum(valid, axis=1)                       # valid shares among the first j+1
    term = np.argmax(pos >= t + 1, axis=1)               # index of the (t+1)-th valid share
    j = np.arange(bad.shape[1])[None, :]
    before = j <= term[:, None]
    out = np.full(bad.shape, _lib.HBG_SHARE_IGNORED, np.uint8)
    out[before & valid] = _lib.HBG_SHARE_ACCEPTED
    out[before & ~valid] = _lib.HBG_SHARE_FAULTY
    return out
