"""One simulated hbbft network spanning several GPUs (BASELINE.json configs[4],
SURVEY.md §8(e)): the reliable-broadcast half of an epoch with one RCCL
all-gather as the only inter-GPU exchange.

N nodes are split evenly over the ranks of a process group (one process per
GPU); rank r hosts nodes [r*m, (r+1)*m), m = N / world.  Every node proposes
one payload, so one epoch runs N Broadcast instances (hbbft Subset, [EXT];
hydrabadger reaches it through ``dhb.propose`` / ``dhb.handle_message`` at
/root/reference/src/hydrabadger/state.rs:484 and :486-487).  Per epoch:

1. ``send_shards`` of the m local proposals (RS(N-2f, 2f) + SHA3 Merkle):
   ``hbg_rbc_encode_merkle`` on this rank's GPU.
2. The Value / Echo exchange: proposer i's shard j (with its proof) goes to
   node j, and node j echoes it to every node, so after the Echo round every
   node holds shard j of every instance from every j.  On the GPUs that is one
   ``all_gather_into_tensor`` of the encoded [m][N][S] shard blocks plus the
   [m][nodes][32] Merkle levels (proofs are index walks over the levels) —
   RCCL over xGMI with backend "nccl".
3. Every echo is checked with ``Proof::validate`` (``hbg_merkle_validate``,
   N*N proofs).  All m local nodes receive the same echoes, so a rank checks
   each echo once on their behalf (the simulation shares, nodes would repeat).
4. ``decode_from_shards`` per instance from the echoes of the first N-f
   senders to arrive (a seeded arrival order per instance, so reconstruct
   really rebuilds f missing rows; decoding needs only N-2f): reconstruct
   + Merkle rebuild + root check + glue (``hbg_rbc_decode``).

The work is in an ``engine`` object: ``DeviceEngine`` (libhbgpu.so on this
rank's GPU) is the product; tests pass a CPU engine built on the oracle to
rehearse the exchange under gloo without a GPU.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, workload
from . import broadcast as bc
from .tdec_workload import G1_GENERATOR


def proof_index_map(n: int) -> tuple[np.ndarray, np.ndarray]:
    """For every leaf j of an n-leaf hbbft tree: the flat-levels node index of
    each sibling digest of ``MerkleTree::proof(j)`` ([n][depth], padded with 0)
    and how many digests the proof carries ([n])."""
    depth = _lib.merkle_depth(n)
    idx = np.zeros((n, max(depth, 1)), np.int64)
    nd = np.zeros(n, np.int32)
    starts, off, cnt = [], 0, n
    while cnt > 1:
        starts.append((off, cnt))
        off += cnt
        cnt = (cnt + 1) // 2
    for j in range(n):
        li, k = j, 0
        for off, cnt in starts:
            if (li ^ 1) < cnt:
                idx[j, k] = off + (li ^ 1)
                k += 1
            li //= 2
        nd[j] = k
    return idx, nd


def all_gather_rows(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """Rank-major concatenation of every rank's equally shaped tensor along
    dim 0: one all_gather_into_tensor (RCCL over xGMI with backend "nccl"; the
    same call under gloo in the CPU rehearsals).  Without a process group the
    tensor is returned as is; a one-rank group still runs the collective (the
    one-GPU box's check of the RCCL branch)."""
    if world == 1 and not dist.is_initialized():
        return t
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def all_to_all_bytes(buf: torch.Tensor, send: list, recv: list, world: int, group=None) -> torch.Tensor:
    """Personalised exchange of a flat byte buffer: rank-major chunks of
    send[r] bytes go to rank r, and recv[r] bytes arrive from rank r (one
    all_to_all_single: RCCL over xGMI with backend "nccl", gloo in the CPU
    rehearsals).  Without a process group the buffer is returned as is."""
    if world == 1 and not dist.is_initialized():
        return buf
    out = torch.empty(int(sum(recv)), dtype=buf.dtype, device=buf.device)
    dist.all_to_all_single(out, buf.contiguous(), output_split_sizes=[int(x) for x in recv],
                           input_split_sizes=[int(x) for x in send], group=group)
    return out


def arrival_mask(instance: int, n: int, epoch: int = 0) -> list:
    """Echo senders whose shard instance `instance` decodes from: the first
    N-f to arrive, in a seeded order (f = (N-1)/3 absent)."""
    f = bc.num_faulty(n)
    return workload.erasure_mask((epoch << 32) ^ (0xEC40 << 16) ^ instance, n, f)


class DeviceEngine:
    """The product engine: libhbgpu.so kernels on this rank's GPU (torch CUDA
    tensors as device buffers).

    Every torch op here (zero fills, gathers, the arrival mask) runs on torch's
    current stream and the engine's kernels read what they produce, so the
    context must enqueue on that same stream: a context created here is bound
    to ``torch.cuda.current_stream(device)``; a context passed in must already
    be bound to the stream the caller runs torch on (bench.py binds its own).
    One stream also makes the caching allocator's reuse of tensors freed while
    an HBG_ASYNC kernel still reads them safe (reuse is ordered on the stream).
    """

    def __init__(self, device: torch.device, ctx: _lib.Context | None = None):
        if device.type != "cuda":
            raise _lib.HbgError(_lib.HBG_E_DEVICE, "DeviceEngine needs a GPU (no CPU fallback)")
        self.device = device
        if ctx is None:
            ctx = _lib.Context(device.index if device.index is not None else 0)
            ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
        self.ctx = ctx

    def zeros(self, shape, dtype=torch.uint8):
        return torch.zeros(shape, dtype=dtype, device=self.device)

    def synth_payloads(self, first: int, m: int, P: int):
        pay = self.zeros((m, (P + 15) // 16 * 16))
        bc.synth_bytes(workload.TAG_PAYLOAD, first, P, pay, ctx=self.ctx, device=True)
        return pay

    def encode_merkle(self, n_nodes: int, pay, P: int):
        m = pay.shape[0]
        L = _lib.shard_len(n_nodes, P)
        S = (L + 15) // 16 * 16
        plen = torch.full((m,), P, dtype=torch.int64, device=self.device)
        shards = self.zeros((m, n_nodes, S))
        levels = self.zeros((m, _lib.merkle_nodes(n_nodes), 32))
        bc.rbc_encode_merkle_batch(n_nodes, pay, plen, L, shards, levels, ctx=self.ctx, device=True,
                                   asynchronous=True)
        return shards, levels

    def validate(self, n_nodes: int, L: int, shards, levels, sib, nd):
        """Proof::validate of every (instance, sender) echo: [N][N] ok bits."""
        n_inst = shards.shape[0]
        idx = torch.from_numpy(sib).to(self.device)
        dig = levels[:, idx].contiguous()                     # [I][N][depth][32]
        index = torch.arange(n_nodes, dtype=torch.int32, device=self.device).repeat(n_inst)
        ndig = torch.from_numpy(nd).to(self.device).repeat(n_inst)
        nodes = levels.shape[1]
        roots = levels[:, nodes - 1:nodes, :].expand(n_inst, n_nodes, 32).contiguous()
        ok = self.zeros((n_inst * n_nodes,))
        S = shards.shape[-1]
        flags = _lib.HBG_DEVICE | _lib.HBG_ASYNC
        _lib.check(_lib.lib().hbg_merkle_validate(self.ctx.h, n_nodes, L, shards.data_ptr(), S, index.data_ptr(),
                                                  dig.data_ptr(), ndig.data_ptr(), roots.data_ptr(), ok.data_ptr(),
                                                  n_inst * n_nodes, flags), "Proof::validate")
        return ok.view(n_inst, n_nodes)

    def decode(self, n_nodes: int, L: int, shards, present, roots, out=None):
        """out: optional [n_inst][OS] zeroed rows to decode into (a slice of a
        larger table: no concatenation copy afterwards)."""
        n_inst = shards.shape[0]
        D, _ = bc.shard_counts(n_nodes)
        OS = (D * L + 15) // 16 * 16
        if out is None:
            out = self.zeros((n_inst, OS))
        assert out.shape == (n_inst, OS) and out.is_contiguous()
        plen = torch.zeros(n_inst, dtype=torch.int64, device=self.device)
        st = self.zeros((n_inst,))
        bc.rbc_decode_batch(n_nodes, L, shards, present, roots, out, plen, st, ctx=self.ctx, device=True,
                            asynchronous=True)
        return out, plen, st

    # ---- the HoneyBadger epoch's primitives (hydrabadger_amd/epoch.py) ----
    def _flags(self):
        return _lib.HBG_DEVICE | _lib.HBG_ASYNC

    def synth(self, tag: int, first: int, m: int, nbytes: int):
        out = self.zeros((m, max(nbytes, 1)))
        bc.synth_bytes(tag, first, nbytes, out, ctx=self.ctx, device=True)
        return out[:, :nbytes]

    def key_points(self, sk32):
        """[s] G1 for each 32-byte scalar (public keys / key shares):
        decrypt_share_no_verify with U = the G1 generator."""
        k = sk32.shape[0]
        g1 = torch.from_numpy(np.frombuffer(G1_GENERATOR, np.uint8).copy()).to(self.device)
        i32 = dict(dtype=torch.int32, device=self.device)
        return self.decrypt_shares(g1.view(1, 48), sk32, torch.zeros(k, **i32), torch.arange(k, **i32))

    def encrypt(self, pk48, msgs, r32):
        m, P = msgs.shape
        off = torch.arange(m + 1, dtype=torch.int64, device=self.device) * P
        U, W = self.zeros((m, 48)), self.zeros((m, 96))
        V = self.zeros((max(m * P, 1),))
        _lib.check(_lib.lib().hbg_tdec_encrypt(self.ctx.h, pk48.contiguous().data_ptr(), m, r32.contiguous().data_ptr(),
                                               msgs.contiguous().data_ptr(), off.data_ptr(), U.data_ptr(), V.data_ptr(),
                                               W.data_ptr(), self._flags()), "encrypt_with_rng")
        return U, V[:m * P].view(m, P), W

    def write_proof_msgs(self, n_nodes: int, L: int, shards, levels, tag: int, inst, index, off):
        out = self.zeros((max(int(off[-1]), 1),))
        bc.write_proof_msgs_batch(n_nodes, L, shards, levels, tag, inst, index, out,
                                  torch.from_numpy(off).to(self.device), ctx=self.ctx, device=True, asynchronous=True)
        return out[:int(off[-1])]

    def read_msgs(self, n_nodes: int, L: int, buf, off):
        M = off.shape[0] - 1
        S = (max(L, 1) + 15) // 16 * 16
        depth = max(_lib.merkle_depth(n_nodes), 1)
        i32 = dict(dtype=torch.int32, device=self.device)
        tag, index, nd, st = (torch.zeros(M, **i32) for _ in range(4))
        vals, dig, roots = self.zeros((M, S)), self.zeros((M, depth, 32)), self.zeros((M, 32))
        bc.read_msgs_batch(n_nodes, L, buf, torch.from_numpy(off).to(self.device), tag, vals, index, dig, nd, roots,
                           st, ctx=self.ctx, device=True, asynchronous=True)
        return tag, vals, index, dig, nd, roots, st

    def validate_table(self, n_nodes: int, L: int, vals, index, dig, nd, roots, views: int = 1):
        """Proof::validate of every row; with views > 1 each of `views` nodes
        validates the whole table itself (ok [views * rows], view-major)."""
        M = vals.shape[0]
        ok = self.zeros((M * views,))
        _lib.check(_lib.lib().hbg_merkle_validate_views(self.ctx.h, n_nodes, L, vals.data_ptr(), vals.shape[-1],
                                                        index.data_ptr(), dig.data_ptr(), nd.data_ptr(),
                                                        roots.data_ptr(), ok.data_ptr(), M, views, self._flags()),
                   "Proof::validate")
        return ok

    def decrypt_shares(self, U48, sk32, pair_ct, pair_sk):
        n = pair_ct.shape[0]
        out = self.zeros((max(n, 1), 48))
        st = torch.zeros(max(n, 1), dtype=torch.int32, device=self.device)
        _lib.check(_lib.lib().hbg_tdec_decrypt_shares(self.ctx.h, U48.shape[0], U48.contiguous().data_ptr(),
                                                      sk32.shape[0], sk32.contiguous().data_ptr(), n,
                                                      pair_ct.data_ptr(), pair_sk.data_ptr(), out.data_ptr(),
                                                      st.data_ptr(), self._flags()), "decrypt_share_no_verify")
        return out[:n]

    def threshold_decrypt(self, t: int, n_nodes: int, U, V, V_off, W, pk48, share48, arrival):
        n_ct = U.shape[0]
        pt = self.zeros((max(int(V.numel()), 1),))
        st = torch.zeros(n_ct, dtype=torch.int32, device=self.device)
        oc = self.zeros((n_ct, n_nodes))
        from . import threshold as th
        th.threshold_decrypt_arrays(t, n_nodes, U.contiguous(), V.contiguous(), V_off, W.contiguous(),
                                    pk48.contiguous(), share48.contiguous(), arrival, pt, st, oc, ctx=self.ctx,
                                    device=True, asynchronous=True)
        return pt[:V.numel()], st, oc

    def sync(self):
        torch.cuda.synchronize(self.device)


@dataclass
class EpochResult:
    payloads: torch.Tensor      # [N][OS] decoded proposals (this rank's view of the epoch's batch)
    lengths: torch.Tensor       # [N]
    status: torch.Tensor        # [N] HBG_DECODE_OK / NONE
    echo_ok: torch.Tensor       # [N][N] Proof::validate of every echo
    times_ms: dict
    exchange_bytes: int         # bytes this rank received in the all-gather


class SpanningEpoch:
    """RBC half of one epoch of an N-node network spread over a process group."""

    def __init__(self, n_nodes: int, payload_len: int, engine, group=None):
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        if n_nodes % world:
            raise ValueError(f"N={n_nodes} nodes must split evenly over {world} ranks")
        self.N, self.P, self.engine, self.group = n_nodes, payload_len, engine, group
        self.world, self.rank, self.m = world, rank, n_nodes // world
        self.L = _lib.shard_len(n_nodes, payload_len)
        self.sib, self.nd = proof_index_map(n_nodes)

    def local_nodes(self) -> range:
        return range(self.rank * self.m, (self.rank + 1) * self.m)

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return all_gather_rows(t, self.world, self.group)

    def run(self, payloads, epoch: int = 0) -> EpochResult:
        """payloads: [m][PS] u8 — this rank's nodes' proposals (engine tensors)."""
        e, N, L = self.engine, self.N, self.L
        t = {}
        t0 = time.perf_counter()
        shards, levels = e.encode_merkle(N, payloads, self.P)
        e.sync()
        t1 = time.perf_counter()
        t["encode_merkle"] = (t1 - t0) * 1e3
        all_shards = self._all_gather(shards)       # [N][N][S]: every instance's Value/Echo shards
        all_levels = self._all_gather(levels)       # [N][nodes][32]: proofs + roots
        e.sync()
        t2 = time.perf_counter()
        t["all_gather"] = (t2 - t1) * 1e3
        ok = e.validate(N, L, all_shards, all_levels, self.sib, self.nd)
        e.sync()
        t3 = time.perf_counter()
        t["validate"] = (t3 - t2) * 1e3
        arrived = torch.tensor([arrival_mask(i, N, epoch) for i in range(N)], dtype=torch.uint8,
                               device=all_shards.device)
        present = (arrived & ok).to(torch.uint8)     # an echo counts only if its proof validates
        nodes = all_levels.shape[1]
        roots = all_levels[:, nodes - 1, :].contiguous()
        out, plen, st = e.decode(N, L, all_shards, present, roots)
        e.sync()
        t["decode"] = (time.perf_counter() - t3) * 1e3
        t["epoch"] = (time.perf_counter() - t0) * 1e3
        recv = (self.world - 1) * (shards.numel() + levels.numel())
        return EpochResult(out, plen, st, ok, t, recv)
