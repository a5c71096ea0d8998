"""One HoneyBadger epoch of an N-node network, batched per rank and spanning a
process group (SURVEY.md §8 f4 + a18; BASELINE.json configs[4]).

N nodes are split evenly over the ranks (one process per GPU); rank r hosts
nodes [r*m, (r+1)*m), m = N / world.  Every node proposes one contribution,
so the epoch runs N Broadcast instances and N ThresholdDecrypt instances
(hbbft HoneyBadger / Subset / Broadcast / ThresholdDecrypt, [EXT]; hydrabadger
reaches them through ``dhb.propose`` / ``dhb.handle_message`` at
/root/reference/src/hydrabadger/state.rs:484 and :486-487 and forwards every
step message to its peers at handler.rs:747-764).  Per epoch:

1. propose: each local contribution is threshold-encrypted under the master
   key (``hbg_tdec_encrypt``) and serialised as U48 | u64 len | V | W96 (the
   tuple layout; parity unpinned);
2. Value: ``send_shards`` of the m local proposals (``hbg_rbc_encode_merkle``)
   and the N*m ``Message::Value(proof_j)`` messages in hbbft's bincode wire
   format (``hbg_rbc_write_proof_msgs``) — one all-gather of the message
   bytes (RCCL over xGMI); every rank parses them (``hbg_rbc_read_msgs``) and
   checks them (``hbg_merkle_validate``): node j accepts p's Value iff it
   parses, is a Value, carries index j and validates;
3. Echo: each local node j sends ``Echo(proof)`` (the Value bytes, variant 1)
   for every accepted Value — one all-gather; every Echo is parsed and
   validated once per rank (all local nodes receive the same echoes) and
   counted iff it carries the sender's index and validates; echoes are
   counted per root hash;
4. Ready: a node sends ``Ready(root)`` (bincode, 36 B) once a root has N - f
   echoes — one all-gather, parsed and counted; an instance is delivered with
   2f + 1 Readys and N - 2f echoes for its root (all correct nodes see the
   same messages, so Ready amplification adds nothing and is not modelled);
5. decode: ``decode_from_shards`` of every delivered instance from the echoes
   carrying its root (``hbg_rbc_decode``);
6. Subset accepts every delivered proposal (binary agreement is out of scope)
   whose bytes parse as a ciphertext;
7. ThresholdDecrypt: each local node's decryption share of every accepted
   ciphertext (``hbg_tdec_decrypt_shares``) — one all-gather — then
   ``hbg_tdec_threshold_decrypt`` with a seeded arrival order per ciphertext:
   set_ciphertext check, faults for invalid shares, the first t+1 valid
   shares (t = f), late shares ignored.

Every rank ends with the same epoch result.  The work is in an ``engine``:
``network.DeviceEngine`` (libhbgpu.so on this rank's GPU) is the product;
tests also drive this orchestration with an oracle-backed engine under gloo
to rehearse the exchange without a GPU, and check both against
oracle/epoch.py, a node-by-node restatement.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from . import broadcast as bc
from . import tdec_workload as tw
from .network import all_gather_rows, proof_index_map
from .workload import SplitMix64

TAG_CONTRIB, TAG_R, TAG_ARRIVAL = 6, 7, 8
CT_HEAD, CT_TAIL = 48 + 8, 96


def ct_bytes(contrib_len: int) -> int:
    """Serialised ciphertext of a contrib_len-byte contribution."""
    return CT_HEAD + contrib_len + CT_TAIL


def instance_id(epoch: int, p: int) -> int:
    return (epoch << 20) | p


def arrival_orders(epoch: int, proposers, n: int) -> np.ndarray:
    """[k][n] senders of instance proposers[k]'s decryption shares in arrival
    order (a seeded permutation: the network's timing, an input)."""
    out = np.zeros((len(proposers), n), np.int64)
    for k, p in enumerate(proposers):
        rng = SplitMix64(TAG_ARRIVAL, instance_id(epoch, int(p)))
        keys = [rng.next() for _ in range(n)]
        out[k] = sorted(range(n), key=lambda s: (keys[s], s))
    return out


@dataclass(frozen=True)
class Faults:
    """Misbehaviour injected into an epoch (tests; the same set oracle/epoch.py takes)."""
    silent: frozenset = frozenset()      # nodes that send nothing
    bad_value: frozenset = frozenset()   # (p, j): p's Value to j carries a flipped shard byte
    bad_echo: frozenset = frozenset()    # nodes whose Echoes carry a flipped value byte
    bad_ct: frozenset = frozenset()      # proposers whose ciphertext V is flipped after encryption
    bad_share: frozenset = frozenset()   # nodes that send a share made with another node's key


@dataclass
class EpochResult:
    value_ok: torch.Tensor       # [N p][N j] node j accepted p's Value
    echo_ok: torch.Tensor        # [N s][N p] s's Echo for instance p counted
    echo_count: torch.Tensor     # [N p] echoes carrying the instance's root
    ready_count: torch.Tensor    # [N p]
    delivered: torch.Tensor      # [N p] Broadcast output
    payloads: torch.Tensor       # [N p][C] decoded proposal bytes (rows of delivered instances)
    payload_ok: torch.Tensor     # [N p] delivered, decoded and parsed as a ciphertext
    accepted: list               # proposers of the accepted ciphertexts, ascending
    ct_status: torch.Tensor      # [k] 0 or HBG_E_INVALID_CIPHERTEXT / HBG_E_NOT_ENOUGH_SHARES
    plaintexts: torch.Tensor     # [k][P] (rows with status 0)
    share_outcome: torch.Tensor  # [k][N] HBG_SHARE_*
    times_ms: dict
    exchange_bytes: int          # bytes this rank received in the epoch's all-gathers


class HoneyBadgerEpoch:
    def __init__(self, n_nodes: int, contrib_len: int, engine, seed: int = 1, group=None):
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        if n_nodes % world:
            raise ValueError(f"N={n_nodes} nodes must split evenly over {world} ranks")
        self.N, self.P, self.engine, self.group = n_nodes, contrib_len, engine, group
        self.world, self.rank, self.m = world, rank, n_nodes // world
        self.f = bc.num_faulty(n_nodes)
        self.t = self.f
        self.C = ct_bytes(contrib_len)
        self.L = _lib.shard_len(n_nodes, self.C)
        _, nd = proof_index_map(n_nodes)
        self.msg_len = np.array([4 + 8 + self.L + 8 + 8 + 32 * int(k) + 32 for k in nd], np.int64)
        # key set of degree t (SyncKeyGen's output, out of scope: seeded scalars)
        coeffs, sks = tw.keyset(n_nodes, self.t, seed)
        sk32 = np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in [coeffs[0]] + sks), np.uint8)
        sk32 = torch.from_numpy(sk32.copy().reshape(n_nodes + 1, 32)).to(engine.device)
        pts = engine.key_points(sk32)
        self.master_pk48, self.pk48 = pts[0].contiguous(), pts[1:].contiguous()
        self.sk32 = sk32[1:].contiguous()
        self.sk32_local = self.sk32[rank * self.m:(rank + 1) * self.m].contiguous()

    def local_nodes(self) -> range:
        return range(self.rank * self.m, (self.rank + 1) * self.m)

    def _gather(self, t: torch.Tensor) -> torch.Tensor:
        g = all_gather_rows(t, self.world, self.group)
        self._recv += (self.world - 1) * t.numel() * t.element_size()
        return g

    def _proposals(self, epoch: int, faults: Faults):
        """[m][pad16(C)] serialised ciphertexts of the local contributions."""
        e, m, P, C = self.engine, self.m, self.P, self.C
        first = instance_id(epoch, self.rank * m)
        msgs = e.synth(TAG_CONTRIB, first, m, P).contiguous()
        r32 = e.synth(TAG_R, first, m, 32).clone()
        r32[:, 31] &= 0x3F                                    # < 2^254 < r
        U, V, W = e.encrypt(self.master_pk48, msgs, r32)
        for p in faults.bad_ct:
            if p in self.local_nodes():
                V[p - self.rank * m, 0] ^= 1
        ser = e.zeros((m, (C + 15) // 16 * 16))
        ser[:, :48] = U
        ser[:, 48:56] = torch.tensor(list(P.to_bytes(8, "little")), dtype=torch.uint8, device=ser.device)
        ser[:, CT_HEAD:CT_HEAD + P] = V
        ser[:, CT_HEAD + P:C] = W
        return ser, msgs

    def run(self, epoch: int = 0, faults: Faults = Faults()) -> EpochResult:
        e, N, m, L, C, P, f = self.engine, self.N, self.m, self.L, self.C, self.P, self.f
        dev = e.device
        r0 = self.rank * m
        local = self.local_nodes()
        self._recv = 0
        times = {}
        t0 = time.perf_counter()
        # ---- 1. propose
        ser, _ = self._proposals(epoch, faults)
        # ---- 2. Value messages, recipient-major within the rank: (j, local p)
        shards, levels = e.encode_merkle(N, ser, C)
        for (p, j) in faults.bad_value:
            if p in local:
                shards[p - r0, j, 0] ^= 0xFF
        inst = torch.arange(m, dtype=torch.int64, device=dev).repeat(N)
        index = torch.arange(N, dtype=torch.int32, device=dev).repeat_interleave(m)
        v_len = np.repeat(self.msg_len, m)                    # message (j, p) has msg_len[j] bytes
        v_off = np.zeros(N * m + 1, np.int64)
        v_off[1:] = np.cumsum(v_len)
        vbuf = e.write_proof_msgs(N, L, shards, levels, _lib.HBG_MSG_VALUE, inst, index, v_off)
        vsent = torch.ones((N, m), dtype=torch.uint8, device=dev)
        for p in faults.silent:
            if p in local:
                vsent[:, p - r0] = 0
        e.sync()
        t1 = time.perf_counter()
        times["propose_encode"] = (t1 - t0) * 1e3
        vall = self._gather(vbuf)                             # [rank][j][p_local] messages
        vsent_all = self._gather(vsent.view(1, N, m)).view(self.world, N, m)
        B = int(v_off[-1])
        g_off = (np.arange(self.world, dtype=np.int64)[:, None] * B + v_off[None, :-1]).reshape(-1)
        g_off = np.append(g_off, self.world * B)
        tag, vals, idx, dig, nd, roots, st = e.read_msgs(N, L, vall, g_off)
        vok = e.validate_table(N, L, vals, idx, dig, nd, roots)
        j_of = torch.arange(N, dtype=torch.int32, device=dev).repeat_interleave(m).repeat(self.world)
        good = ((st == 0) & (tag == _lib.HBG_MSG_VALUE) & (idx == j_of) & (vok == 1)).view(self.world, N, m)
        good = good & (vsent_all == 1)
        value_ok = good.permute(0, 2, 1).reshape(N, N)      # [p][j]
        e.sync()
        t2 = time.perf_counter()
        times["value"] = (t2 - t1) * 1e3
        # ---- 3. Echo: node j's Echo of p's proof = the Value bytes with variant 1
        runs = []
        for j in local:
            lo, hi = m * int(self.msg_len[:j].sum()), m * int(self.msg_len[:j + 1].sum())
            for r in range(self.world):
                runs.append(vall[r * B + lo:r * B + hi])
        ebuf = torch.cat(runs).clone()                        # [j local][p] messages of msg_len[j]
        e_len = np.repeat(self.msg_len[r0:r0 + m], N)
        e_off = np.zeros(m * N + 1, np.int64)
        e_off[1:] = np.cumsum(e_len)
        starts = torch.from_numpy(e_off[:-1]).to(dev)
        ebuf[starts] = _lib.HBG_MSG_ECHO                      # u32 LE variant: byte 0 (Value = 0)
        for j in faults.bad_echo:
            if j in local:
                q = torch.from_numpy(e_off[(j - r0) * N:(j - r0 + 1) * N] + 12).to(dev)
                ebuf[q] ^= 0xFF                               # first value byte
        esent = value_ok[:, r0:r0 + m].t().contiguous().to(torch.uint8)   # [j local][p]
        for j in faults.silent:
            if j in local:
                esent[j - r0] = 0
        eall = self._gather(ebuf)                             # [s][p] messages of msg_len[s]
        esent_all = self._gather(esent)                       # [N s][N p]
        ge_len = np.repeat(self.msg_len, N)
        ge_off = np.zeros(N * N + 1, np.int64)
        ge_off[1:] = np.cumsum(ge_len)
        tag, vals, idx, dig, nd, roots, st = e.read_msgs(N, L, eall, ge_off)
        eok = e.validate_table(N, L, vals, idx, dig, nd, roots)
        s_of = torch.arange(N, dtype=torch.int32, device=dev).repeat_interleave(N)
        echo_ok = ((st == 0) & (tag == _lib.HBG_MSG_ECHO) & (idx == s_of) & (eok == 1)).view(N, N)
        echo_ok = echo_ok & (esent_all == 1)                  # [s][p]
        # echoes per root: the root with the most valid echoes (ties: lowest sender)
        R = roots.view(N, N, 32).permute(1, 0, 2)             # [p][s][32]
        ok_ps = echo_ok.t()                                   # [p][s]
        same = (R.unsqueeze(2) == R.unsqueeze(1)).all(-1) & ok_ps.unsqueeze(1)   # [p][s][s']
        cnt = torch.where(ok_ps, same.sum(-1), torch.full_like(ok_ps, -1, dtype=torch.int64))
        key = cnt * (N + 1) + (N - torch.arange(N, device=dev))                 # max count, then lowest s
        best = key.argmax(dim=1)                              # [p]
        ar = torch.arange(N, device=dev)
        echo_count = cnt[ar, best].clamp(min=0)
        root_p = R[ar, best]                                  # [p][32]
        holds = same[ar, best] & ok_ps                        # [p][s] valid echoes carrying root_p
        e.sync()
        t3 = time.perf_counter()
        times["echo"] = (t3 - t2) * 1e3
        # ---- 4. Ready
        rbuf = e.zeros((m, N, 36))
        rbuf[:, :, 0] = _lib.HBG_MSG_READY
        rbuf[:, :, 4:] = root_p.unsqueeze(0)
        rsent = (echo_count >= N - f).to(torch.uint8).unsqueeze(0).repeat(m, 1)   # [j local][p]
        for j in faults.silent:
            if j in local:
                rsent[j - r0] = 0
        rall = self._gather(rbuf.view(m * N, 36)).view(-1)
        rsent_all = self._gather(rsent)                       # [N j][N p]
        r_off = np.arange(N * N + 1, dtype=np.int64) * 36
        tag, _, _, _, _, rroots, st = e.read_msgs(N, 16, rall, r_off)   # digests only: no value table needed
        rgood = (st == 0) & (tag == _lib.HBG_MSG_READY)
        rmatch = (rroots.view(N, N, 32) == root_p.unsqueeze(0)).all(-1) & rgood.view(N, N) & (rsent_all == 1)
        ready_count = rmatch.sum(0)                           # [p]
        delivered = (ready_count >= 2 * f + 1) & (echo_count >= N - 2 * f)
        # ---- 5. decode from the echoes carrying the root
        D = N - 2 * f
        S = vals.shape[-1]
        sh = vals.view(N, N, S).permute(1, 0, 2).contiguous()  # [p][s][S]
        present = (holds & delivered.unsqueeze(1)).to(torch.uint8).contiguous()
        out, plen, dst = e.decode(N, L, sh, present, root_p.contiguous())
        out = out[:, :C] if out.shape[1] >= C else torch.nn.functional.pad(out, (0, C - out.shape[1]))
        le = (out[:, 48:56].to(torch.int64) << (8 * torch.arange(8, device=dev))).sum(1)
        payload_ok = delivered & (dst == _lib.HBG_DECODE_OK) & (plen == C) & (le == P)
        e.sync()
        t4 = time.perf_counter()
        times["ready_decode"] = (t4 - t3) * 1e3
        # ---- 6/7. Subset accepts; ThresholdDecrypt of every accepted ciphertext
        acc = torch.nonzero(payload_ok).flatten().tolist()
        k = len(acc)
        if k:
            at = torch.tensor(acc, device=dev)
            U, V, W = out[at, :48].contiguous(), out[at, CT_HEAD:CT_HEAD + P].contiguous(), out[at, CT_HEAD + P:C]
            pc = torch.arange(k, dtype=torch.int32, device=dev).repeat_interleave(m)
            pj = torch.arange(m, dtype=torch.int32, device=dev).repeat(k)
            sk_use = self.sk32_local.clone()
            for j in faults.bad_share:
                if j in local:
                    sk_use[j - r0] = self.sk32[(j + 1) % N]
            shares = e.decrypt_shares(U, sk_use, pc, pj).view(k, m, 48)
            sall = self._gather(shares.permute(1, 0, 2).contiguous())   # [N s][k][48]
            share48 = sall.permute(1, 0, 2).contiguous()                # [k][N][48]
            order = arrival_orders(epoch, acc, N)
            silent = np.array([s in faults.silent for s in range(N)])
            arr = np.full((k, N), -1, np.int32)
            for q in range(k):
                o = order[q][~silent[order[q]]]
                arr[q, :len(o)] = o
            V_off = torch.arange(k + 1, dtype=torch.int64, device=dev) * P
            pt, ct_status, outcome = e.threshold_decrypt(self.t, N, U, V.reshape(-1), V_off, W.contiguous(),
                                                         self.pk48, share48, torch.from_numpy(arr).to(dev))
            plaintexts = pt.view(k, P)
        else:
            ct_status = torch.zeros(0, dtype=torch.int32, device=dev)
            plaintexts = e.zeros((0, P))
            outcome = e.zeros((0, N))
        e.sync()
        t5 = time.perf_counter()
        times["tdec"] = (t5 - t4) * 1e3
        times["epoch"] = (t5 - t0) * 1e3
        return EpochResult(value_ok, echo_ok, echo_count, ready_count, delivered, out, payload_ok, acc,
                           ct_status, plaintexts, outcome, times, self._recv)
