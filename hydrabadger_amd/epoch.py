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
   With ``per_node`` (the default) the Values travel by one all-to-all: a
   rank receives only the messages addressed to its own nodes, and node j
   validates its N Values (hbbft rejects a Value for another index before
   hashing it), N*m per rank instead of N*N;
3. Echo: each local node j sends ``Echo(proof)`` (the Value bytes, variant 1)
   for every accepted Value — one all-gather; every Echo is parsed once per
   rank and validated by EVERY local node (``per_node``: m*N*N
   ``Proof::validate`` per rank, the N^3 of the network spread over the
   ranks; the shared view validates each echo once on behalf of all local
   nodes) and counted iff it carries the sender's index and validates;
   echoes are counted per root hash;
4. Ready: a node sends ``Ready(root)`` (bincode, 36 B) once a root has N - f
   echoes — one all-gather, parsed and counted; an instance is delivered with
   2f + 1 Readys and N - 2f echoes for its root (all correct nodes see the
   same messages, so Ready amplification adds nothing and is not modelled);
5. decode: ``decode_from_shards`` of every delivered instance from the echoes
   carrying its root (``hbg_rbc_decode``) — by every local node (``per_node``:
   each reconstructs its own copy, m*N decodes per rank, in chunks of nodes);
6. Subset accepts every delivered proposal (binary agreement is out of scope)
   whose bytes parse as a ciphertext;
7. ThresholdDecrypt: each local node's decryption share of every accepted
   ciphertext (``hbg_tdec_decrypt_shares``) — one all-gather — then
   ``hbg_tdec_threshold_decrypt``: with ``per_node`` every local node runs
   its own instance of every accepted ciphertext with its own seeded arrival
   order (m*k instances per rank: set_ciphertext / Ciphertext::verify and
   the verification of every share it handles, at every node, as hbbft
   does); the shared view runs one instance per ciphertext for all nodes.
   Either way: faults for invalid shares, the first t+1 valid shares
   (t = f), late shares ignored.

The RBC outcomes are the same at every node under full delivery; the TDec
results come per view (``views``: this rank's node ids, or [-1] for the
shared view).  The work is in an ``engine``:
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
from .network import all_gather_rows, all_to_all_bytes, proof_index_map
from .workload import BASE_SEED, GAMMA, SplitMix64

TAG_CONTRIB, TAG_R, TAG_ARRIVAL = 6, 7, 8
CT_HEAD, CT_TAIL = 48 + 8, 96


def ct_bytes(contrib_len: int) -> int:
    """Serialised ciphertext of a contrib_len-byte contribution."""
    return CT_HEAD + contrib_len + CT_TAIL


def instance_id(epoch: int, p: int) -> int:
    # bits [0, 20) proposer, [20, 40) epoch; arrival_id puts node + 1 in [40, 48)
    # and the stream tag sits at bit 48, so every field must stay in its range
    if not (0 <= p < 1 << 20 and 0 <= epoch < 1 << 20):
        raise ValueError(f"instance id fields out of range: epoch {epoch}, proposer {p}")
    return (epoch << 20) | p


def arrival_id(epoch: int, p: int, node: int = -1) -> int:
    """Seed id of an arrival order: instance p's shared view (node -1) or node `node`'s."""
    if node >= 255:
        raise ValueError(f"node {node} does not fit the arrival id's 8-bit node field")
    return instance_id(epoch, p) | (0 if node < 0 else (node + 1) << 40)


def _copies(x: torch.Tensor, c: int) -> torch.Tensor:
    """c stacked copies of x along dim 0 (every view's own copy of a table).
    Byte tables whose rows are a multiple of 8 bytes are copied as int64
    (torch copies uint8 element by element: 6.7 ms per 12.5 GB chunk of echo
    tables at N = 128, the word copy runs near the HBM rate)."""
    if c == 1:
        return x
    reps = (c,) + (1,) * (x.dim() - 1)
    if x.dtype == torch.uint8 and x.dim() >= 1 and x.shape[-1] % 8 == 0 and x.is_contiguous():
        return x.view(torch.int64).repeat(*reps).view(torch.uint8)
    return x.repeat(*reps)


class _CopyPipe:
    """Every decode chunk's views get their own copy of the shard table (the
    decoder reconstructs in place).  On a GPU the copies of chunk i + 1 are
    made on a side stream while chunk i decodes (two buffers: chunk i + 2's
    copy waits for chunk i's decode); elsewhere they are made on demand."""

    def __init__(self, x: torch.Tensor, chunks, dev):
        self.x, self.chunks = x, chunks
        self.gpu = dev.type == "cuda" and len(chunks) > 1
        if not self.gpu:
            return
        self.main = torch.cuda.current_stream(dev)
        self.side = torch.cuda.Stream(dev)
        cmax = max(c for _, c in chunks)
        self.bufs = [torch.empty((cmax,) + tuple(x.shape), dtype=x.dtype, device=dev) for _ in range(2)]
        self.copied, self.decoded = {}, {}
        self.side.wait_stream(self.main)   # x is written on the main stream
        self._copy(0)

    def _copy(self, i: int):
        c = self.chunks[i][1]
        with torch.cuda.stream(self.side):
            if i >= 2:
                self.side.wait_event(self.decoded[i - 2])
            dst = self.bufs[i % 2][:c]
            src = self.x.unsqueeze(0).expand((c,) + tuple(self.x.shape))
            if self.x.dtype == torch.uint8 and self.x.shape[-1] % 8 == 0 and self.x.is_contiguous():
                dst, src = dst.view(torch.int64), self.x.view(torch.int64).unsqueeze(0).expand((c,) + tuple(
                    self.x.view(torch.int64).shape))
            dst.copy_(src)
            ev = torch.cuda.Event()
            ev.record(self.side)
            self.copied[i] = ev

    def get(self, i: int) -> torch.Tensor:
        c = self.chunks[i][1]
        if not self.gpu:
            return _copies(self.x, c)
        if i + 1 < len(self.chunks):
            self._copy(i + 1)
        self.main.wait_event(self.copied[i])
        return self.bufs[i % 2][:c].reshape((c * self.x.shape[0],) + tuple(self.x.shape[1:]))

    def done(self, i: int):
        if self.gpu:
            ev = torch.cuda.Event()
            ev.record(self.main)
            self.decoded[i] = ev


def arrival_orders(epoch: int, proposers, n: int, node: int = -1) -> np.ndarray:
    """[k][n] senders of instance proposers[k]'s decryption shares in arrival
    order at `node` (-1: the shared view) — a seeded permutation: the
    network's timing, an input."""
    return arrival_orders_views(epoch, proposers, n, [node])[0]


def _i64(x: int) -> int:
    """A u64 constant as the int64 with the same bits (torch arithmetic wraps)."""
    return x - (1 << 64) if x >= 1 << 63 else x


def arrival_orders_views(epoch: int, proposers, n: int, nodes, device=None) -> np.ndarray:
    """[len(nodes)][k][n]: arrival_orders for several views at once — the
    same SplitMix64 streams (sender s's key = the stream's (s+1)-th output,
    ties by sender), evaluated as wrapping 64-bit tensor arithmetic (on
    `device` when given) instead of one Python call per key (a 128-node epoch
    has 128 x 128 x 128 keys)."""
    return arrival_orders_views_t(epoch, proposers, n, nodes, device).cpu().numpy().astype(np.int64)


def arrival_orders_views_t(epoch: int, proposers, n: int, nodes, device=None) -> torch.Tensor:
    """arrival_orders_views as an int64 tensor on `device`."""
    ids = [[arrival_id(epoch, int(p), int(v)) ^ BASE_SEED ^ (TAG_ARRIVAL << 48) for p in proposers] for v in nodes]
    seed = torch.tensor([[_i64(x) for x in row] for row in ids], dtype=torch.int64, device=device)   # [v][k]
    z = seed.unsqueeze(-1) + _i64(GAMMA) * torch.arange(1, n + 1, dtype=torch.int64, device=device)

    def shr(x, k):  # logical shift of the u64 bits
        return (x >> k) & ((1 << (64 - k)) - 1)
    z = (z ^ shr(z, 30)) * _i64(0xBF58476D1CE4E5B9)
    z = (z ^ shr(z, 27)) * _i64(0x94D049BB133111EB)
    z = z ^ shr(z, 31)
    key = z ^ (-(1 << 63))  # u64 order as int64 order
    return torch.sort(key, dim=-1, stable=True).indices


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
    views: list                  # TDec views: this rank's node ids (per node) or [-1] (shared view)
    ct_status: torch.Tensor      # [view][k] 0 or HBG_E_INVALID_CIPHERTEXT / HBG_E_NOT_ENOUGH_SHARES
    plaintexts: torch.Tensor     # [view][k][P] (rows with status 0)
    share_outcome: torch.Tensor  # [view][k][N] HBG_SHARE_*
    times_ms: dict
    exchange_bytes: int          # bytes this rank received in the epoch's collectives
    work: dict                   # per-rank counts: Value / Echo validations, decodes, TDec instances and shares


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

    def _value_round(self, vbuf, v_off, vsent, per_node: bool):
        """Deliver the Value messages and check them at their recipients.
        Returns (value_ok [N p][N j], the received bytes, the byte offset of
        (source rank, local recipient a)'s run of m messages, validations)."""
        e, N, m, L, r0 = self.engine, self.N, self.m, self.L, self.rank * self.m
        dev = e.device
        lens = self.msg_len
        vsent_all = self._gather(vsent.view(1, N, m)).view(self.world, N, m)   # [r'][j][p local to r']
        if per_node:
            # all-to-all: rank r' sends rank r the messages (j in r's nodes, p in r')
            rank_bytes = [m * int(lens[q * m:(q + 1) * m].sum()) for q in range(self.world)]
            B = rank_bytes[self.rank]
            vrecv = all_to_all_bytes(vbuf, rank_bytes, [B] * self.world, self.world, self.group)
            self._recv += (self.world - 1) * B
            mine = lens[r0:r0 + m]
            g_len = np.tile(np.repeat(mine, m), self.world)   # (r', a, b): msg_len[r0 + a]
            run_off = lambda rs, a: rs * B + m * int(mine[:a].sum())
            j_of = torch.arange(r0, r0 + m, dtype=torch.int32, device=dev).repeat_interleave(m).repeat(self.world)
            sent = vsent_all[:, r0:r0 + m, :]                 # [r'][a][b]
        else:
            vrecv = self._gather(vbuf)                        # [r'][j][p local to r']: every message
            B = int(v_off[-1])
            g_len = np.tile(np.repeat(lens, m), self.world)
            run_off = lambda rs, a: rs * B + m * int(lens[:r0 + a].sum())
            j_of = torch.arange(N, dtype=torch.int32, device=dev).repeat_interleave(m).repeat(self.world)
            sent = vsent_all
        g_off = np.zeros(len(g_len) + 1, np.int64)
        g_off[1:] = np.cumsum(g_len)
        tag, vals, idx, dig, nd, roots, st = e.read_msgs(N, L, vrecv, g_off)
        vok = e.validate_table(N, L, vals, idx, dig, nd, roots)
        good = (st == 0) & (tag == _lib.HBG_MSG_VALUE) & (idx == j_of) & (vok == 1)
        if per_node:
            good = good.view(self.world, m, m) & (sent == 1)  # [r'][a][b]
            local_ok = good.permute(0, 2, 1).reshape(N, m)    # [p][j local]
            value_ok = self._gather(local_ok.t().contiguous().to(torch.uint8)).t().bool()   # [p][j]
        else:
            good = good.view(self.world, N, m) & (sent == 1)
            value_ok = good.permute(0, 2, 1).reshape(N, N)
        return value_ok, vrecv, run_off, len(g_len)

    def run(self, epoch: int = 0, faults: Faults = Faults(), per_node: bool = True,
            decode_chunk: int = 32) -> EpochResult:
        """One epoch.  per_node: every local node does its own work (Values
        addressed to it, all echoes, its decodes, its ThresholdDecrypt of every
        accepted ciphertext with its own arrival order); otherwise the shared
        view (one check / decode / TDec instance per rank on behalf of all
        its nodes).  decode_chunk: local nodes whose decode copies are
        resident (and launched) at once (the decoder reconstructs in place)."""
        e, N, m, L, C, P, f = self.engine, self.N, self.m, self.L, self.C, self.P, self.f
        dev = e.device
        r0 = self.rank * m
        local = self.local_nodes()
        views = list(local) if per_node else [-1]
        nv = len(views)
        self._recv = 0
        work = {}
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
        value_ok, vrecv, run_off, n_val = self._value_round(vbuf, v_off, vsent, per_node)
        work["value_validations"] = n_val
        e.sync()
        t2 = time.perf_counter()
        times["value"] = (t2 - t1) * 1e3
        # ---- 3. Echo: node j's Echo of p's proof = the Value bytes with variant 1
        runs = []
        for a in range(m):
            j = r0 + a
            for rs in range(self.world):
                lo = run_off(rs, a)
                runs.append(vrecv[lo:lo + m * int(self.msg_len[j])])
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
        s_of = torch.arange(N, dtype=torch.int32, device=dev).repeat_interleave(N)
        parsed = (st == 0) & (tag == _lib.HBG_MSG_ECHO) & (idx == s_of)
        # every view validates every echo it receives (hbbft handle_echo): each
        # view hashes the N x N echoes itself, all views in one launch over the
        # one parsed table (hbg_merkle_validate_views: one view's N*N proofs
        # are too few lanes to fill the chip; no per-view copies)
        eok = list(e.validate_table(N, L, vals, idx, dig, nd, roots, views=nv).view(nv, -1))
        work["echo_validations"] = nv * N * N
        echo_ok_v = torch.stack([(parsed & (x == 1)).view(N, N) & (esent_all == 1) for x in eok])   # [v][s][p]
        # echoes per root: the root with the most valid echoes (ties: lowest sender)
        R = roots.view(N, N, 32).permute(1, 0, 2)             # [p][s][32]
        eq = (R.unsqueeze(2) == R.unsqueeze(1)).all(-1)       # [p][s][s']
        ok_ps = echo_ok_v.permute(0, 2, 1)                    # [v][p][s]
        cnt_all = torch.einsum("pst,vpt->vps", eq.to(torch.float32), ok_ps.to(torch.float32)).round().to(torch.int64)
        cnt = torch.where(ok_ps, cnt_all, torch.full_like(cnt_all, -1))
        key = cnt * (N + 1) + (N - torch.arange(N, device=dev))                  # max count, then lowest s
        best = key.argmax(dim=2)                              # [v][p]
        echo_count = cnt.gather(2, best.unsqueeze(2)).squeeze(2).clamp(min=0)   # [v][p]
        ar = torch.arange(N, device=dev)
        root_p = R[ar.unsqueeze(0), best]                     # [v][p][32]
        holds = eq[ar.unsqueeze(0), best] & ok_ps             # [v][p][s] valid echoes carrying root_p
        e.sync()
        t3 = time.perf_counter()
        times["echo"] = (t3 - t2) * 1e3
        # ---- 4. Ready (node j's Readys: its own echo count; every node counts the same messages)
        rv = (torch.arange(m, device=dev) if per_node else torch.zeros(m, dtype=torch.int64, device=dev))
        rbuf = e.zeros((m, N, 36))
        rbuf[:, :, 0] = _lib.HBG_MSG_READY
        rbuf[:, :, 4:] = root_p[rv]
        rsent = (echo_count[rv] >= N - f).to(torch.uint8)     # [j local][p]
        for j in faults.silent:
            if j in local:
                rsent[j - r0] = 0
        rall = self._gather(rbuf.view(m * N, 36)).view(-1)
        rsent_all = self._gather(rsent)                       # [N j][N p]
        r_off = np.arange(N * N + 1, dtype=np.int64) * 36
        tag, _, _, _, _, rroots, st = e.read_msgs(N, 16, rall, r_off)   # digests only: no value table needed
        rgood = ((st == 0) & (tag == _lib.HBG_MSG_READY)).view(N, N) & (rsent_all == 1)
        rmatch = (rroots.view(1, N, N, 32) == root_p.unsqueeze(1)).all(-1) & rgood.unsqueeze(0)   # [v][j][p]
        ready_count = rmatch.sum(1)                           # [v][p]
        delivered = (ready_count >= 2 * f + 1) & (echo_count >= N - 2 * f)       # [v][p]
        # ---- 5. decode from the echoes carrying the root: every view its own copy
        S = vals.shape[-1]
        sh = vals.view(N, N, S).permute(1, 0, 2).contiguous()  # [p][s][S]
        present = (holds & delivered.unsqueeze(2)).to(torch.uint8)   # [v][p][s]
        D = bc.shard_counts(N)[0]
        OS = (D * L + 15) // 16 * 16
        out = e.zeros((nv, N, OS))                            # every view's decodes, written in place
        plens, dsts = [], []
        chunks = [(c0, min(decode_chunk, nv - c0)) for c0 in range(0, nv, decode_chunk)]
        copies = _CopyPipe(sh, chunks, dev)   # chunk i+1's copies made beside chunk i's decode
        for i, (c0, c) in enumerate(chunks):
            _, pl, ds = e.decode(N, L, copies.get(i), present[c0:c0 + c].reshape(c * N, N).contiguous(),
                                 root_p[c0:c0 + c].reshape(c * N, 32).contiguous(),
                                 out=out[c0:c0 + c].view(c * N, OS))
            copies.done(i)
            plens.append(pl.view(c, N))
            dsts.append(ds.view(c, N))
        plen, dst = torch.cat(plens), torch.cat(dsts)          # [v][p]
        work["decodes"] = nv * N
        out = out[..., :C] if out.shape[-1] >= C else torch.nn.functional.pad(out, (0, C - out.shape[-1]))
        le = (out[..., 48:56].to(torch.int64) << (8 * torch.arange(8, device=dev))).sum(-1)
        payload_ok = delivered & (dst == _lib.HBG_DECODE_OK) & (plen == C) & (le == P)   # [v][p]
        if not bool((payload_ok == payload_ok[0:1]).all()):
            # Subset's output is agreed by binary agreement (out of scope): with
            # full delivery every view must deliver the same set
            raise RuntimeError("views disagree on the delivered proposals")
        e.sync()
        t4 = time.perf_counter()
        times["ready_decode"] = (t4 - t3) * 1e3
        # ---- 6/7. Subset accepts; ThresholdDecrypt of every accepted ciphertext, per view
        acc = torch.nonzero(payload_ok[0]).flatten().tolist()
        k = len(acc)
        if k:
            at = torch.tensor(acc, device=dev)
            U, V, W = out[0, at, :48].contiguous(), out[0, at, CT_HEAD:CT_HEAD + P].contiguous(), out[0, at, CT_HEAD + P:C]
            pc = torch.arange(k, dtype=torch.int32, device=dev).repeat_interleave(m)
            pj = torch.arange(m, dtype=torch.int32, device=dev).repeat(k)
            sk_use = self.sk32_local.clone()
            for j in faults.bad_share:
                if j in local:
                    sk_use[j - r0] = self.sk32[(j + 1) % N]
            shares = e.decrypt_shares(U, sk_use, pc, pj).view(k, m, 48)
            sall = self._gather(shares.permute(1, 0, 2).contiguous())   # [N s][k][48]
            share48 = sall.permute(1, 0, 2).contiguous()                # [k][N][48]
            # the arrival lists, built on the device ([v][k][N]: 2.1 M entries at N = 128)
            silent = torch.tensor([s in faults.silent for s in range(N)], device=dev)
            order = arrival_orders_views_t(epoch, acc, N, views, dev)       # [v][k][N]
            keep = ~silent[order]
            per_node = views[0] >= 0
            vv = torch.tensor(views, dtype=torch.int64, device=dev).view(-1, 1, 1)
            if per_node:  # a node's own share is no network arrival: its start_decryption inserts it
                keep &= order != vv
            # silent senders' entries dropped, the rest kept in arrival order, -1 padded
            order = torch.take_along_dim(order, torch.argsort((~keep).to(torch.uint8), dim=-1, stable=True), -1)
            order = torch.where(torch.arange(N, device=dev) < keep.sum(-1, keepdim=True), order, -1)
            if per_node:  # hbbft start_decryption at validator v (HBG_ARRIVAL_OWN | v) before any arrival
                order = torch.cat([(vv | _lib.HBG_ARRIVAL_OWN).expand(nv, k, 1), order], -1)
            arr = torch.where(order >= 1 << 31, order - (1 << 32), order).to(torch.int32)  # u32 bits
            # view v's instance of ciphertext q: its own copy of (U, V, W) and the N shares
            sh = _copies(share48, nv).view(nv, k, N, 48)
            for vi, v in enumerate(views):
                if per_node and v in faults.bad_share:  # it sends a wrong share, but holds its true one
                    sh[vi, :, v] = e.decrypt_shares(U, self.sk32[v:v + 1].contiguous(),
                                                    torch.arange(k, dtype=torch.int32, device=dev),
                                                    torch.zeros(k, dtype=torch.int32, device=dev)).view(k, 48)
            V_off = torch.arange(nv * k + 1, dtype=torch.int64, device=dev) * P
            pt, ct_status, outcome = e.threshold_decrypt(
                self.t, N, _copies(U, nv), _copies(V, nv).reshape(-1), V_off, _copies(W.contiguous(), nv),
                self.pk48, sh.reshape(nv * k, N, 48), arr.reshape(nv * k, -1).contiguous())
            plaintexts = pt.view(nv, k, P)
            ct_status = ct_status.view(nv, k)
            outcome = outcome.view(nv, k, N)
        else:
            ct_status = torch.zeros((nv, 0), dtype=torch.int32, device=dev)
            plaintexts = e.zeros((nv, 0, P))
            outcome = e.zeros((nv, 0, N))
        work["tdec_instances"] = nv * k
        work["tdec_shares"] = nv * k * N
        e.sync()
        t5 = time.perf_counter()
        times["tdec"] = (t5 - t4) * 1e3
        times["epoch"] = (t5 - t0) * 1e3
        return EpochResult(value_ok, echo_ok_v[0], echo_count[0], ready_count[0], delivered[0], out[0],
                           payload_ok[0], acc, views, ct_status, plaintexts, outcome, times, self._recv, work)
