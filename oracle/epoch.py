"""One HoneyBadger epoch, node by node and message by message (TEST
INFRASTRUCTURE ONLY — see oracle/__init__.py; SURVEY.md §8 f4 + a18).

The checker for hydrabadger_amd/epoch.py.  It restates, for a fully
connected N-node network that delivers every message, what each node's hbbft
state machines do with the epoch's messages [EXT, VegeBun-csj/hbbft master,
unvendored; reached from /root/reference/src/hydrabadger/state.rs:484
(propose) and :486-487 (handle_message), messages forwarded to all peers at
handler.rs:747-764]:

* HoneyBadger::propose: the contribution is threshold-encrypted under the
  master key (encrypt_with_rng) and the serialised ciphertext is proposed.
* Broadcast (one instance per proposer p):
  - send_shards: Value(proof_j) to node j (bincode wire messages, oracle/wire.py);
  - handle_value(p, proof) at node j: accepted iff proof.index == j and
    proof.validate(N) (else FaultKind::InvalidProof); then Echo(proof) to all;
  - handle_echo(s, proof): counted iff proof.index == s and validate(N);
    echoes are counted per root hash;
  - Ready(root) once the root has N - f echoes;
  - output once the root has 2f + 1 Readys and N - 2f echoes:
    decode_from_shards over the echoes carrying that root.
  With every message delivered, all correct nodes see the same echoes, so
  Ready amplification (f + 1 Readys) adds nothing and is not modelled.
* Subset: every delivered instance is accepted (binary agreement, out of
  scope, decides 1 for each of them under full delivery).
* ThresholdDecrypt per accepted ciphertext (threshold t = f): every node's
  share (decrypt_share_no_verify), handled in a seeded arrival order
  (tcrypto.threshold_decrypt: set_ciphertext, faults, first t+1 valid,
  late shares ignored).

Two views of the TDec stage (``per_node``): every node runs its own
ThresholdDecrypt instance of every accepted ciphertext, with its own seeded
arrival order (the network's per-node work, hbbft's behaviour); or, the
shared view, one instance per ciphertext on behalf of all nodes.  The RBC
stages' outcomes are the same at every node under full delivery (every
node receives the same Values for its index and the same Echoes / Readys),
so they are restated once.

Faults injected (the same set epoch.py takes): silent nodes (send nothing),
corrupted Values (p, j), nodes that echo a corrupted value, proposers whose
ciphertext is corrupted after encryption, nodes that send a share computed
with another node's key.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

from . import bls12_381 as B
from . import merkle, rbc, synth, tcrypto as T, wire

TAG_CONTRIB, TAG_R, TAG_ARRIVAL = 6, 7, 8
CT_HEAD, CT_TAIL = 48 + 8, 96


@dataclass(frozen=True)
class Faults:
    silent: frozenset = frozenset()
    bad_value: frozenset = frozenset()   # (p, j)
    bad_echo: frozenset = frozenset()
    bad_ct: frozenset = frozenset()
    bad_share: frozenset = frozenset()


def instance_id(epoch: int, p: int) -> int:
    # bits [0, 20) proposer, [20, 40) epoch; arrival_id puts node + 1 in [40, 48)
    # and the stream tag sits at bit 48, so every field must stay in its range
    if not (0 <= p < 1 << 20 and 0 <= epoch < 1 << 20):
        raise ValueError(f"instance id fields out of range: epoch {epoch}, proposer {p}")
    return (epoch << 20) | p


def keyset(n: int, t: int, seed: int):
    """hydrabadger_amd/tdec_workload.py keyset(): coefficients and shares."""
    rng = synth.SplitMix64(synth.TAG_TDEC, 0xC0EF ^ seed)
    coeffs = []
    for _ in range(t + 1):
        v = 0
        for _ in range(4):
            v = (v << 64) | rng.next()
        coeffs.append(v % B.R)
    return coeffs, [T.SecretKeySet(coeffs).secret_key_share(i) for i in range(n)]


def contribution(epoch: int, p: int, P: int) -> bytes:
    return synth.synth_bytes(TAG_CONTRIB, instance_id(epoch, p), P)


def encryption_scalar(epoch: int, p: int) -> int:
    b = bytearray(synth.synth_bytes(TAG_R, instance_id(epoch, p), 32))
    b[31] &= 0x3F
    return int.from_bytes(b, "little")


def arrival_id(epoch: int, p: int, node: int | None = None) -> int:
    """Seed id of an arrival order: instance p's shared view, or node `node`'s."""
    if node is not None and not 0 <= node < 255:
        raise ValueError(f"node {node} does not fit the arrival id's 8-bit node field")
    return instance_id(epoch, p) | (0 if node is None else (node + 1) << 40)


def arrival_order(epoch: int, p: int, n: int, node: int | None = None) -> list:
    """Senders of instance p's decryption shares in arrival order (at `node`,
    or the shared view)."""
    rng = synth.SplitMix64(TAG_ARRIVAL, arrival_id(epoch, p, node))
    keys = [rng.next() for _ in range(n)]
    return sorted(range(n), key=lambda s: (keys[s], s))


def serialize_ct(ct: T.Ciphertext) -> bytes:
    return B.g1_compress(ct.U) + struct.pack("<Q", len(ct.V)) + bytes(ct.V) + B.g2_compress(ct.W)


def parse_ct(b: bytes, P: int):
    """(U48, V, W96) of a serialised ciphertext of a P-byte contribution, or None."""
    if len(b) != CT_HEAD + P + CT_TAIL or struct.unpack_from("<Q", b, 48)[0] != P:
        return None
    return b[:48], b[CT_HEAD:CT_HEAD + P], b[CT_HEAD + P:]


@dataclass
class EpochOut:
    value_ok: list = field(default_factory=list)     # [p][j]
    echo_ok: list = field(default_factory=list)      # [s][p]
    echo_count: list = field(default_factory=list)   # [p]
    ready_count: list = field(default_factory=list)  # [p]
    delivered: list = field(default_factory=list)    # [p]
    payloads: list = field(default_factory=list)     # [p] decoded bytes or None
    accepted: list = field(default_factory=list)     # proposers of the accepted ciphertexts
    views: list = field(default_factory=list)        # TDec views: node ids (per node) or [None] (shared)
    ct_status: list = field(default_factory=list)    # [view][k]
    plaintexts: list = field(default_factory=list)   # [view][k] bytes or None
    share_outcome: list = field(default_factory=list)  # [view][k][s]


def run_epoch(N: int, P: int, seed: int = 1, epoch: int = 0, faults: Faults = Faults(),
              per_node: bool = True) -> EpochOut:
    f = rbc.num_faulty(N)
    t = f
    coeffs, sks = keyset(N, t, seed)
    master_pk = B.g1_mul(B.G1, coeffs[0])
    pk_shares = [B.g1_mul(B.G1, s) for s in sks]
    out = EpochOut()
    # ---- proposals: encrypt, serialise, send_shards, Value messages
    values = [[None] * N for _ in range(N)]      # values[p][j]: wire bytes of p's Value to j
    for p in range(N):
        ct = T.encrypt(master_pk, contribution(epoch, p, P), encryption_scalar(epoch, p))
        if p in faults.bad_ct:
            ct = T.Ciphertext(ct.U, bytes([ct.V[0] ^ 1]) + ct.V[1:], ct.W)
        if p in faults.silent:
            continue
        _, tree = rbc.send_shards(serialize_ct(ct), N)
        for j in range(N):
            pr = tree.proof(j)
            if (p, j) in faults.bad_value:
                pr = merkle.Proof(bytes([pr.value[0] ^ 0xFF]) + bytes(pr.value[1:]), pr.index, pr.digests,
                                  pr.root_hash)
            values[p][j] = wire.serialize_proof_msg(wire.VALUE, pr)
    # ---- handle_value at node j, Echo to all
    out.value_ok = [[False] * N for _ in range(N)]
    echoes = [[None] * N for _ in range(N)]      # echoes[s][p]: wire bytes of s's Echo for instance p
    for p in range(N):
        for j in range(N):
            if values[p][j] is None:
                continue
            st, tag, pr = wire.deserialize(values[p][j])
            ok = st == wire.OK and tag == wire.VALUE and pr.index == j and pr.validate(N)
            out.value_ok[p][j] = ok
            if ok and j not in faults.silent:
                if j in faults.bad_echo:
                    pr = merkle.Proof(bytes([pr.value[0] ^ 0xFF]) + bytes(pr.value[1:]), pr.index, pr.digests,
                                      pr.root_hash)
                echoes[j][p] = wire.serialize_proof_msg(wire.ECHO, pr)
    # ---- handle_echo (every node sees the same echoes), Ready, output
    out.echo_ok = [[False] * N for _ in range(N)]
    for p in range(N):
        by_root = {}
        for s in range(N):
            if echoes[s][p] is None:
                continue
            st, tag, pr = wire.deserialize(echoes[s][p])
            if st == wire.OK and tag == wire.ECHO and pr.index == s and pr.validate(N):
                out.echo_ok[s][p] = True
                by_root.setdefault(bytes(pr.root_hash), {})[s] = pr
        root, held = max(by_root.items(), key=lambda kv: (len(kv[1]), -min(kv[1]))) if by_root else (None, {})
        n_echo = len(held)
        readys = [wire.serialize_digest_msg(wire.READY, root) for j in range(N)
                  if j not in faults.silent and n_echo >= N - f]
        n_ready = sum(1 for m in readys if wire.deserialize(m)[2] == root)
        out.echo_count.append(n_echo)
        out.ready_count.append(n_ready)
        delivered = n_ready >= 2 * f + 1 and n_echo >= N - 2 * f
        out.delivered.append(delivered)
        payload = None
        if delivered:
            import numpy as np
            leaves = [np.frombuffer(held[s].value, np.uint8).copy() if s in held else None for s in range(N)]
            payload = rbc.decode_from_shards(leaves, N, root)
        out.payloads.append(payload)
    # ---- Subset accepts the delivered instances; ThresholdDecrypt each ciphertext
    cts = []
    for p in range(N):
        if not out.delivered[p] or out.payloads[p] is None:
            continue
        parts = parse_ct(out.payloads[p], P)
        if parts is None:
            continue
        out.accepted.append(p)
        try:
            cts.append(T.Ciphertext(B.g1_decompress(parts[0]), parts[1], B.g2_decompress(parts[2])))
        except ValueError:
            cts.append(None)
    shares = []   # [k][s]: every node's decryption share of each accepted ciphertext
    for ct in cts:
        shares.append(None if ct is None else
                      [None if s in faults.silent else
                       T.decrypt_share(sks[(s + 1) % N] if s in faults.bad_share else sks[s], ct) for s in range(N)])
    caches = [{} for _ in cts]   # verdicts are the same at every node: computed once per ciphertext
    out.views = list(range(N)) if per_node else [None]
    for node in out.views:
        st_v, pt_v, oc_v = [], [], []
        for q, (p, ct) in enumerate(zip(out.accepted, cts)):
            if ct is None:
                st_v.append(T.E_INVALID_CIPHERTEXT)
                pt_v.append(None)
                oc_v.append([T.SHARE_NONE] * N)
                continue
            order = [s for s in arrival_order(epoch, p, N, node) if s not in faults.silent and s != node]
            sh, cache = shares[q], caches[q]
            if node is not None:
                # validator `node`: start_decryption (before any arrival) inserts its own share,
                # decrypt_share_no_verify with its own key — also when it is silent or sends a bad one
                order = [T.ARRIVAL_OWN | node] + order
                if node in faults.silent or node in faults.bad_share:
                    sh = list(sh)
                    sh[node] = T.decrypt_share(sks[node], ct)
                    cache = None
            st, pt, oc = T.threshold_decrypt(t, ct, pk_shares, sh, order, cache=cache)
            st_v.append(st)
            pt_v.append(pt)
            oc_v.append(list(oc))
        out.ct_status.append(st_v)
        out.plaintexts.append(pt_v)
        out.share_outcome.append(oc_v)
    return out
