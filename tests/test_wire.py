"""hbbft broadcast wire format (bincode of
``Message::{Value,Echo}(Proof)`` / ``Ready(Digest)``).

CPU tests pin the oracle (oracle/wire.py) against the committed fixture
tests/golden/wire_golden.json (generator: tests/golden/make_golden_wire.py) and
against its own Proof::validate; GPU tests run ``hbg_rbc_write_proof_msgs`` /
``hbg_rbc_read_msgs`` through the C ABI and compare bytes, fields and statuses
with the oracle and the fixture bit for bit, and at BASELINE size (N=64,
1 MiB) check the write -> read -> validate round trip.  Parity of the hbbft
type layout itself is unpinned (no hbbft source/fixture in the container)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from oracle import merkle, rbc as orbc, synth, wire

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "wire_golden.json")))


# ------------------------------------------------------------------ oracle (CPU)
def test_oracle_regenerates_fixture_messages():
    for t in GOLD["trees"]:
        pl = synth.payload(t["instance"], t["P"])
        shards, tree = orbc.send_shards(pl, t["N"])
        assert shards.tobytes().hex() == t["shards_hex"]
        assert tree.root_hash.hex() == t["root"]
        for i, h in enumerate(t["msgs"]):
            tag = wire.VALUE if i % 2 == 0 else wire.ECHO
            assert wire.serialize_proof_msg(tag, tree.proof(i)).hex() == h
            assert len(h) // 2 == 12 + t["L"] + 16 + 32 * wire.proof_digests(t["N"], i) + 32


def test_oracle_roundtrip_and_validate():
    for t in GOLD["trees"]:
        for i, h in enumerate(t["msgs"]):
            st, tag, p = wire.deserialize(bytes.fromhex(h))
            assert st == wire.OK and tag == (i % 2) and p.index == i
            assert p.validate(t["N"])
            assert wire.serialize_proof_msg(tag, p).hex() == h
        st, tag, d = wire.deserialize(bytes.fromhex(t["ready"]))
        assert (st, tag, d.hex()) == (wire.OK, wire.READY, t["root"])


def test_oracle_malformed_cases_match_fixture():
    for c in GOLD["malformed"]["cases"]:
        st, tag, p = wire.deserialize(bytes.fromhex(c["hex"]))
        assert st == c["status"], c["name"]
        assert tag == c["tag"], c["name"]


def test_proof_digest_counts_match_tree():
    for n in [1, 2, 3, 4, 5, 7, 16, 63, 64, 100, 128, 256]:
        tree = merkle.MerkleTree([bytes([i]) for i in range(n)])
        for i in range(n):
            assert len(tree.proof(i).digests) == wire.proof_digests(n, i)


def test_abi_message_lengths():
    from hydrabadger_amd import _lib
    l = _lib.lib()
    for n in [1, 4, 7, 64, 128]:
        for i in range(n):
            assert l.hbg_proof_digests(n, i) == wire.proof_digests(n, i)
            assert l.hbg_proof_msg_len(n, i, 47663) == 12 + 47663 + 16 + 32 * wire.proof_digests(n, i) + 32
        assert l.hbg_proof_msg_len(n, n, 10) == 0
    assert l.hbg_strerror(_lib.HBG_E_WIRE_EOF) == b"UnexpectedEof"
    assert l.hbg_strerror(_lib.HBG_E_WIRE_TAG) == b"InvalidVariant"


# ------------------------------------------------------------------ GPU (C ABI)
def _bc():
    from hydrabadger_amd import broadcast as bc
    return bc


@pytest.mark.gpu
@pytest.mark.parametrize("ti", range(len(GOLD["trees"])))
def test_gpu_serialize_matches_fixture(ti):
    bc = _bc()
    t = GOLD["trees"][ti]
    N, L = t["N"], t["L"]
    sh = np.frombuffer(bytes.fromhex(t["shards_hex"]), np.uint8).reshape(N, L)
    tree = bc.MerkleTree.from_vec([sh[i].tobytes() for i in range(N)])
    vals = bc.serialize_proof_messages(tree, bc.Message.VALUE)
    echo = bc.serialize_proof_messages(tree, bc.Message.ECHO, indices=list(range(N))[::-1])
    for i in range(N):
        ref = bytes.fromhex(t["msgs"][i])
        if i % 2 == 0:
            assert vals[i] == ref, i
        else:
            assert echo[N - 1 - i] == ref, i


@pytest.mark.gpu
@pytest.mark.parametrize("ti", range(len(GOLD["trees"])))
def test_gpu_deserialize_fixture_and_validate(ti):
    bc = _bc()
    t = GOLD["trees"][ti]
    N, L = t["N"], t["L"]
    msgs = [bytes.fromhex(h) for h in t["msgs"]] + [bytes.fromhex(t["ready"])]
    out = bc.deserialize_messages(msgs, N, L)
    for i in range(N):
        m = out[i]
        assert isinstance(m, bc.Message) and m.kind == i % 2
        _, _, ref = wire.deserialize(msgs[i])
        assert (m.payload.value, m.payload.index, m.payload.digests, m.payload.root_hash) == \
            (ref.value, ref.index, ref.digests, ref.root_hash)
    assert out[N].kind == bc.Message.READY and out[N].payload.hex() == t["root"]
    ok = bc.validate_proofs([m.payload for m in out[:N]], N)
    assert ok.all()


@pytest.mark.gpu
def test_gpu_malformed_messages():
    bc = _bc()
    from hydrabadger_amd import _lib
    t = GOLD["trees"][GOLD["malformed"]["tree"]]
    N, L = t["N"], t["L"]
    cases = GOLD["malformed"]["cases"]
    out = bc.deserialize_messages([bytes.fromhex(c["hex"]) for c in cases], N, L)
    for c, m in zip(cases, out):
        if c["status"] != 0:
            assert isinstance(m, bc.WireError) and m.code == c["status"], c["name"]
        elif c["tag"] <= 1 and c["value_len"] != L:
            assert isinstance(m, bc.WireError) and m.code == _lib.HBG_E_INCORRECT_SHARD_SIZE, c["name"]
        elif c["tag"] <= 1:
            assert isinstance(m, bc.Message) and m.kind == c["tag"], c["name"]
            assert m.payload.index == c["index"] and m.payload.root_hash.hex() == c["root"]
            assert bool(bc.validate_proofs([m.payload], N)[0]) == c["validates"], c["name"]
        else:
            assert isinstance(m, bc.Message) and m.kind == c["tag"] and m.payload.hex() == c["digest"], c["name"]


@pytest.mark.gpu
def test_gpu_read_table_fields_for_bad_layouts():
    """Raw table output: INCORRECT_SHARD_SIZE keeps tag/index/root; an
    over-long digest list is marked 0xFFFFFFFF and validates false."""
    bc = _bc()
    from hydrabadger_amd import _lib
    t = GOLD["trees"][3]
    N, L = t["N"], t["L"]
    cases = {c["name"]: bytes.fromhex(c["hex"]) for c in GOLD["malformed"]["cases"]}
    msgs = [cases["short_value"], cases["extra_digest"], bytes.fromhex(t["msgs"][6])]
    m = len(msgs)
    off = np.zeros(m + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in msgs])
    buf = np.frombuffer(b"".join(msgs), np.uint8).copy()
    depth = _lib.merkle_depth(N)
    tag, index, nd, st = (np.zeros(m, np.uint32), np.zeros(m, np.uint32), np.zeros(m, np.uint32),
                          np.zeros(m, np.int32))
    vals, dig, roots = np.zeros((m, L), np.uint8), np.zeros((m, depth, 32), np.uint8), np.zeros((m, 32), np.uint8)
    bc.read_msgs_batch(N, L, buf, off, tag, vals, index, dig, nd, roots, st)
    assert list(st) == [_lib.HBG_E_INCORRECT_SHARD_SIZE, 0, 0]
    assert list(tag) == [0, 1, 0] and list(index) == [2, 2, 6]
    assert nd[1] == 0xFFFFFFFF and nd[2] == wire.proof_digests(N, 6)
    assert roots[0].tobytes().hex() == t["root"] == roots[1].tobytes().hex()
    ok = np.zeros(m, np.uint8)
    from hydrabadger_amd._lib import lib, ptr, default_context
    assert lib().hbg_merkle_validate(default_context().h, N, L, ptr(vals), L, ptr(index), ptr(dig), ptr(nd),
                                     ptr(roots), ptr(ok), m, 0) == 0
    assert list(ok[1:]) == [0, 1]
    # each of three views validates the table itself (host mode), view-major
    ok3 = np.full(3 * m, 7, np.uint8)
    assert lib().hbg_merkle_validate_views(default_context().h, N, L, ptr(vals), L, ptr(index), ptr(dig), ptr(nd),
                                           ptr(roots), ptr(ok3), m, 3, 0) == 0
    assert np.array_equal(ok3, np.tile(ok, 3))
    assert lib().hbg_merkle_validate_views(default_context().h, N, L, ptr(vals), L, ptr(index), ptr(dig), ptr(nd),
                                           ptr(roots), ptr(ok3), m, 0, 0) == _lib.HBG_E_ARG


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("N,P,n", [(64, 1 << 20, 4), (16, 65536, 16), (128, 1 << 20, 2), (5, 333, 40)])
def test_gpu_device_batch_write_read_validate(N, P, n):
    """BASELINE sizes, device-resident: every Value message of every instance
    is bit-identical to the oracle's serialisation (spot instances), parses
    back to the shard batch, and every parsed proof validates; a flipped byte
    in a value makes exactly that proof fail."""
    torch = _torch()
    bc = _bc()
    from hydrabadger_amd import _lib
    from oracle import corc
    L = _lib.shard_len(N, P)
    S = (L + 15) // 16 * 16
    dev = torch.device("cuda:0")
    pay = torch.empty((n, (P + 15) // 16 * 16), dtype=torch.uint8, device=dev)
    bc.synth_bytes(synth.TAG_PAYLOAD, 77, P, pay, device=True)
    plen = torch.full((n,), P, dtype=torch.int64, device=dev)
    shards = torch.empty((n, N, S), dtype=torch.uint8, device=dev)
    levels = torch.empty((n, _lib.merkle_nodes(N), 32), dtype=torch.uint8, device=dev)
    bc.rbc_encode_merkle_batch(N, pay, plen, L, shards, levels, device=True)
    inst = np.repeat(np.arange(n, dtype=np.uint64), N)
    idx = np.tile(np.arange(N, dtype=np.uint32), n)
    off = bc.proof_msg_offsets(N, L, idx)
    total = int(off[-1])
    out = torch.zeros(total + 16, dtype=torch.uint8, device=dev)
    d_inst = torch.from_numpy(inst.astype(np.int64)).to(dev)
    d_idx = torch.from_numpy(idx.astype(np.int32)).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    bc.write_proof_msgs_batch(N, L, shards, levels, bc.Message.VALUE, d_inst, d_idx, out, d_off, device=True)
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    for k in sorted({0, n - 1}):
        payload = np.frombuffer(synth.payload(77 + k, P), np.uint8).copy()
        rs, _ = corc.rbc_encode_merkle(N, payload)
        tree = merkle.MerkleTree([rs[i].tobytes() for i in range(N)])
        for i in sorted({0, 1, N // 2, N - 1}):
            j = k * N + i
            assert host[off[j]:off[j + 1]].tobytes() == wire.serialize_proof_msg(wire.VALUE, tree.proof(i)), (k, i)
    m = n * N
    depth = max(_lib.merkle_depth(N), 1)
    # one corrupted value byte per instance (message k*N + (k % N))
    bad = [k * N + (k % N) for k in range(n)]
    for j in bad:
        out[int(off[j]) + 12 + (j * 7919) % L] ^= 0x5A
    tag = torch.empty(m, dtype=torch.int32, device=dev)
    vals = torch.empty((m, S), dtype=torch.uint8, device=dev)
    rindex = torch.empty(m, dtype=torch.int32, device=dev)
    dig = torch.empty((m, depth, 32), dtype=torch.uint8, device=dev)
    nd = torch.empty(m, dtype=torch.int32, device=dev)
    roots = torch.empty((m, 32), dtype=torch.uint8, device=dev)
    st = torch.empty(m, dtype=torch.int32, device=dev)
    bc.read_msgs_batch(N, L, out, d_off, tag, vals, rindex, dig, nd, roots, st, device=True)
    ok = torch.empty(m, dtype=torch.uint8, device=dev)
    h = _lib.default_context().h
    assert _lib.lib().hbg_merkle_validate(h, N, L, _lib.ptr(vals), S, _lib.ptr(rindex), _lib.ptr(dig), _lib.ptr(nd),
                                          _lib.ptr(roots), _lib.ptr(ok), m, _lib.HBG_DEVICE) == 0
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and int(tag.sum()) == 0
    assert torch.equal(rindex.cpu(), d_idx.cpu())
    expect = np.ones(m, np.uint8)
    expect[bad] = 0
    assert np.array_equal(ok.cpu().numpy(), expect)
    # every view of a rank validates the whole table itself, one launch, no copies
    views = 5
    okv = torch.full((views * m,), 7, dtype=torch.uint8, device=dev)
    assert _lib.lib().hbg_merkle_validate_views(h, N, L, _lib.ptr(vals), S, _lib.ptr(rindex), _lib.ptr(dig),
                                                _lib.ptr(nd), _lib.ptr(roots), _lib.ptr(okv), m, views,
                                                _lib.HBG_DEVICE) == 0
    torch.cuda.synchronize()
    assert np.array_equal(okv.cpu().numpy(), np.tile(expect, views))
    good = np.setdiff1d(np.arange(m), bad)
    ref_vals = shards.reshape(m, S)[:, :L]
    assert torch.equal(vals[torch.from_numpy(good).to(dev), :L], ref_vals[torch.from_numpy(good).to(dev)])
    lv = levels[:, -1, :]
    assert torch.equal(roots.reshape(n, N, 32), lv[:, None, :].expand(n, N, 32))
