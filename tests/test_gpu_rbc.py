"""GPU parity tests for the RBC coding path (family 1 + 2), through the C ABI.

Every result is compared bit-for-bit with the oracle (oracle/: numpy + C
restatements of rse / hbbft / tiny-keccak, pinned in tests/test_oracle_rbc.py)
on the same seeded inputs.  Full BASELINE sizes (N=64, 1 MiB) are covered by
size-independent properties: encode -> erase 2f -> decode round trips, proof
validation of every leaf, and oracle spot checks of whole instances.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import corc, gf256, merkle, rbc as orbc, synth

pytestmark = pytest.mark.gpu

CONFIGS = [1, 2, 3, 4, 5, 7, 10, 16, 31, 64, 100, 128, 256]


def _bc():
    from hydrabadger_amd import broadcast as bc
    return bc


@pytest.mark.parametrize("N", CONFIGS)
@pytest.mark.parametrize("P", [0, 1, 5, 117, 1000, 4099])
def test_send_shards_matches_oracle(N, P):
    bc = _bc()
    payload = synth.payload(N * 1000 + P, P)
    shards, tree = bc.send_shards(payload, N)
    ref_shards, ref_tree = orbc.send_shards(payload, N)
    assert np.array_equal(shards, ref_shards)
    assert tree.root_hash() == ref_tree.root_hash
    assert [list(l) for l in tree.levels()] == [list(l) for l in ref_tree.levels]
    for i in range(N):
        p, rp = tree.proof(i), ref_tree.proof(i)
        assert p.digests == rp.digests and p.index == rp.index and p.value == rp.value


@pytest.mark.parametrize("D,Q", [(2, 2), (6, 10), (22, 42), (44, 84), (5, 5), (1, 1), (3, 7), (10, 3),
                                 (100, 100), (17, 80), (200, 56), (1, 255), (255, 1)])
@pytest.mark.parametrize("L", [1, 3, 4, 17, 136, 1001])
def test_rs_encode_matches_oracle(D, Q, L):
    bc = _bc()
    n = 3
    rows = np.frombuffer(synth.synth_bytes(synth.TAG_PAYLOAD, D * 7919 + Q * 31 + L, n * (D + Q) * L),
                         np.uint8).reshape(n, D + Q, L).copy()
    ref = rows.copy()
    for k in range(n):
        corc.rs_encode(D, Q, ref[k])
    got = rows.copy()
    bc.Coding(D, Q).encode_batch(got)
    assert np.array_equal(got[:, :D], rows[:, :D])  # data untouched
    assert np.array_equal(got, ref)


def test_backblaze_kat_on_gpu():
    bc = _bc()
    sh = np.zeros((10, 2), np.uint8)
    sh[:5] = [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]]
    bc.Coding(5, 5).encode(sh)
    assert sh[5:].tolist() == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]


def test_encode_list_of_rows_and_errors():
    bc = _bc()
    rows = [bytearray(b"\x00\x01"), bytearray(b"\x04\x05"), bytearray(2), bytearray(2)]
    bc.Coding(2, 2).encode(rows)
    ref = np.zeros((4, 2), np.uint8)
    ref[0], ref[1] = [0, 1], [4, 5]
    corc.rs_encode(2, 2, ref)
    assert [bytes(r) for r in rows] == [r.tobytes() for r in ref]
    with pytest.raises(bc.RseError) as e:
        bc.Coding(2, 2).encode([bytearray(2)] * 3)
    assert e.value.kind == "TooFewShards"
    with pytest.raises(bc.RseError) as e:
        bc.Coding(2, 2).encode([bytearray(2), bytearray(3), bytearray(2), bytearray(2)])
    assert e.value.kind == "IncorrectShardSize"
    with pytest.raises(bc.RseError) as e:
        bc.Coding(0, 2)
    assert e.value.kind == "TooFewDataShards"
    with pytest.raises(bc.RseError) as e:
        bc.Coding(200, 57)
    assert e.value.kind == "TooManyShards"


@pytest.mark.parametrize("D,Q", [(2, 2), (6, 10), (22, 42), (44, 84), (1, 1), (3, 7), (86, 170), (255, 1)])
def test_reconstruct_matches_oracle(D, Q):
    bc = _bc()
    N, L, n = D + Q, 257, 6
    data = np.frombuffer(synth.synth_bytes(synth.TAG_PAYLOAD, N * 13 + 1, n * N * L), np.uint8).reshape(n, N, L).copy()
    for k in range(n):
        corc.rs_encode(D, Q, data[k])
    present = np.ones((n, N), np.uint8)
    for k in range(n):
        erase = [0, Q, Q // 2, 1, max(Q - 1, 0), Q + 1][k]  # incl. all-present and too-few
        m = synth.erasure_mask(1000 * D + k, N, min(erase, N))
        present[k] = np.array(m, np.uint8)
    damaged = data.copy()
    damaged[present == 0] = 0xEE  # garbage where shards are absent
    st = bc.Coding(D, Q).reconstruct_batch(damaged, present)
    for k in range(n):
        np_ = int(present[k].sum())
        if np_ < D:
            assert st[k] == -14  # TooFewShardsPresent
            continue
        assert st[k] == 0
        ref = data[k].copy()
        ref[present[k] == 0] = 0
        assert corc.rs_reconstruct(D, Q, ref, present[k]) == 0
        assert np.array_equal(damaged[k], ref), (k, D, Q)
        assert np.array_equal(damaged[k], data[k])


def test_reconstruct_keeps_present_as_received():
    """rse uses the FIRST D present rows; a corrupted later present shard is
    kept verbatim and does not influence the rebuilt rows."""
    bc = _bc()
    D, Q, L = 6, 10, 40
    N = D + Q
    sh = np.frombuffer(synth.synth_bytes(1, 99, N * L), np.uint8).reshape(N, L).copy()
    corc.rs_encode(D, Q, sh)
    present = np.ones(N, bool)
    present[[0, 3, 7]] = False
    rows = [sh[i].copy() if present[i] else None for i in range(N)]
    rows[15] = rows[15].copy()
    rows[15][0] ^= 0xFF  # corrupted, but not among the first D present
    oracle_rows = [r.copy() if r is not None else None for r in rows]
    gf256.ReedSolomon(D, Q).reconstruct(oracle_rows)
    bc.Coding(D, Q).reconstruct_shards(rows)
    for i in range(N):
        assert np.array_equal(rows[i], oracle_rows[i]), i
    assert rows[15][0] == sh[15][0] ^ 0xFF


@pytest.mark.parametrize("N", [1, 2, 3, 4, 7, 16, 64, 100, 128, 256])
@pytest.mark.parametrize("L", [0, 1, 8, 135, 136, 137, 272, 1000])
def test_merkle_build_matches_oracle(N, L):
    bc = _bc()
    vals = [synth.synth_bytes(1, N * 1000 + L * 7 + i, L) for i in range(N)]
    t = bc.MerkleTree.from_vec(vals)
    r = merkle.MerkleTree.from_vec(vals)
    assert t.root_hash() == r.root_hash
    assert t.levels() == r.levels


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 7, 16, 64, 100, 256])
def test_proof_validate_matches_oracle(N):
    bc = _bc()
    L = 150
    vals = [synth.synth_bytes(1, N * 31 + i, L) for i in range(N)]
    r = merkle.MerkleTree.from_vec(vals)
    proofs = []
    for i in range(N):
        p = r.proof(i)
        proofs.append(bc.Proof(p.value, p.index, list(p.digests), p.root_hash))
    # negatives: flipped value byte, wrong index, missing / extra digest, wrong root
    bad = []
    for i in range(min(N, 4)):
        p = r.proof(i)
        v = bytearray(p.value)
        v[i % L] ^= 1
        bad.append(bc.Proof(bytes(v), p.index, list(p.digests), p.root_hash))
        bad.append(bc.Proof(p.value, (p.index + 1) % N, list(p.digests), p.root_hash))
        bad.append(bc.Proof(p.value, p.index, list(p.digests)[:-1], p.root_hash))
        bad.append(bc.Proof(p.value, p.index, list(p.digests) + [b"\x00" * 32], p.root_hash))
        bad.append(bc.Proof(p.value, p.index, list(p.digests), b"\x01" * 32))
    allp = proofs + bad
    ok = bc.validate_proofs(allp, N)
    ref = [merkle.Proof(p.value, p.index, list(p.digests), p.root_hash).validate(N) for p in allp]
    assert ok.tolist() == [int(x) for x in ref]
    assert all(ok[:N])


@pytest.mark.parametrize("N", [1, 3, 4, 16, 64, 128])
def test_decode_from_shards_matches_oracle(N):
    bc = _bc()
    data, parity = bc.shard_counts(N)
    for trial, P in enumerate([0, 3, 100, 5000]):
        payload = synth.payload(N * 10 + trial, P)
        shards, tree = bc.send_shards(payload, N)
        mask = synth.erasure_mask(N * 10 + trial, N, parity)
        leaves = [shards[i].copy() if mask[i] else None for i in range(N)]
        ref_leaves = [l.copy() if l is not None else None for l in leaves]
        out = bc.decode_from_shards(leaves, bc.Coding(data, parity), data, tree.root_hash())
        ref = orbc.decode_from_shards(ref_leaves, N, tree.root_hash())
        assert out == ref == payload
        # too few shards -> None
        if parity:
            m2 = synth.erasure_mask(N * 10 + trial + 1, N, parity + 1)
            l2 = [shards[i].copy() if m2[i] else None for i in range(N)]
            assert bc.decode_from_shards(l2, bc.Coding(data, parity), data, tree.root_hash()) is None
        # wrong root -> None (faulty proposer)
        l3 = [shards[i].copy() if mask[i] else None for i in range(N)]
        assert bc.decode_from_shards(l3, bc.Coding(data, parity), data, b"\x42" * 32) is None


def test_decode_corrupted_present_shard_is_none():
    bc = _bc()
    N = 16
    data, parity = bc.shard_counts(N)
    payload = synth.payload(5, 3000)
    shards, tree = bc.send_shards(payload, N)
    leaves = [shards[i].copy() for i in range(N)]
    leaves[2] = None
    leaves[9][7] ^= 0x10  # corrupt a used shard -> rebuilt tree root differs
    ref = orbc.decode_from_shards([l.copy() if l is not None else None for l in leaves], N, tree.root_hash())
    out = bc.decode_from_shards(leaves, bc.Coding(data, parity), data, tree.root_hash())
    assert out is None and ref is None


def test_decode_length_prefix_truncation():
    """glue_shards takes `len` bytes and silently truncates when the value is
    shorter; a forged length prefix with a matching root must behave the same."""
    bc = _bc()
    N = 4
    data, parity = bc.shard_counts(N)
    L = 10
    sh = np.zeros((N, L), np.uint8)
    sh[:data] = np.frombuffer(synth.synth_bytes(1, 3, data * L), np.uint8).reshape(data, L)
    sh[0, :4] = [0, 0, 1, 0]  # claims 256 bytes, only 16 available
    corc.rs_encode(data, parity, sh)
    root = merkle.MerkleTree.from_vec([bytes(r) for r in sh]).root_hash
    leaves = [sh[i].copy() for i in range(N)]
    leaves[1] = None
    out = bc.decode_from_shards(leaves, bc.Coding(data, parity), data, root)
    ref = orbc.decode_from_shards([sh[i].copy() if i != 1 else None for i in range(N)], N, root)
    assert out == ref and len(out) == data * L - 4


# ------------------------------------------------------------------ device-resident batches (BASELINE sizes)
def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _device_batch(N, P, n, first=0):
    torch = _torch()
    bc = _bc()
    from hydrabadger_amd import _lib
    L = _lib.shard_len(N, P)
    S = (L + 15) // 16 * 16
    PS = max(16, (P + 15) // 16 * 16)
    dev = torch.device("cuda:0")
    pay = torch.zeros((n, PS), dtype=torch.uint8, device=dev)
    if P:
        bc.synth_bytes(synth.TAG_PAYLOAD, first, P, pay, device=True)
    plen = torch.full((n,), P, dtype=torch.int64, device=dev)
    shards = torch.empty((n, N, S), dtype=torch.uint8, device=dev)
    levels = torch.empty((n, _lib.merkle_nodes(N), 32), dtype=torch.uint8, device=dev)
    bc.rbc_encode_merkle_batch(N, pay, plen, L, shards, levels, device=True)
    torch.cuda.synchronize()
    return pay, shards, levels, L, S


def test_device_synth_matches_oracle():
    torch = _torch()
    bc = _bc()
    out = torch.zeros((3, 64), dtype=torch.uint8, device="cuda:0")
    bc.synth_bytes(1, 40, 61, out, device=True)
    got = out.cpu().numpy()
    for k in range(3):
        assert got[k, :61].tobytes() == synth.synth_bytes(1, 40 + k, 61)


@pytest.mark.parametrize("N,P,n", [(16, 65536, 24), (64, 1 << 20, 6), (128, 1 << 20, 3), (4, 230, 100),
                                   # (D, Q) without a compile-time encoder: pack_rows + rs_code_generic, n > 1
                                   (5, 333, 40), (7, 1000, 9), (100, 5000, 3), (3, 50, 7)])
def test_device_batch_encode_matches_oracle(N, P, n):
    pay, shards, levels, L, S = _device_batch(N, P, n, first=11)
    sh = shards.cpu().numpy()
    lv = levels.cpu().numpy()
    for k in [0, n // 2, n - 1]:
        payload = np.frombuffer(synth.payload(11 + k, P), np.uint8).copy()
        rs, rl = corc.rbc_encode_merkle(N, payload)
        assert np.array_equal(sh[k, :, :L], rs), k
        assert np.array_equal(lv[k], rl), k


@pytest.mark.parametrize("N,P,n", [(64, 1 << 20, 8), (16, 65536, 32)])
def test_device_roundtrip_erase_decode(N, P, n):
    """Size-independent property at BASELINE sizes: encode -> erase exactly 2f
    shards (seeded Fisher-Yates) -> decode == payload, every instance."""
    torch = _torch()
    bc = _bc()
    pay, shards, levels, L, S = _device_batch(N, P, n, first=500)
    data, parity = bc.shard_counts(N)
    nodes = levels.shape[1]
    present = torch.tensor([synth.erasure_mask(500 + k, N, parity) for k in range(n)], dtype=torch.uint8,
                           device="cuda:0")
    dmg = shards.clone()
    dmg[present == 0] = 0x5A
    roots = levels[:, nodes - 1, :].contiguous()
    OS = (data * L + 15) // 16 * 16
    out = torch.zeros((n, OS), dtype=torch.uint8, device="cuda:0")
    plen = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    bc.rbc_decode_batch(N, L, dmg, present, roots, out, plen, st, device=True)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [1] * n
    assert plen.cpu().tolist() == [P] * n
    assert torch.equal(out[:, :P], pay[:, :P])
    assert torch.equal(dmg[:, :, :L], shards[:, :, :L])
    # flip the expected root of one instance -> None for that one only
    roots2 = roots.clone()
    roots2[1, 0] ^= 1
    dmg2 = shards.clone()
    bc.rbc_decode_batch(N, L, dmg2, present, roots2, out, plen, st, device=True)
    torch.cuda.synchronize()
    s = st.cpu().tolist()
    assert s[1] == 0 and all(v == 1 for i, v in enumerate(s) if i != 1)


def test_device_batch_mixed_payload_lengths():
    """Per-instance payload lengths that share one shard length L (the batch
    contract): exercises the encoder's interior/edge block split at every
    tail position (last-row padding boundary moves with P)."""
    torch = _torch()
    bc = _bc()
    from hydrabadger_amd import _lib
    N = 64
    D, _ = bc.shard_counts(N)
    P0 = 1 << 20
    L = _lib.shard_len(N, P0)
    lens = [D * L - 4, D * L - 5, D * (L - 1) - 3, P0, P0 - 1, P0 - 9, D * (L - 1) - 2]
    assert all(_lib.shard_len(N, p) == L for p in lens)
    n = len(lens)
    S = (L + 15) // 16 * 16
    dev = torch.device("cuda:0")
    PS = (max(lens) + 15) // 16 * 16
    pays = [np.frombuffer(synth.payload(1300 + k, p), np.uint8) for k, p in enumerate(lens)]
    host = np.zeros((n, PS), np.uint8)
    for k, p in enumerate(pays):
        host[k, :len(p)] = p
    pay = torch.from_numpy(host).to(dev)
    plen = torch.tensor(lens, dtype=torch.int64, device=dev)
    shards = torch.empty((n, N, S), dtype=torch.uint8, device=dev)
    levels = torch.empty((n, _lib.merkle_nodes(N), 32), dtype=torch.uint8, device=dev)
    bc.rbc_encode_merkle_batch(N, pay, plen, L, shards, levels, device=True)
    torch.cuda.synchronize()
    sh = shards.cpu().numpy()
    lv = levels.cpu().numpy()
    for k in range(n):
        rs, rl = corc.rbc_encode_merkle(N, pays[k].copy())
        assert np.array_equal(sh[k, :, :L], rs), k
        assert np.array_equal(lv[k], rl), k


@pytest.mark.parametrize("N,P,n", [(64, 1 << 20, 5), (16, 65536, 21), (128, 1 << 20, 3), (4, 230, 70), (64, 5000, 9)])
def test_fused_schedule_matches_two_launch_schedule(N, P, n):
    """hbg_test_set_rbc_fused: the single-launch rbc_encode_merkle kernel
    (encode pass + SHA3 leaves + tree) writes the same shards
    and levels as rs_encode_const -> merkle_build, and both match the oracle
    on sampled instances (mixed payload lengths that share L included)."""
    torch = _torch()
    bc = _bc()
    from hydrabadger_amd import _lib
    L = _lib.shard_len(N, P)
    D, _ = bc.shard_counts(N)
    lens = [P if k % 3 else D * L - 4 - (k % min(4, D)) for k in range(n)]
    assert all(_lib.shard_len(N, p) == L for p in lens)
    S = (L + 15) // 16 * 16
    PS = (max(lens) + 15) // 16 * 16
    dev = torch.device("cuda:0")
    pays = [np.frombuffer(synth.payload(2100 + k, p), np.uint8) for k, p in enumerate(lens)]
    host = np.zeros((n, PS), np.uint8)
    for k, p in enumerate(pays):
        host[k, :len(p)] = p
    pay = torch.from_numpy(host).to(dev)
    plen = torch.tensor(lens, dtype=torch.int64, device=dev)
    out = []
    ctx = _lib.Context(0)
    try:
        for fused in (0, 1):
            _lib.check(_lib.lib().hbg_test_set_rbc_fused(ctx.h, fused))
            shards = torch.full((n, N, S), 0xA5, dtype=torch.uint8, device=dev)
            levels = torch.full((n, _lib.merkle_nodes(N), 32), 0x5A, dtype=torch.uint8, device=dev)
            bc.rbc_encode_merkle_batch(N, pay, plen, L, shards, levels, ctx=ctx, device=True)
            torch.cuda.synchronize()
            out.append((shards[:, :, :L].cpu().numpy(), levels.cpu().numpy()))
    finally:
        ctx.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    for k in (0, n // 2, n - 1):
        rs, rl = corc.rbc_encode_merkle(N, pays[k].copy())
        assert np.array_equal(out[1][0][k], rs), k
        assert np.array_equal(out[1][1][k], rl), k


@pytest.mark.parametrize("N,L,n", [(16, 10924, 10000), (16, 10924, 21), (5, 137, 700), (64, 16384, 7),
                                   (128, 135, 300), (100, 1000, 77), (1, 7, 50), (2, 272, 33), (7, 0, 9),
                                   (16, 136, 4100), (128, 8, 1000)])
def test_merkle_pairs_schedule_matches(N, L, n):
    """hbg_test_set_merkle_pairs: merkle_build hashing every leaf on a lane pair
    (1), on one lane (0) and the default split (-1: lane pairs for a partial
    last block generation — configs[1]'s 10,000 x 16 leaves included) write
    identical levels, and they match the oracle's tree on sampled instances
    (block-boundary lengths: 0, 7, 8, 135, 136, 137, 272)."""
    torch = _torch()
    from hydrabadger_amd import _lib
    S = max(16, (L + 15) // 16 * 16)
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(N * 131 + L * 7 + n)
    shards = torch.randint(0, 256, (n, N, S), dtype=torch.uint8, generator=g).to(dev)
    nodes = _lib.merkle_nodes(N)
    out = []
    ctx = _lib.Context(0)
    try:
        for mode in (0, 1, -1):
            _lib.check(_lib.lib().hbg_test_set_merkle_pairs(ctx.h, mode))
            levels = torch.full((n, nodes, 32), 0x5A, dtype=torch.uint8, device=dev)
            _lib.check(_lib.lib().hbg_merkle_build(ctx.h, N, L, shards.data_ptr(), S, levels.data_ptr(), n,
                                                   _lib.HBG_DEVICE))
            torch.cuda.synchronize()
            out.append(levels.cpu().numpy())
        assert _lib.lib().hbg_test_set_merkle_pairs(ctx.h, 2) == _lib.HBG_E_ARG
    finally:
        ctx.close()
    assert np.array_equal(out[0], out[1]) and np.array_equal(out[0], out[2])
    host = shards.cpu().numpy()
    for k in sorted({0, n // 2, n - 1}):
        ref = merkle.MerkleTree.from_vec([host[k, i, :L].tobytes() for i in range(N)])
        assert [out[1][k, j].tobytes() for j in range(nodes)] == ref.flat_levels(), k


@pytest.mark.parametrize("D,Q", [(2, 2), (6, 10), (22, 42), (44, 84)])
@pytest.mark.parametrize("L", [1, 5, 257, 4099])
def test_reconstruct_split_schedule_matches_one_pass(D, Q, L):
    """hbg_test_set_rs_split: missing data rows by the run-time coder, then the
    missing parity rows by the constant encoder (rse's own order) — the same
    shards as the one-pass coder and the oracle, for erasure patterns with no
    missing data row, no missing parity row, exactly 2f missing, too few
    present, and a corrupted present parity row past the first D (kept as
    received, not re-encoded)."""
    bc = _bc()
    from hydrabadger_amd import _lib
    N, n = D + Q, 8
    data = np.frombuffer(synth.synth_bytes(synth.TAG_PAYLOAD, N * 17 + L, n * N * L), np.uint8).reshape(n, N, L).copy()
    for k in range(n):
        corc.rs_encode(D, Q, data[k])
    present = np.ones((n, N), np.uint8)
    present[1, D:] = 0                                        # parity only missing
    present[2, :min(D, Q)] = 0                                # data only missing
    for k in (3, 4, 5):
        present[k] = synth.erasure_mask(77 * D + k, N, Q)     # exactly 2f missing
    present[6] = synth.erasure_mask(91 * D, N, Q + 1)         # too few present
    present[7] = synth.erasure_mask(93 * D, N, Q - 1)
    last = int(np.flatnonzero(present[7])[-1])
    assert last >= D
    data[7, last, 0] ^= 0xFF                                  # corrupted, not among the first D present
    outs = []
    ctx = _lib.Context(0)
    try:
        for split in (0, 1):
            _lib.check(_lib.lib().hbg_test_set_rs_split(ctx.h, split))
            dmg = data.copy()
            dmg[present == 0] = 0xEE
            st = bc.Coding(D, Q, ctx=ctx).reconstruct_batch(dmg, present)
            outs.append((dmg, st))
    finally:
        ctx.close()
    assert np.array_equal(outs[0][1], outs[1][1])
    for k in range(n):
        if present[k].sum() < D:
            assert outs[1][1][k] == -14
            continue
        assert outs[1][1][k] == 0
        ref = data[k].copy()
        ref[present[k] == 0] = 0
        assert corc.rs_reconstruct(D, Q, ref, present[k]) == 0
        assert np.array_equal(outs[0][0][k], ref), (k, "one pass")
        assert np.array_equal(outs[1][0][k], ref), (k, "split")


@pytest.mark.parametrize("N,P,n", [(64, 1 << 20, 6), (16, 65536, 24), (128, 1 << 20, 3)])
def test_decode_split_schedule_matches_one_pass(N, P, n):
    """Decode (reconstruct + tree + root check + glue) at BASELINE sizes with
    both reconstruct schedules: the same payloads, statuses and rebuilt shards."""
    torch = _torch()
    bc = _bc()
    from hydrabadger_amd import _lib
    pay, shards, levels, L, S = _device_batch(N, P, n, first=700)
    data, parity = bc.shard_counts(N)
    nodes = levels.shape[1]
    present = torch.tensor([synth.erasure_mask(700 + k, N, parity) for k in range(n)], dtype=torch.uint8,
                           device="cuda:0")
    roots = levels[:, nodes - 1, :].contiguous()
    OS = (data * L + 15) // 16 * 16
    res = []
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        for split in (0, 1):
            _lib.check(_lib.lib().hbg_test_set_rs_split(ctx.h, split))
            dmg = shards.clone()
            dmg[present == 0] = 0x5A
            out = torch.zeros((n, OS), dtype=torch.uint8, device="cuda:0")
            plen = torch.zeros(n, dtype=torch.int64, device="cuda:0")
            st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
            bc.rbc_decode_batch(N, L, dmg, present, roots, out, plen, st, ctx=ctx, device=True)
            torch.cuda.synchronize()
            res.append((dmg, out, plen, st))
    finally:
        ctx.close()
    for dmg, out, plen, st in res:
        assert st.cpu().tolist() == [1] * n
        assert plen.cpu().tolist() == [P] * n
        assert torch.equal(out[:, :P], pay[:, :P])
        assert torch.equal(dmg[:, :, :L], shards[:, :, :L])


def test_batch_larger_than_one_grid_is_an_argument_error():
    """A device-mode batch whose grid would not fit one dispatch (2^32 work-
    items) is refused with HBG_E_ARG before anything is launched, instead of
    running on a truncated grid; the context stays usable."""
    torch = _torch()
    from hydrabadger_amd import _lib
    out = torch.zeros((4, 16), dtype=torch.uint8, device="cuda:0")
    ctx = _lib.Context(0)
    try:
        rc = _lib.lib().hbg_synth_bytes(ctx.h, 1, 0, 8, _lib.ptr(out), 16, 1 << 40, _lib.HBG_DEVICE)
        assert rc == _lib.HBG_E_ARG
        rc = _lib.lib().hbg_synth_bytes(ctx.h, 1, 0, 8, _lib.ptr(out), 16, 4, _lib.HBG_DEVICE)
        assert rc == _lib.HBG_OK
        torch.cuda.synchronize()
        assert bool((out[:, :8] != 0).any())
    finally:
        ctx.close()


@pytest.mark.parametrize("P,n", [(1 << 20, 10), (5000, 10), (0, 10), (47, 10)])
def test_fused_decode_matches_three_launch_decode(P, n):
    """hbg_test_set_rbc_decode_fused: the single-launch rbc_decode_merkle
    (reconstruct + Merkle rebuild at N = 64) gives the same rebuilt shards,
    statuses, lengths and payloads as rs_plan -> coders -> merkle_build, and
    the oracle's decode, for: exactly 2f erased, only parity rows erased, every
    data row erased, nothing erased, too few present, a wrong root, and a
    corrupted present row past the first D (kept as received: None)."""
    torch = _torch()
    bc = _bc()
    from hydrabadger_amd import _lib
    N = 64
    pay, shards, levels, L, S = _device_batch(N, P, n, first=900)
    data, parity = bc.shard_counts(N)
    nodes = levels.shape[1]
    pm = np.stack([synth.erasure_mask(900 + k, N, parity) for k in range(n)]).astype(np.uint8)
    pm[1] = 1
    pm[1, data:] = 0                                # only parity rows erased (42)
    pm[2] = 1
    pm[2, :data] = 0                                # every data row erased (22)
    pm[3] = 1                                       # nothing erased
    pm[4] = synth.erasure_mask(904, N, parity + 1)  # too few present -> None
    pm[6] = synth.erasure_mask(906, N, parity - 5)
    last = int(np.flatnonzero(pm[6])[-1])
    present = torch.from_numpy(pm).to("cuda:0")
    roots = levels[:, nodes - 1, :].contiguous()
    roots[5, 3] ^= 0x40                             # wrong root -> None
    base = shards.clone()
    base[6, last, 0] ^= 0xFF                        # corrupted row past the first D: kept, root differs
    OS = (data * L + 15) // 16 * 16
    res = []
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        for fused in (0, 1):
            _lib.check(_lib.lib().hbg_test_set_rbc_decode_fused(ctx.h, fused))
            dmg = base.clone()
            dmg[present == 0] = 0x5A
            out = torch.zeros((n, OS), dtype=torch.uint8, device="cuda:0")
            plen = torch.zeros(n, dtype=torch.int64, device="cuda:0")
            st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
            bc.rbc_decode_batch(N, L, dmg, present, roots, out, plen, st, ctx=ctx, device=True)
            torch.cuda.synchronize()
            res.append((dmg.cpu().numpy(), out.cpu().numpy(), plen.cpu().tolist(), st.cpu().tolist()))
    finally:
        ctx.close()
    (d0, o0, l0, s0), (d1, o1, l1, s1) = res
    assert s0 == s1 and l0 == l1
    assert s1 == [1, 1, 1, 1, 0, 0, 0] + [1] * (n - 7)
    ok = [k for k in range(n) if s1[k] == 1]
    assert np.array_equal(d0[ok, :, :L], d1[ok, :, :L])     # rebuilt rows (rse: present rows as received)
    for k in ok:
        assert np.array_equal(o0[k, :l1[k]], o1[k, :l1[k]])
        assert o1[k, :P].tobytes() == synth.payload(900 + k, P), k
        assert np.array_equal(d1[k, :, :L], shards[k, :, :L].cpu().numpy()), k
    # the oracle's decode_from_shards (C restatement) on a sampled instance of each kind
    host = base.cpu().numpy()
    for k in (0, 2, 6):
        sh = np.ascontiguousarray(host[k, :, :L]).copy()
        ref = corc.rbc_decode(N, L, sh, pm[k].copy(), roots[k].cpu().numpy().tobytes())
        assert (ref is None) == (s1[k] == 0), k
        if ref is not None:
            assert o1[k, :len(ref)].tobytes() == ref, k


def test_fused_decode_many_erasure_patterns():
    """The fused decoder over 1,024 instances with independent random 2f
    erasures (every count of missing data rows the distribution reaches, so
    every group of the run-time coder runs with padding rows in it): each
    payload comes back and every rebuilt shard row equals the encoder's."""
    torch = _torch()
    bc = _bc()
    from hydrabadger_amd import _lib
    N, P, n = 64, 16384 + 5, 1024
    pay, shards, levels, L, S = _device_batch(N, P, n, first=3000)
    data, parity = bc.shard_counts(N)
    nodes = levels.shape[1]
    pm = np.stack([synth.erasure_mask(3000 + k, N, parity) for k in range(n)]).astype(np.uint8)
    missing_data = (pm[:, :data] == 0).sum(1)
    assert missing_data.min() <= 10 and missing_data.max() >= 19
    present = torch.from_numpy(pm).to("cuda:0")
    roots = levels[:, nodes - 1, :].contiguous()
    OS = (data * L + 15) // 16 * 16
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        _lib.check(_lib.lib().hbg_test_set_rbc_decode_fused(ctx.h, 1))
        dmg = shards.clone()
        dmg[present == 0] = 0x5A
        out = torch.zeros((n, OS), dtype=torch.uint8, device="cuda:0")
        plen = torch.zeros(n, dtype=torch.int64, device="cuda:0")
        st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
        bc.rbc_decode_batch(N, L, dmg, present, roots, out, plen, st, ctx=ctx, device=True)
        torch.cuda.synchronize()
    finally:
        ctx.close()
    assert st.cpu().tolist() == [1] * n
    assert plen.cpu().tolist() == [P] * n
    assert torch.equal(out[:, :P], pay[:, :P])
    assert torch.equal(dmg[:, :, :L], shards[:, :, :L])
