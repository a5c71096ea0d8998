"""GPU parity tests for SURVEY.md §8(f1) and (f2) through the C ABI:
PublicKey::encrypt_with_rng (r explicit), SecretKeyShare::decrypt_share_no_verify,
SecretKey::sign and PublicKey::verify (hydrabadger wire messages,
src/lib.rs:405-416, :434) — against the committed fixture
(tests/golden/bls_ops.json) and the oracle, plus an end-to-end
encrypt -> shares -> verify -> combine round trip entirely on the device."""
from __future__ import annotations

import json
import os
import random

import numpy as np
import pytest

from oracle import bls12_381 as B
from oracle import tcrypto as T
from tests.tdec_fixtures import scenario

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["latency-build", "throughput-build"], autouse=True)
def _bls_build(request):
    """Every test here runs on both builds of the BLS12-381 kernels (same
    results; hbgpu_testing.h hbg_test_set_latency_lanes)."""
    from hydrabadger_amd import _lib
    prev = _lib.lib().hbg_test_set_latency_lanes((1 << 64) - 1 if request.param == "latency-build" else 0)
    yield
    _lib.lib().hbg_test_set_latency_lanes(prev)

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bls_ops.json")))


def _th():
    from hydrabadger_amd import threshold as th
    return th


def _le(h: str) -> int:
    return int.from_bytes(bytes.fromhex(h), "little")


def test_sign_matches_fixture():
    th = _th()
    sks = [_le(k) for k in G["sign"]["sk"]]
    items = [(it["sk"], bytes.fromhex(it["msg"])) for it in G["sign"]["items"]]
    sigs = th.sign_batch(sks, items)
    assert [s.hex() for s in sigs] == [it["sig"] for it in G["sign"]["items"]]
    assert th.SecretKey(sks[0]).sign(b"") == sigs[0]


def test_verify_matches_oracle():
    th = _th()
    pks = [bytes.fromhex(p) for p in G["sign"]["pk"]]
    items, expect = [], []
    for it in G["sign"]["items"]:
        m, sig = bytes.fromhex(it["msg"]), bytes.fromhex(it["sig"])
        items += [(it["sk"], m, sig), (it["sk"], m + b"!", sig), (1 - it["sk"], m, sig)]
        expect += [1, 0, 0]
    sig0 = bytearray(bytes.fromhex(G["sign"]["items"][0]["sig"]))
    sig0[0] &= 0x7F                                              # not compressed-flagged
    items.append((0, b"", bytes(sig0))); expect.append(0)
    inf = bytearray(96); inf[0] = 0xC0                           # identity signature
    items.append((0, b"", bytes(inf))); expect.append(0)
    bad_inf = bytearray(inf); bad_inf[95] = 1                    # malformed identity encoding
    items.append((0, b"", bytes(bad_inf))); expect.append(0)
    tampered = bytearray(bytes.fromhex(G["sign"]["items"][1]["sig"]))
    tampered[60] ^= 1                                            # other x: off-curve or outside G2
    items.append((1, bytes.fromhex(G["sign"]["items"][1]["msg"]), bytes(tampered))); expect.append(0)
    ok = th.verify_sig_batch(pks, items)
    assert ok.tolist() == expect
    assert th.PublicKey(pks[0]).verify(bytes.fromhex(G["sign"]["items"][0]["sig"]), b"")


def test_sign_verify_random_batch():
    """200 messages of random lengths (0..600 B) under 5 keys: device signs,
    device verifies, the oracle checks a sample; every 7th signature is
    swapped to another message (must fail)."""
    th = _th()
    rng = random.Random(7)
    sks = [rng.randrange(1, B.R) for _ in range(5)]
    pks = [B.g1_compress(B.g1_mul(B.G1, k)) for k in sks]
    msgs = [bytes(rng.randrange(256) for _ in range(rng.randrange(600))) for _ in range(200)]
    items = [(k % 5, m) for k, m in enumerate(msgs)]
    sigs = th.sign_batch(sks, items)
    for k in (0, 1, 199):
        assert sigs[k] == B.g2_compress(T.sign(sks[k % 5], msgs[k]))
    vitems = [(k % 5, msgs[k], sigs[(k + 1) % 200] if k % 7 == 3 else sigs[k]) for k in range(200)]
    ok = th.verify_sig_batch(pks, vitems)
    assert ok.tolist() == [0 if k % 7 == 3 else 1 for k in range(200)]


def test_encrypt_and_decrypt_share_match_fixture():
    th = _th()
    e = G["encrypt"]
    cts = th.encrypt_batch(bytes.fromhex(e["pk"]), [bytes.fromhex(it["msg"]) for it in e["items"]],
                           [bytes.fromhex(it["r"]) for it in e["items"]])
    for ct, it in zip(cts, e["items"]):
        assert (ct.U.hex(), ct.V.hex(), ct.W.hex()) == (it["U"], it["V"], it["W"])
    assert th.ct_verify_batch(cts).all()
    shares, st = th.decrypt_shares_batch(cts, [_le(e["sk"])], [(k, 0) for k in range(len(cts))])
    assert st.tolist() == [0] * len(cts)
    assert [s.hex() for s in shares] == [it["share"] for it in e["items"]]
    bad = th.Ciphertext(b"\x00" * 48, b"", cts[0].W)             # undecodable U
    _, st = th.decrypt_shares_batch([bad], [1], [(0, 0)])
    assert st[0] != 0


def test_epoch_round_trip_on_device():
    """One ThresholdDecrypt epoch at N=7 t=2 with everything on the GPU: encrypt
    3 contributions, every node's decrypt_share, verify all shares, combine the
    first t+1 — plaintexts equal the messages; the shares equal the oracle's."""
    th = _th()
    s = scenario()
    ks, t, n = s["ks"], s["t"], len(s["pk_shares"])
    pk = B.g1_compress(ks.public_key())
    rng = random.Random(11)
    msgs = [bytes(rng.randrange(256) for _ in range(L)) for L in (0, 33, 257)]
    rs = [rng.randrange(1, B.R) for _ in msgs]
    cts = th.encrypt_batch(pk, msgs, rs)
    assert th.ct_verify_batch(cts).all()
    sks = [ks.secret_key_share(i) for i in range(n)]
    pairs = [(c, i) for c in range(len(cts)) for i in range(n)]
    shares, st = th.decrypt_shares_batch(cts, sks, pairs)
    assert (st == 0).all()
    ref_ct = T.encrypt(ks.public_key(), msgs[1], rs[1])
    assert shares[1 * n + 3] == B.g1_compress(T.decrypt_share(sks[3], ref_ct))
    pk_shares = [B.g1_compress(p) for p in s["pk_shares"]]
    ok = th.verify_shares_batch(cts, pk_shares, [(shares[c * n + i], c, i) for c, i in pairs])
    assert ok.all()
    pts, st = th.combine_batch(t, cts, [[(i, shares[c * n + i]) for i in range(n)][:t + 1] for c in range(len(cts))])
    assert st.tolist() == [0] * len(cts) and pts == msgs


def test_coin_sign_verify_combine_matches_fixture():
    """§8(f3): signature shares (hbg_bls_sign with key shares), share
    verification (hbg_bls_verify with public key shares) and
    combine_signatures + parity (hbg_sig_combine) reproduce the fixture."""
    th = _th()
    c = G["coin"]
    t = c["t"]
    s = scenario()
    ks, n = s["ks"], len(s["pk_shares"])
    sks = [ks.secret_key_share(i) for i in range(n)]
    pks = [bytes.fromhex(p) for p in c["pk_shares"]]
    for coin in c["coins"]:
        doc = bytes.fromhex(coin["doc"])
        shares = th.sign_batch(sks, [(i, doc) for i in range(n)])
        assert [x.hex() for x in shares] == coin["shares"]
        items = [(i, doc, shares[i]) for i in range(n)] + [(3, doc, shares[4]), (2, doc + b"x", shares[2])]
        assert th.verify_sig_batch(pks, items).tolist() == [1] * n + [0, 0]
        for lo in (0, 1, n - t - 1):
            sig, par = th.combine_signatures(t, [(i, shares[i]) for i in range(lo, lo + t + 1)])
            assert sig.hex() == coin["sig"] and par == coin["parity"]
        with pytest.raises(th.DuplicateEntry):
            th.combine_signatures(t, [(1, shares[1])] * (t + 1))
        assert th.PublicKey(bytes.fromhex(c["pk"])).verify(bytes.fromhex(coin["sig"]), doc)


@pytest.mark.parametrize("t", [0, 3, 21, 31, 42, 63])
def test_coin_combine_arbitrary_points(t):
    """hbg_sig_combine over arbitrary G2 points (interpolation does not need
    valid shares), odd coin count, identity shares, sparse shuffled indices,
    and an undecodable share — against the oracle's interpolate_g2 + parity."""
    th = _th()
    from hydrabadger_amd import _lib
    rng = random.Random(2000 + t)
    coins, expect = [], []
    for k in range(3):
        ids = rng.sample(range(100), t + 1)
        pts = [None if (k == 1 and j == 0) else B.g2_mul(B.G2, rng.randrange(1, B.R)) for j in range(t + 1)]
        items = [(i, B.g2_compress(p)) for i, p in zip(ids, pts)]
        if k == 2:
            junk = bytearray(items[-1][1]); junk[0] &= 0x7F
            items[-1] = (items[-1][0], bytes(junk))
            expect.append(None)
        else:
            sig = T.combine_signatures(t, list(zip(ids, pts)))
            expect.append((B.g2_compress(sig), T.sig_parity(sig)))
        coins.append(items)
    sigs, par, st = th.sig_combine_batch(t, coins)
    for k, e in enumerate(expect):
        if e is None:
            assert st[k] == _lib.HBG_E_INVALID_POINT
        else:
            assert st[k] == 0 and sigs[k] == e[0] and bool(par[k]) == e[1], k


@pytest.mark.parametrize("seed,bad_rate", [(1, 0.0), (2, 0.03), (3, 0.4)])
def test_coin_share_verify_batched(seed, bad_rate):
    """§8(f3) hbg_sig_verify_shares (PublicKeyShare::verify of coin shares,
    hash_g2 once per document, weighted batches + group testing) gives the
    same bits as the per-share hbg_bls_verify and as the expected validity, in
    every schedule (batched, batched + fixed-base key tables, per share):
    batches crossing 64, ragged documents, wrong-key claims, shares of another
    document, undecodable / tampered / identity shares, an undecodable key."""
    th = _th()
    from hydrabadger_amd import _lib
    s = scenario()
    ks, n = s["ks"], len(s["pk_shares"])
    sks = [ks.secret_key_share(i) for i in range(n)]
    pks = [B.g1_compress(p) for p in s["pk_shares"]]
    junk_pk = bytearray(pks[0]); junk_pk[0] &= 0x7F
    pks.append(bytes(junk_pk))                                   # key index n: undecodable
    rng = random.Random(seed)
    docs = [bytes(rng.randrange(256) for _ in range(L)) for L in (0, 17, 64, 200, 9)]
    signed = th.sign_batch(sks, [(i, d) for d in docs for i in range(n)])
    good = {(d, i): signed[d * n + i] for d in range(len(docs)) for i in range(n)}
    items, expect = [], []
    for d, count in enumerate((150, 64, 5, 65, 1)):
        for q in range(count):
            i = rng.randrange(n)
            r = rng.random()
            if r < bad_rate / 3:
                items.append((d, (i + 1) % n, good[(d, i)])); expect.append(0)          # wrong key
            elif r < 2 * bad_rate / 3:
                items.append((d, i, good[((d + 1) % len(docs), i)])); expect.append(0)  # another doc's share
            elif r < bad_rate:
                t = bytearray(good[(d, i)]); t[40] ^= 1                                 # tampered x
                items.append((d, i, bytes(t))); expect.append(0)
            else:
                items.append((d, i, good[(d, i)])); expect.append(1)
    junk = bytearray(good[(0, 1)]); junk[0] &= 0x7F
    inf = bytearray(96); inf[0] = 0xC0
    items += [(0, 1, bytes(junk)), (3, 2, bytes(inf)), (1, n, good[(1, 0)])]
    expect += [0, 0, 0]
    order = list(range(len(items)))
    rng.shuffle(order)
    items = [items[k] for k in order]
    expect = np.array([expect[k] for k in order], np.uint8)
    ref = th.verify_sig_batch(pks, [(p, docs[d], sg) for d, p, sg in items])
    assert np.array_equal(ref, expect)
    ctx = _lib.Context(0)
    try:
        outs = []
        for mode in (1, 2, 3, 0):
            _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, mode))
            outs.append(th.verify_sig_shares_batch(pks, docs, items, ctx))
    finally:
        ctx.close()
    for o in outs:
        assert np.array_equal(o, expect)


def test_coin_share_cancelling_pair_rejected():
    """§8(f3) coin shares: sig_a + D and sig_b - D (G2) for two signers of one
    document — an unweighted batch sum would pass — both 0 on every schedule
    and under HBG_VERIFY_PER_SHARE; the other shares 1."""
    th = _th()
    from hydrabadger_amd import _lib
    s = scenario()
    ks, n = s["ks"], len(s["pk_shares"])
    sks = [ks.secret_key_share(i) for i in range(n)]
    pks = [B.g1_compress(p) for p in s["pk_shares"]]
    docs = [b"coin nonce 0", b"coin nonce 1"]
    signed = th.sign_batch(sks, [(i, d) for d in docs for i in range(n)])
    D = B.g2_mul(B.G2, 987654321)
    items, expect = [], []
    for d in range(len(docs)):
        for rep in range(10):          # 70 shares a document: batches of 64 + 6
            for i in range(n):
                sg = signed[d * n + i]
                if d == 0 and rep == 2 and i in (1, 4):
                    p = B.g2_decompress(sg)
                    sg = B.g2_compress(B.g2_add(p, D if i == 1 else B.g2_neg(D)))
                    expect.append(0)
                else:
                    expect.append(1)
                items.append((d, i, sg))
    expect = np.array(expect, np.uint8)
    ctx = _lib.Context(0)
    try:
        for mode in (1, 2, 3, 0):
            _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, mode))
            assert np.array_equal(th.verify_sig_shares_batch(pks, docs, items, ctx), expect), mode
        ctx.set_share_verify(_lib.HBG_VERIFY_PER_SHARE)
        assert np.array_equal(th.verify_sig_shares_batch(pks, docs, items, ctx), expect)
    finally:
        ctx.close()


def test_long_contributions_encrypt_verify_decrypt():
    """HoneyBadger threshold-encrypts the whole serialised contribution, so V
    is as long as a proposal (BASELINE.json configs[4]: 1 MiB).  encrypt_with_rng
    (U, V, W), Ciphertext::verify and PublicKeySet::decrypt for lengths around
    the SHA3 block (136 B), the hash_g1_g2 cut (64 B) and up to 1 MiB, packed at
    unaligned offsets: V and W equal the oracle's (vectorised keystream for V,
    hashlib SHA3 inside hash_g1_g2), every ciphertext verifies (C oracle), and
    the t+1-share combination returns the message."""
    import hashlib

    from oracle import chacha, corb
    th = _th()
    s = scenario()
    ks, t, n = s["ks"], s["t"], len(s["pk_shares"])
    pkp = ks.public_key()
    pk = B.g1_compress(pkp)
    rng = random.Random(23)
    lens = [0, 1, 63, 64, 65, 135, 136, 137, 271, 5003, 70001, 1 << 20]
    msgs = [bytes(rng.getrandbits(8) for _ in range(L)) if L < 100000 else
            np.random.default_rng(5).integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    rs = [rng.randrange(1, B.R) for _ in msgs]
    cts = th.encrypt_batch(pk, msgs, rs)
    for k in (0, 2, 3, 4, 6, 7, 9, 11):
        r, L = rs[k], lens[k]
        seed = hashlib.sha3_256(B.g1_compress(B.g1_mul(pkp, r))).digest()
        v = bytes(a ^ b for a, b in zip(msgs[k], chacha.keystream_u8(seed, L))) if L < 100000 else \
            (np.frombuffer(msgs[k], np.uint8) ^ np.frombuffer(chacha.keystream_u8(seed, L), np.uint8)).tobytes()
        assert cts[k].V == v, L
        u = B.g1_mul(B.G1, r)
        assert cts[k].U == B.g1_compress(u), L
        assert cts[k].W == B.g2_compress(B.g2_mul(T.hash_g1_g2(u, v), r)), L
    assert th.ct_verify_batch(cts).all()
    assert all(corb.ct_verify(c.U, c.V, c.W) for c in cts[-4:])
    sks = [ks.secret_key_share(i) for i in range(n)]
    pairs = [(c, i) for c in range(len(cts)) for i in range(t + 1)]
    shares, st = th.decrypt_shares_batch(cts, sks, pairs)
    assert (st == 0).all()
    pts, st = th.combine_batch(t, cts, [[(i, shares[c * (t + 1) + i]) for i in range(t + 1)] for c in range(len(cts))])
    assert st.tolist() == [0] * len(cts)
    assert pts == msgs
