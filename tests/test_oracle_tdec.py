"""Pins the BLS12-381 / threshold_crypto oracle (CPU) against known answers
(SURVEY.md §8(c)): curve constants and generators, RFC 8439 ChaCha20, the
crate's final-exponentiation chain (= plain exponentiation cubed), pairing
bilinearity / non-degeneracy, and encrypt -> share -> verify -> combine round
trips.  hash_g2 itself is "parity unpinned" (version-dependent)."""
from __future__ import annotations

import json
import os

import pytest

from oracle import bls12_381 as B
from oracle import chacha
from oracle import tcrypto as T
from tests.tdec_fixtures import scenario

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "tdec_golden.json")


def test_constants():
    x = -B.BLS_X
    assert x ** 4 - x ** 2 + 1 == B.R
    assert (x - 1) ** 2 * B.R % 3 == 0 and (x - 1) ** 2 * B.R // 3 + x == B.P
    assert B.g1_on_curve(B.G1) and B.g2_on_curve(B.G2)
    assert B.g1_mul(B.G1, B.R) is None and B.g2_mul(B.G2, B.R) is None
    assert B.g1_compress(B.G1).hex().startswith("97f1d3a73197d794")
    h2 = (x ** 8 - 4 * x ** 7 + 5 * x ** 6 - 4 * x ** 4 + 6 * x ** 3 - 4 * x ** 2 - 4 * x + 13) // 9
    assert h2 == B.G2_COFACTOR


def test_chacha_rfc8439_block():
    w = chacha.block(bytes(range(32)), 1, bytes.fromhex("000000090000004a00000000"))
    assert w[0] == 0xE4E7F110 and w[1] == 0x15593BD1 and w[15] == 0x4E3C50A2


def test_vectorised_keystream_matches_scalar_stream():
    seed = bytes(range(7, 39))
    for n in (0, 1, 15, 16, 17, 333, 1000):
        assert chacha.keystream_u8(seed, n) == chacha.ChaChaRng(seed).u8_stream(n), n


def test_compression_roundtrip():
    for k in (1, 2, 12345):
        p = B.g1_mul(B.G1, k)
        assert B.g1_decompress(B.g1_compress(p)) == p
        q = B.g2_mul(B.G2, k)
        assert B.g2_decompress(B.g2_compress(q)) == q


def test_pairing_bilinear_and_chain():
    e = B.pairing(B.G1, B.G2)
    assert e != B.F12_ONE
    assert B.pairing(B.g1_mul(B.G1, 6), B.g2_mul(B.G2, 7)) == B.f12_pow(e, 42)
    f = B.miller_loop([(B.G1, B.g2_prepare(B.G2))])
    assert B.final_exponentiation(f) == B.f12_pow(B.final_exponentiation_plain(f), 3)
    assert B.f12_pow(e, B.R) == B.F12_ONE


def test_threshold_roundtrip_and_negatives():
    s = scenario()
    t, ct = s["t"], s["cts"][0]
    assert ct.verify()
    h = T.hash_g1_g2(ct.U, ct.V)
    for i, sh in enumerate(s["shares"][0]):
        assert T.verify_decryption_share(s["pk_shares"][i], sh, ct, h)
    bad = B.g1_add(s["shares"][0][1], B.G1)
    assert not T.verify_decryption_share(s["pk_shares"][1], bad, ct, h)
    assert not T.verify_decryption_share(s["pk_shares"][2], s["shares"][0][1], ct, h)  # wrong key
    items = list(enumerate(s["shares"][0]))
    assert T.decrypt(t, items[3:], ct) == s["msgs"][0]
    assert T.decrypt(t, items[:t + 1], ct) == s["msgs"][0]
    with pytest.raises(T.NotEnoughShares):
        T.decrypt(t, items[:t], ct)
    tampered = T.Ciphertext(ct.U, ct.V, B.g2_mul(ct.W, 2))
    assert not tampered.verify()


def test_hash_g2_is_in_g2():
    for m in (b"", b"abc", bytes(100)):
        h = T.hash_g2(m)
        assert B.g2_on_curve(h) and B.g2_mul(h, B.R) is None


def test_golden_tdec_reproduces():
    with open(GOLDEN) as f:
        g = json.load(f)
    for case in g["hash_g2"]:
        assert B.g2_compress(T.hash_g2(bytes.fromhex(case["msg"]))).hex() == case["point"]
    s = scenario(**g["scenario"]["params"])
    sc = g["scenario"]
    assert [B.g1_compress(p).hex() for p in s["pk_shares"]] == sc["pk_shares"]
    for k, ct in enumerate(s["cts"]):
        c = sc["cts"][k]
        assert (B.g1_compress(ct.U).hex(), ct.V.hex(), B.g2_compress(ct.W).hex()) == (c["U"], c["V"], c["W"])
        assert [B.g1_compress(x).hex() for x in s["shares"][k]] == c["shares"]
        assert s["msgs"][k].hex() == c["plaintext"]


# --------------------------------------------------------------------------- C restatement (oracle/c/bls_oracle.c)
def _fixture(name):
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", name)))["scenario"]


@pytest.mark.parametrize("name", ["tdec_golden.json", "tdec_n64.json"])
def test_c_oracle_matches_fixtures(name):
    """The C restatement (bench's TDec cpu_baseline) reproduces the committed
    fixtures: every fixture share verifies, wrong-key / other-ciphertext /
    undecodable shares do not, ciphertexts verify, plaintexts match."""
    from oracle import corb
    g = _fixture(name)
    cts = [(bytes.fromhex(c["U"]), bytes.fromhex(c["V"]), bytes.fromhex(c["W"])) for c in g["cts"]]
    pk = [bytes.fromhex(p) for p in g["pk_shares"]]
    n = len(pk)
    items, expect = [], []
    for c, ct in enumerate(g["cts"]):
        for i in list(range(min(n, 6))) + [n - 1]:
            items.append((bytes.fromhex(ct["shares"][i]), c, i)); expect.append(1)
        items.append((bytes.fromhex(ct["shares"][1]), c, 2)); expect.append(0)            # wrong key
        other = g["cts"][(c + 1) % len(g["cts"])]["shares"][0]
        items.append((bytes.fromhex(other), c, 0)); expect.append(0)                     # another ciphertext's share
    junk = bytearray(bytes.fromhex(g["cts"][0]["shares"][0])); junk[0] &= 0x7F
    items.append((bytes(junk), 0, 0)); expect.append(0)                                   # undecodable
    assert corb.verify_shares(cts, pk, items, threads=4).tolist() == expect
    assert all(corb.ct_verify(*c) for c in cts)
    U, V, W = cts[0]
    assert not corb.ct_verify(U, V + b"x", W)
    t = g["t"]
    pts, st = corb.decrypt_batch(t, cts, [[(i, bytes.fromhex(x)) for i, x in enumerate(c["shares"])] for c in g["cts"]])
    assert st.tolist() == [0] * len(cts)
    assert [p.hex() for p in pts] == [c["plaintext"] for c in g["cts"]]
    # shares in a different order / a different subset interpolate to the same plaintext
    sub = [[(i, bytes.fromhex(c["shares"][i])) for i in reversed(range(n - t - 1, n))] for c in g["cts"]]
    pts2, st2 = corb.decrypt_batch(t, cts, sub)
    assert pts2 == pts and st2.tolist() == [0] * len(cts)
    dup = [[(1, bytes.fromhex(c["shares"][1]))] * (t + 1) for c in g["cts"]]
    _, st3 = corb.decrypt_batch(t, cts, dup)
    assert st3.tolist() == [-21] * len(cts)


def test_c_oracle_matches_python_oracle_on_edge_points():
    """Identity share / identity key / out-of-subgroup share: C and Python
    restatements agree bit for bit (Python oracle on a small scenario)."""
    from oracle import corb
    s = scenario()
    ct = s["cts"][0]
    cts = [(B.g1_compress(ct.U), ct.V, B.g2_compress(ct.W))]
    h = T.hash_g1_g2(ct.U, ct.V)
    pk = [B.g1_compress(p) for p in s["pk_shares"]]
    x = 5
    while B.fq_sqrt((x ** 3 + 4) % B.P) is None:
        x += 1
    bad_sub = bytearray(x.to_bytes(48, "big")); bad_sub[0] |= 0x80
    items = [(B.g1_compress(None), 0, 0), (bytes(bad_sub), 0, 1), (B.g1_compress(s["shares"][0][2]), 0, 2)]
    ref = [int(T.verify_decryption_share(s["pk_shares"][0], None, ct, h)), 0, 1]
    assert corb.verify_shares(cts, pk, items).tolist() == ref


def test_sign_verify_oracle_and_bls_golden():
    """SecretKey::sign / PublicKey::verify restatement and
    the committed f1/f2 fixture (tests/golden/bls_ops.json) reproduce."""
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bls_ops.json")))
    sks = [int.from_bytes(bytes.fromhex(k), "little") for k in g["sign"]["sk"]]
    for it in g["sign"]["items"]:
        m = bytes.fromhex(it["msg"])
        sig = T.sign(sks[it["sk"]], m)
        assert B.g2_compress(sig).hex() == it["sig"]
        pk = B.g1_mul(B.G1, sks[it["sk"]])
        assert T.verify(pk, sig, m)
        assert not T.verify(pk, sig, m + b"!")
        assert not T.verify(B.g1_mul(B.G1, sks[1 - it["sk"]]), sig, m)
    pk = B.g1_decompress(bytes.fromhex(g["encrypt"]["pk"]))
    sk = int.from_bytes(bytes.fromhex(g["encrypt"]["sk"]), "little")
    for it in g["encrypt"]["items"]:
        ct = T.encrypt(pk, bytes.fromhex(it["msg"]), int.from_bytes(bytes.fromhex(it["r"]), "little"))
        assert (B.g1_compress(ct.U).hex(), ct.V.hex(), B.g2_compress(ct.W).hex()) == (it["U"], it["V"], it["W"])
        assert ct.verify()
        assert B.g1_compress(T.decrypt_share(sk, ct)).hex() == it["share"]
        # t = 0 keyset: the single share decrypts
        assert T.decrypt(0, [(0, T.decrypt_share(sk, ct))], ct) == bytes.fromhex(it["msg"])


def test_coin_oracle_fixture():
    """§8(f3) common coin: signature shares interpolate to the master key's
    signature for any t+1 subset; parity recorded in the fixture."""
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bls_ops.json")))["coin"]
    t = g["t"]
    pk = B.g1_decompress(bytes.fromhex(g["pk"]))
    for c in g["coins"]:
        doc = bytes.fromhex(c["doc"])
        shares = [B.g2_decompress(bytes.fromhex(x)) for x in c["shares"]]
        for lo in (0, len(shares) - t - 1):
            sig = T.combine_signatures(t, [(i, shares[i]) for i in range(lo, lo + t + 1)])
            assert B.g2_compress(sig).hex() == c["sig"]
        assert T.sig_parity(B.g2_decompress(bytes.fromhex(c["sig"]))) == c["parity"]
        assert T.verify(pk, B.g2_decompress(bytes.fromhex(c["sig"])), doc)
        pks = [B.g1_decompress(bytes.fromhex(p)) for p in g["pk_shares"]]
        assert T.verify(pks[3], shares[3], doc) and not T.verify(pks[3], shares[4], doc)
