"""GPU parity tests for the ThresholdDecrypt path (family 3), through the C ABI.

Layer by layer against the oracle (oracle/bls12_381.py, oracle/tcrypto.py):
field mul / inverse / Fq2 sqrt, G1 / G2 decompression with subgroup checks,
the crate's Miller loop, final exponentiation and pairing (exact Fq12 values),
hash_g2, then the drop-in surfaces: verify_decryption_share bits (valid,
corrupted, wrong-key, invalid encodings), Ciphertext::verify, and
PublicKeySet::decrypt plaintexts incl. DuplicateEntry.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

from oracle import bls12_381 as B
from oracle import tcrypto as T
from oracle.chacha import ChaChaRng
from tests.tdec_fixtures import from_limbs, limbs, scenario

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["latency-build", "throughput-build"], autouse=True)
def _bls_build(request):
    """Every test here runs on both builds of the BLS12-381 kernels (same
    results; hbgpu_testing.h hbg_test_set_latency_lanes)."""
    from hydrabadger_amd import _lib
    prev = _lib.lib().hbg_test_set_latency_lanes((1 << 64) - 1 if request.param == "latency-build" else 0)
    yield
    _lib.lib().hbg_test_set_latency_lanes(prev)


def _th():
    from hydrabadger_amd import threshold as th
    return th


def _rnd(seed):
    r = random.Random(seed)
    return lambda: r.randrange(B.P)


def test_fp_mul_inv():
    th = _th()
    rnd = _rnd(1)
    vals = [(rnd(), rnd()) for _ in range(200)] + [(0, 5), (B.P - 1, B.P - 1), (1, 1)]
    inp = np.array([limbs(a) + limbs(b) for a, b in vals], np.uint32)
    out = th.test_bls(0, inp, 12)
    for (a, b), o in zip(vals, out):
        assert from_limbs(o) == a * b % B.P
    inv_in = np.array([limbs(a) + [0] * 12 for a, _ in vals if a], np.uint32)
    out = th.test_bls(1, inv_in, 12)
    for row, o in zip(inv_in, out):
        a = from_limbs(row[:12])
        assert from_limbs(o) == pow(a, B.P - 2, B.P)


def test_fp2_sqrt():
    th = _th()
    rnd = _rnd(2)
    xs = [(rnd(), rnd()) for _ in range(40)]
    sq = [B.f2_sqr(x) for x in xs]
    nonsq = []
    while len(nonsq) < 10:
        c = (rnd(), rnd())
        if B.f2_sqrt(c) is None:
            nonsq.append(c)
    vals = sq + nonsq
    out = th.test_bls(2, np.array([limbs(a) + limbs(b) for a, b in vals], np.uint32), 25)
    for i, (v, o) in enumerate(zip(vals, out)):
        if i < len(sq):
            assert o[24] == 1
            r = (from_limbs(o[:12]), from_limbs(o[12:24]))
            assert B.f2_sqr(r) == v
        else:
            assert o[24] == 0


def _g1_words(b: bytes):
    return list(np.frombuffer(b.ljust(48, b"\0"), np.uint32))


def test_g1_decompress_and_subgroup():
    th = _th()
    pts = [B.g1_mul(B.G1, k) for k in (1, 2, 3, 77, 2 ** 200 + 5)]
    encs = [B.g1_compress(p) for p in pts] + [B.g1_compress(None)]
    # on the curve but outside G1
    x = 5
    while B.fq_sqrt((x ** 3 + 4) % B.P) is None:
        x += 1
    y = B.fq_sqrt((x ** 3 + 4) % B.P)
    bad_sub = bytearray(x.to_bytes(48, "big"))
    bad_sub[0] |= 0x80
    not_curve = bytearray((3).to_bytes(48, "big"))
    not_curve[0] |= 0x80
    if B.fq_sqrt((27 + 4) % B.P) is not None:
        not_curve = bytearray((4).to_bytes(48, "big")); not_curve[0] |= 0x80
    no_flag = bytearray(B.g1_compress(pts[0]))
    no_flag[0] &= 0x7F
    encs += [bytes(bad_sub), bytes(not_curve), bytes(no_flag)]
    out = th.test_bls(3, np.array([_g1_words(e) for e in encs], np.uint32), 26)
    for i, p in enumerate(pts):
        assert out[i][24] == 1 and (from_limbs(out[i][:12]), from_limbs(out[i][12:24])) == p
    assert out[len(pts)][24] == 1 and out[len(pts)][25] == 1
    assert [int(o[24]) for o in out[len(pts) + 1:]] == [0, 0, 0]
    assert y is not None


def test_g2_decompress_and_subgroup():
    th = _th()
    pts = [B.g2_mul(B.G2, k) for k in (1, 5, 1234567)]
    encs = [B.g2_compress(p) for p in pts]
    tampered = bytearray(encs[0])
    tampered[50] ^= 1  # different x: almost surely off-curve or outside G2
    encs.append(bytes(tampered))
    out = th.test_bls(4, np.array([list(np.frombuffer(e, np.uint32)) for e in encs], np.uint32), 50)
    for i, p in enumerate(pts):
        assert out[i][48] == 1
        got = ((from_limbs(out[i][0:12]), from_limbs(out[i][12:24])), (from_limbs(out[i][24:36]),
                                                                       from_limbs(out[i][36:48])))
        assert got == p
    try:
        B.g2_decompress(bytes(tampered))
        ref_ok = 1
    except ValueError:
        ref_ok = 0
    assert out[3][48] == ref_ok


def _f12_from_words(o):
    c = [from_limbs(o[12 * i:12 * i + 12]) for i in range(12)]
    return (((c[0], c[1]), (c[2], c[3]), (c[4], c[5])), ((c[6], c[7]), (c[8], c[9]), (c[10], c[11])))


def _pq_words(p, q):
    return limbs(p[0]) + limbs(p[1]) + limbs(q[0][0]) + limbs(q[0][1]) + limbs(q[1][0]) + limbs(q[1][1])


def test_miller_loop_final_exp_pairing_exact():
    th = _th()
    pairs = [(B.G1, B.G2), (B.g1_mul(B.G1, 9), B.g2_mul(B.G2, 11)), (B.g1_mul(B.G1, 2 ** 100 + 3), B.G2)]
    inp = np.array([_pq_words(p, q) for p, q in pairs], np.uint32)
    ml = th.test_bls(7, inp, 144)
    for (p, q), o in zip(pairs, ml):
        assert _f12_from_words(o) == B.miller_loop([(p, B.g2_prepare(q))])
    pe = th.test_bls(5, inp, 144)
    for (p, q), o in zip(pairs, pe):
        assert _f12_from_words(o) == B.pairing(p, q)
    fe = th.test_bls(8, ml, 144)
    for o, m in zip(fe, ml):
        assert _f12_from_words(o) == B.final_exponentiation(_f12_from_words(m))


def test_hash_g2_from_seed():
    th = _th()
    from oracle.merkle import sha3
    seeds = [sha3(bytes([i]) * i) for i in range(6)]
    out = th.test_bls(6, np.array([list(np.frombuffer(s, np.uint32)) for s in seeds], np.uint32), 48)
    for s, o in zip(seeds, out):
        ref = T._rand_g2(ChaChaRng(s))
        got = ((from_limbs(o[0:12]), from_limbs(o[12:24])), (from_limbs(o[24:36]), from_limbs(o[36:48])))
        assert got == ref


def _gpu_cts(th, cts):
    return [th.Ciphertext(B.g1_compress(c.U), c.V, B.g2_compress(c.W)) for c in cts]


def test_verify_shares_matches_oracle():
    th = _th()
    s = scenario()
    n = len(s["pk_shares"])
    cts = _gpu_cts(th, s["cts"])
    pk = [B.g1_compress(p) for p in s["pk_shares"]]
    items, ref = [], []
    for c, ct in enumerate(s["cts"]):
        h = T.hash_g1_g2(ct.U, ct.V)
        for i in range(n):
            items.append((B.g1_compress(s["shares"][c][i]), c, i))
            ref.append(True)
        # corrupted share, wrong key index, identity share, share of another ct
        bad = B.g1_add(s["shares"][c][0], B.G1)
        items.append((B.g1_compress(bad), c, 0))
        ref.append(T.verify_decryption_share(s["pk_shares"][0], bad, ct, h))
        items.append((B.g1_compress(s["shares"][c][1]), c, 2))
        ref.append(False)
        items.append((B.g1_compress(None), c, 3))
        ref.append(T.verify_decryption_share(s["pk_shares"][3], None, ct, h))
        other = (c + 1) % len(s["cts"])
        items.append((B.g1_compress(s["shares"][other][4]), c, 4))
        ref.append(False)
    # invalid encoding
    junk = bytearray(B.g1_compress(s["shares"][0][5]))
    junk[0] &= 0x7F
    items.append((bytes(junk), 0, 5))
    ref.append(False)
    ok = th.verify_shares_batch(cts, pk, items)
    assert ok.tolist() == [int(r) for r in ref]


def test_ct_verify_matches_oracle():
    th = _th()
    s = scenario()
    cts = list(s["cts"])
    tampered = T.Ciphertext(cts[0].U, cts[0].V, B.g2_mul(cts[0].W, 3))
    vt = T.Ciphertext(cts[1].U, bytes([cts[1].V[0] ^ 1]) + cts[1].V[1:], cts[1].W)
    allc = cts + [tampered, vt]
    ok = th.ct_verify_batch(_gpu_cts(th, allc))
    assert ok.tolist() == [int(c.verify()) for c in allc]


def test_combine_matches_oracle():
    th = _th()
    s = scenario()
    t = s["t"]
    cts = _gpu_cts(th, s["cts"])
    pks = th.PublicKeySet(t)
    for c, ct in enumerate(s["cts"]):
        for start in (0, 2, len(s["pk_shares"]) - t - 1):
            items = [(i, B.g1_compress(s["shares"][c][i])) for i in range(start, start + t + 1)]
            got = pks.decrypt(items, cts[c])
            ref = T.decrypt(t, [(i, s["shares"][c][i]) for i in range(start, start + t + 1)], ct)
            assert got == ref == s["msgs"][c]
    with pytest.raises(th.NotEnoughShares):
        pks.decrypt([(0, B.g1_compress(s["shares"][0][0]))], cts[0])
    dup = [(1, B.g1_compress(s["shares"][0][1]))] * (t + 1)
    with pytest.raises(th.DuplicateEntry):
        pks.decrypt(dup, cts[0])


def test_golden_tdec_on_gpu():
    """The committed fixture (tests/golden/tdec_golden.json) verifies and
    decrypts on the device without recomputing anything in Python."""
    import json
    import os
    th = _th()
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tdec_golden.json")))
    sc = g["scenario"]
    cts = [th.Ciphertext(bytes.fromhex(c["U"]), bytes.fromhex(c["V"]), bytes.fromhex(c["W"])) for c in sc["cts"]]
    pk = [bytes.fromhex(p) for p in sc["pk_shares"]]
    items = [(bytes.fromhex(sh), k, i) for k, c in enumerate(sc["cts"]) for i, sh in enumerate(c["shares"])]
    assert th.verify_shares_batch(cts, pk, items).all()
    assert th.ct_verify_batch(cts).all()
    t = sc["t"]
    pts, st = th.combine_batch(t, cts, [[(i, bytes.fromhex(x)) for i, x in enumerate(c["shares"])][:t + 1]
                                        for c in sc["cts"]])
    assert st.tolist() == [0] * len(cts)
    assert [p.hex() for p in pts] == [c["plaintext"] for c in sc["cts"]]


@pytest.mark.parametrize("bad_rate,seed", [(0.0, 1), (0.03, 2), (0.3, 3), (1.0, 4)])
def test_batched_verify_equals_per_share(bad_rate, seed):
    """hbg_tdec_verify_shares' batched schedule (weighted batch sums per
    ciphertext, sub-batches of 8, per-share fallback) returns exactly the bits
    of one pairing check per share — on the N=64 t=21 fixture's 4 ciphertexts
    x 64 shares, replicated to 150 ciphertexts (ragged last batches: 150*64
    shares in shuffled order, so batches cut mid-group), with a seeded fraction
    of shares claimed under the wrong key or corrupted, plus invalid
    encodings and out-of-subgroup / identity shares."""
    import json
    import os
    from hydrabadger_amd import _lib
    th = _th()
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tdec_n64.json")))["scenario"]
    K, n = len(g["cts"]), len(g["pk_shares"])
    n_ct = 150
    cts = [th.Ciphertext(bytes.fromhex(g["cts"][j % K]["U"]), bytes.fromhex(g["cts"][j % K]["V"]),
                         bytes.fromhex(g["cts"][j % K]["W"])) for j in range(n_ct)]
    pk = [bytes.fromhex(p) for p in g["pk_shares"]]
    rng = np.random.default_rng(seed)
    items, expect = [], []
    for j in range(n_ct):
        for i in range(n if j < n_ct - 1 else 37):          # ragged last ciphertext
            sh = bytes.fromhex(g["cts"][j % K]["shares"][i])
            r = rng.random()
            if r < bad_rate / 2:
                items.append((sh, j, (i + 1) % n)); expect.append(0)        # wrong key
            elif r < bad_rate:
                other = bytes.fromhex(g["cts"][(j + 1) % K]["shares"][i])
                items.append((other, j, i)); expect.append(0)              # share of another ct
            else:
                items.append((sh, j, i)); expect.append(1)
    junk = bytearray(items[5][0]); junk[0] &= 0x7F                            # invalid encoding
    items.append((bytes(junk), 3, 5)); expect.append(0)
    items.append((B.g1_compress(B.G1), 7, 9)); expect.append(0)               # valid point, wrong share
    items.append((bytes([0xC0]) + bytes(47), 11, 3)); expect.append(0)          # identity share (in G1, wrong)
    order = rng.permutation(len(items))
    items = [items[k] for k in order]
    expect = np.array([expect[k] for k in order], np.uint8)
    ctx = _lib.Context(0)
    try:
        outs = []
        for mode in (1, 2, 3, 0):
            _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, mode))
            outs.append(th.verify_shares_batch(cts, pk, items, ctx))
    finally:
        ctx.close()
    for o in outs:  # auto, batched + tables, batched, per share
        assert np.array_equal(o, expect)


def test_cancelling_pair_rejected_on_every_schedule():
    """Two invalid shares whose errors cancel in an unweighted sum —
    S_a + D and S_b - D for sender a, b's true shares S_a, S_b of one
    ciphertext — planted in one batch of 64 (and again across two
    ciphertexts' batches): the batch sum with equal weights would pass, the
    secret 127-bit weights make it fail, and the binary splitting reaches both
    singles, so both bits are 0 on every schedule (test hook 1, 2, 3, 0) and
    under the production HBG_VERIFY_PER_SHARE flag; every other share is 1.
    An unknown schedule mode is refused."""
    import json
    import os
    from hydrabadger_amd import _lib
    th = _th()
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tdec_n64.json")))["scenario"]
    K, n = len(g["cts"]), len(g["pk_shares"])
    cts = [th.Ciphertext(bytes.fromhex(c["U"]), bytes.fromhex(c["V"]), bytes.fromhex(c["W"])) for c in g["cts"]]
    pk = [bytes.fromhex(p) for p in g["pk_shares"]]
    D = B.g1_mul(B.G1, 0x1234567890ABCDEF)
    shares = [[bytes.fromhex(x) for x in c["shares"]] for c in g["cts"]]

    def shifted(j, i, sign):
        p = B.g1_decompress(shares[j][i])
        return B.g1_compress(B.g1_add(p, D if sign > 0 else B.g1_neg(D)))

    items, expect = [], []
    for j in range(K):
        for i in range(n):
            if (j, i) in ((0, 3), (1, 17), (2, 60)):
                items.append((shifted(j, i, +1), j, i)); expect.append(0)
            elif (j, i) in ((0, 41), (1, 18), (3, 5)):
                items.append((shifted(j, i, -1), j, i)); expect.append(0)
            else:
                items.append((shares[j][i], j, i)); expect.append(1)
    expect = np.array(expect, np.uint8)
    ctx = _lib.Context(0)
    try:
        for mode in (1, 2, 3, 0):
            _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, mode))
            assert np.array_equal(th.verify_shares_batch(cts, pk, items, ctx), expect), mode
        _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, 3))
        ctx.set_share_verify(_lib.HBG_VERIFY_PER_SHARE)     # overrides the test hook
        assert np.array_equal(th.verify_shares_batch(cts, pk, items, ctx), expect)
        ctx.set_share_verify(_lib.HBG_VERIFY_BATCHED)
        assert np.array_equal(th.verify_shares_batch(cts, pk, items, ctx), expect)
        with pytest.raises(_lib.HbgError):
            ctx.set_share_verify(2)
    finally:
        ctx.close()


def test_batched_lines_beside_leaves():
    """8,200 ciphertexts (the fixture's 4 replicated) x 64 shares, 1 % bad:
    with 8,193..131,072 ciphertexts (api.hip kLinesBesideLeavesMin/Max) the
    batched schedule builds H (sponge inline) and W's line tables in one grid
    beside the share leaves (launch_lines, tdec_ct_prepare_hw); its bits equal
    the fixture's per-share truth.  The other two branches of launch_lines:
    below 8,193 ciphertexts (W on the aux stream, H on the main one) with
    round-capacity overflow into the per-share round —
    test_batched_verify_equals_per_share's 150 ciphertexts at 30 % / 100 %
    bad; above 131,072 — test_batched_lines_above_beside_max."""
    import json
    import os
    from hydrabadger_amd import _lib
    th = _th()
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tdec_n64.json")))["scenario"]
    K, n = len(g["cts"]), len(g["pk_shares"])
    n_ct = 8200
    cts = [th.Ciphertext(bytes.fromhex(g["cts"][j % K]["U"]), bytes.fromhex(g["cts"][j % K]["V"]),
                         bytes.fromhex(g["cts"][j % K]["W"])) for j in range(n_ct)]
    pk = [bytes.fromhex(p) for p in g["pk_shares"]]
    shares = [[bytes.fromhex(x) for x in c["shares"]] for c in g["cts"]]
    rng = np.random.default_rng(11)
    bad = rng.random(n_ct * n) < 0.01
    items = [(shares[j % K][i], j, (i + 1) % n if bad[j * n + i] else i) for j in range(n_ct) for i in range(n)]
    expect = (~bad).astype(np.uint8)
    ctx = _lib.Context(0)
    try:
        _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, 2))
        out = th.verify_shares_batch(cts, pk, items, ctx)
    finally:
        ctx.close()
    assert np.array_equal(out, expect)


def test_batched_lines_above_beside_max():
    """131,200 device-generated ciphertexts x 16 shares (2 % bad, three
    kinds): past kLinesBesideLeavesMax the deferred line tables fall back to
    W on the aux stream and H (SHA3(V) by tdec_v_digest) on the main stream;
    every bit equals construction."""
    torch = pytest.importorskip("torch")
    from hydrabadger_amd import _lib, tdec_workload as tw
    dev = torch.device("cuda:0")
    ctx = _lib.Context(0)
    try:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        n_ct, N = 131_200, 16
        ep = tw.make_epoch(ctx, dev, n_ct=n_ct, n_nodes=N, msg_len=32, bad_rate=0.02, seed=5)
        n = n_ct * N
        sct = torch.arange(n_ct, dtype=torch.int32, device=dev).repeat_interleave(N)
        spk = torch.arange(N, dtype=torch.int32, device=dev).repeat(n_ct)
        ok = torch.zeros(n, dtype=torch.uint8, device=dev)
        _lib.check(_lib.lib().hbg_tdec_verify_shares(ctx.h, n_ct, ep.U.data_ptr(), ep.V.data_ptr(),
                                                     ep.V_off.data_ptr(), ep.W.data_ptr(), N, ep.pk48.data_ptr(), n,
                                                     ep.share48.data_ptr(), sct.data_ptr(), spk.data_ptr(),
                                                     ok.data_ptr(), _lib.HBG_DEVICE), "verify_decryption_share")
        assert np.array_equal(ok.cpu().numpy().reshape(n_ct, N).astype(bool), ~ep.bad)
    finally:
        ctx.close()


def test_g1_mul_u64_and_add():
    """Device G1 scalar multiplication by 64-bit weights and Jacobian addition
    (the batched verifier's building blocks) against the oracle."""
    th = _th()
    pts = [B.G1, B.g1_mul(B.G1, 7), B.g1_mul(B.G1, 2 ** 200 + 12345)]
    ks = [1, 2, 3, 0xFFFFFFFFFFFFFFFF, 0x8000000000000001, 0x123456789ABCDEF1]
    rows, ref = [], []
    for p in pts:
        for k in ks:
            rows.append(limbs(p[0]) + limbs(p[1]) + [k & 0xFFFFFFFF, k >> 32])
            ref.append(B.g1_mul(p, k))
    out = th.test_bls(9, np.array(rows, np.uint32), 25)
    for o, r in zip(out, ref):
        assert (from_limbs(o[:12]), from_limbs(o[12:24])) == r and o[24] == 0
    pairs = [(pts[0], pts[1]), (pts[1], pts[1]), (pts[2], B.g1_neg(pts[2])), (pts[1], pts[2])]
    out = th.test_bls(10, np.array([limbs(p[0]) + limbs(p[1]) + limbs(q[0]) + limbs(q[1]) for p, q in pairs],
                                   np.uint32), 25)
    for o, (p, q) in zip(out, pairs):
        r = B.g1_add(p, q)
        if r is None:
            assert o[24] == 1
        else:
            assert (from_limbs(o[:12]), from_limbs(o[12:24])) == r and o[24] == 0


@pytest.mark.parametrize("t", [0, 5, 21, 31, 32, 40, 42, 63, 70])
def test_combine_kernels_interpolate_arbitrary_points(t):
    """hbg_tdec_combine over arbitrary G1 points (interpolation does not care
    whether shares are valid): t + 1 <= 24 runs the 16-lane-group kernel,
    t + 1 <= 32 the 32-lane one, t + 1 <= 64 (32: one share in the second
    row; 40, 42 = configs[4]'s t; 63) the 32-lane one with two shares a lane,
    t = 70 the one-lane-per-ciphertext kernel.  Shuffled sparse indices, identity
    shares, an odd ciphertext count (half-live last group), and per-ciphertext
    DuplicateEntry / undecodable-share statuses in the same call."""
    from hydrabadger_amd import _lib
    th = _th()
    rng = random.Random(1000 + t)
    n_ct = 5
    cts_o, items, expect = [], [], []
    for c in range(n_ct):
        U = B.g1_mul(B.G1, rng.randrange(1, B.R))
        V = bytes(rng.randrange(256) for _ in range(rng.choice([0, 7, 64, 65, 300])))
        W = B.g2_mul(B.G2, rng.randrange(1, B.R))
        cts_o.append(T.Ciphertext(U, V, W))
        ids = rng.sample(range(200), t + 1)
        pts = [None if (j == 1 and c == 2) else B.g1_mul(B.G1, rng.randrange(1, B.R)) for j in range(t + 1)]
        it = [(i, B.g1_compress(p)) for i, p in zip(ids, pts)]
        st = 0
        if c == 3 and t > 0:
            it[-1] = (it[0][0], it[-1][1])            # duplicate index -> DuplicateEntry
            st = 1
        if c == 4:
            junk = bytearray(it[0][1]); junk[0] &= 0x7F  # undecodable share
            it[0] = (it[0][0], bytes(junk))
            st = 2 if st == 0 else st
        items.append(it)
        expect.append((st, None if st else T.decrypt(t, list(zip(ids, pts)), cts_o[-1])))
    cts = [th.Ciphertext(B.g1_compress(c.U), c.V, B.g2_compress(c.W)) for c in cts_o]
    pts_out, status = th.combine_batch(t, cts, items)
    for c, (st, pt) in enumerate(expect):
        if st == 0:
            assert status[c] == 0 and pts_out[c] == pt, c
        elif st == 1:
            assert status[c] == _lib.HBG_E_DUPLICATE_ENTRY, c
        else:
            assert status[c] == _lib.HBG_E_INVALID_POINT, c


def test_legendre_and_fp2_square_test():
    """The Jacobi-algorithm quadratic-residue screen of hash_g2's
    try-and-increment (tdec_kernels.hip fp_legendre / fp2_is_square) agrees
    with Euler's criterion and with the oracle's Fq2 sqrt."""
    th = _th()
    rnd = _rnd(11)
    vals = [(0, 0), (1, 0), (B.P - 1, 0), (4, 0), (2, 0), (3, 5), (0, 7)] + [(rnd(), rnd()) for _ in range(300)]
    vals += [((a * a) % B.P, 0) for a in (rnd() for _ in range(20))]
    out = th.test_bls(11, np.array([limbs(a) + limbs(b) for a, b in vals], np.uint32), 2)
    for (a, b), o in zip(vals, out):
        e = pow(a, (B.P - 1) // 2, B.P)
        leg = 0 if a == 0 else (1 if e == 1 else -1)
        assert int(np.int32(o[0])) == leg, (a, o[0])
        assert bool(o[1]) == (B.f2_sqrt((a, b)) is not None)


def test_hash_g2_many_seeds_fast_cofactor():
    """hash_g2 with the Budroni-Pintore + psi-decomposed cofactor clearing and
    the Legendre screen equals the oracle's plain [h2] multiplication for 48
    seeds (random and structured)."""
    th = _th()
    from oracle.merkle import sha3
    seeds = [sha3(b"hbg-hash-g2-%d" % i) for i in range(40)] + [bytes([i]) * 32 for i in range(8)]
    out = th.test_bls(6, np.array([list(np.frombuffer(s, np.uint32)) for s in seeds], np.uint32), 48)
    for s, o in zip(seeds, out):
        ref = T._rand_g2(ChaChaRng(s))
        got = ((from_limbs(o[0:12]), from_limbs(o[12:24])), (from_limbs(o[24:36]), from_limbs(o[36:48])))
        assert got == ref
