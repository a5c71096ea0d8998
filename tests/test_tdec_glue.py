"""hbbft ThresholdDecrypt glue, batched over an epoch.

The oracle (oracle/tcrypto.py threshold_decrypt) restates hbbft's
set_ciphertext / handle_message / try_output; CPU tests pin its semantics on
hand-built cases (first t+1 valid arrivals, faults before termination, late
shares ignored, NotEnoughShares, rejected ciphertext).  GPU tests run
hbg_tdec_threshold_decrypt through the C ABI and must match the oracle's
status, per-sender outcome and plaintext exactly, including seeded random
arrival orders with the three corruption kinds of the bench.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

from oracle import bls12_381 as B
from oracle import tcrypto as T
from tests import tdec_fixtures as fx

ACC, FLT, IGN, NONE, REP = T.SHARE_ACCEPTED, T.SHARE_FAULTY, T.SHARE_IGNORED, T.SHARE_NONE, T.SHARE_REPEAT


def _case(seed=5):
    return fx.scenario(7, 3, 40, seed=seed)


# ------------------------------------------------------------------ oracle semantics (CPU)
def test_oracle_first_t_plus_one_valid_arrivals():
    sc = _case()
    t, ct, pks = sc["t"], sc["cts"][0], sc["pk_shares"]
    shares = list(sc["shares"][0])
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares)
    assert st == 0 and pt == sc["msgs"][0]
    assert oc == [ACC] * (t + 1) + [IGN] * (7 - t - 1)
    # a bad share before termination is a fault; the next valid one is taken instead
    shares[1] = B.g1_add(shares[1], B.G1)
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares)
    assert st == 0 and pt == sc["msgs"][0]
    assert oc == [ACC, FLT, ACC, ACC, IGN, IGN, IGN]
    # arrival order decides which shares are held; a held sender's second
    # message is a MultipleDecryptionShares fault and adds nothing
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[6, 6, 1, 5, 0, 3, 2])
    assert st == 0 and pt == sc["msgs"][0]
    assert oc == [ACC, FLT, IGN, IGN, NONE, ACC, ACC | REP]
    # a faulty sender's second message is faulted again; after termination nothing is checked
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[1, 0, 1, 2, 3, 3, 1])
    assert st == 0 and oc == [ACC, FLT, ACC, ACC, NONE, NONE, NONE]


def test_oracle_shares_before_the_ciphertext():
    """Shares that arrive before HoneyBadger outputs the ciphertext are held
    unverified (a repeat is faulted at once); start_decryption drops the
    invalid ones and try_output fires on what is left."""
    sc = _case()
    t, ct, pks = sc["t"], sc["cts"][0], sc["pk_shares"]
    shares = list(sc["shares"][0])
    shares[1] = B.g1_add(shares[1], B.G1)
    M = T.ARRIVAL_CIPHERTEXT
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[3, 1, 3, M, 0, 2, 4])
    assert st == 0 and pt == sc["msgs"][0]
    assert oc == [ACC, FLT, ACC, ACC | REP, IGN, NONE, NONE]
    # more than t+1 valid before the ciphertext: output at once with the first t+1 by node id
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[5, 4, 6, 0, M, 1, 2])
    assert st == 0 and pt == sc["msgs"][0]
    assert oc == [ACC, IGN, IGN, NONE, ACC, ACC, ACC]
    # a second marker changes nothing; no marker = the ciphertext came first
    assert T.threshold_decrypt(t, ct, pks, shares, arrival=[M, 0, M, 2, 3]) == \
        T.threshold_decrypt(t, ct, pks, shares, arrival=[0, 2, 3])
    # an invalid ciphertext ends the instance at the marker (repeat faults already logged stay)
    bad_ct = T.Ciphertext(ct.U, ct.V, B.g2_mul(ct.W, 2))
    st, pt, oc = T.threshold_decrypt(t, bad_ct, pks, shares, arrival=[0, 0, M, 2, 3])
    assert st == T.E_INVALID_CIPHERTEXT and pt is None and oc == [REP] + [NONE] * 6
    # too few valid shares by the end of the list
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[1, 0, M, 1, 2])
    assert st == T.E_NOT_ENOUGH_SHARES and oc == [ACC, FLT, ACC, NONE, NONE, NONE, NONE]


def test_oracle_own_share_at_start_decryption():
    """A validator's start_decryption (ARRIVAL_OWN | i) inserts its own share
    after dropping the invalid held shares and BEFORE try_output (hbbft
    threshold_decrypt.rs, via state.rs:486-487): with t+1 valid shares already
    held at the ciphertext the own share is still accepted and, being among
    the first t+1 by node id, interpolated; it is never verified."""
    sc = _case()
    t, ct, pks = sc["t"], sc["cts"][2], sc["pk_shares"]
    shares = list(sc["shares"][2])
    shares[4] = B.g1_add(shares[4], B.G1)
    M, OWN = T.ARRIVAL_CIPHERTEXT, T.ARRIVAL_OWN
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[3, 5, 6, 4, OWN | 0, 1, 2])
    assert st == 0 and pt == sc["msgs"][2]
    assert oc == [ACC, IGN, IGN, ACC, FLT, ACC, ACC]
    # the observer's marker at the same point: output at the marker from 3, 5, 6; 0 never arrives
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[3, 5, 6, 4, M, 1, 2])
    assert st == 0 and pt == sc["msgs"][2] and oc == [NONE, IGN, IGN, ACC, FLT, ACC, ACC]
    # no marker before it: start_decryption (own share first) precedes every arrival
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[OWN | 6, 4, 5, 1])
    assert st == 0 and oc == [NONE, ACC, NONE, NONE, FLT, ACC, ACC]
    # the own share is trusted: an invalid own share is inserted unverified (and the output is garbage)
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[OWN | 4, 0, 1])
    assert st == 0 and oc[4] == ACC and pt != sc["msgs"][2]
    # an own marker with an index >= N ends the list like any other entry >= N
    assert T.threshold_decrypt(t, ct, pks, shares, arrival=[0, 1, OWN | 7, 2]) == \
        T.threshold_decrypt(t, ct, pks, shares, arrival=[0, 1])


def test_oracle_not_enough_and_invalid_ciphertext():
    sc = _case()
    t, ct, pks = sc["t"], sc["cts"][1], sc["pk_shares"]
    shares = list(sc["shares"][1])
    st, pt, oc = T.threshold_decrypt(t, ct, pks, shares, arrival=[0, 4])
    assert st == T.E_NOT_ENOUGH_SHARES and pt is None and oc == [ACC, NONE, NONE, NONE, ACC, NONE, NONE]
    bad_ct = T.Ciphertext(ct.U, ct.V, B.g2_mul(ct.W, 2))
    st, pt, oc = T.threshold_decrypt(t, bad_ct, pks, shares)
    assert st == T.E_INVALID_CIPHERTEXT and oc == [NONE] * 7


# ------------------------------------------------------------------ GPU vs oracle
def _th():
    from hydrabadger_amd import threshold as th
    return th


def _corrupt(kind, k, i, sc, rng):
    """The bench's three corruption kinds for sender i's share of ct k."""
    n_ct, n = len(sc["cts"]), len(sc["pk_shares"])
    if kind == 0:   # another node's share (claimed under the wrong key)
        return sc["shares"][k][(i + 1) % n]
    if kind == 1:   # the same node's share of another ciphertext
        return sc["shares"][(k + 1) % n_ct][i]
    return B.g1_mul(B.G1, rng.randrange(1, B.R))   # a random valid point


@pytest.mark.gpu
def test_gpu_glue_matches_oracle_hand_cases():
    th = _th()
    sc = _case()
    t, pks = sc["t"], [B.g1_compress(p) for p in sc["pk_shares"]]
    ct0, ct1, ct2 = sc["cts"]
    bad_ct = T.Ciphertext(ct2.U, ct2.V, B.g2_mul(ct2.W, 2))
    cts = [ct0, ct0, ct1, bad_ct]
    sh = [list(sc["shares"][0]), list(sc["shares"][0]), list(sc["shares"][1]), list(sc["shares"][2])]
    sh[1][1] = B.g1_add(sh[1][1], B.G1)
    M = T.ARRIVAL_CIPHERTEXT
    cts += [ct0, ct0, bad_ct, ct1]
    sh += [list(sh[1]), list(sh[1]), list(sc["shares"][2]), list(sc["shares"][1])]
    O = T.ARRIVAL_OWN
    arrivals = [None, [6, 6, 1, 5, 0, 3, 2], [0, 4], None,
                [3, 1, 3, M, 0, 2, 4], [5, 4, 6, 0, M, 1, 2], [0, 0, M, 2, 3], [1, 0, 1, M, 1, 2, 2, 5]]
    # validator markers: own share inserted at start_decryption (also with t+1 already held; an own
    # index past N ends the list; an invalid own share is trusted)
    cts += [ct0, ct1, ct2, ct0, ct1]
    sh += [list(sc["shares"][0]), list(sc["shares"][1]), list(sc["shares"][2]), list(sh[1]), list(sh[1])]
    arrivals += [[3, 5, 6, 4, O | 0, 1, 2], [O | 6, 4, 5, 1], [5, 4, 6, 0, O | 2, 1], [0, 2, O | 1, 3],
                 [1, O | 7, 2, 3]]
    pts, st, oc = th.threshold_decrypt_batch(
        t, [th.Ciphertext(B.g1_compress(c.U), c.V, B.g2_compress(c.W)) for c in cts], pks,
        [[B.g1_compress(x) for x in row] for row in sh], arrivals)
    for k in range(len(cts)):
        rst, rpt, roc = T.threshold_decrypt(t, cts[k], sc["pk_shares"], sh[k], arrivals[k])
        assert st[k] == rst and list(oc[k]) == roc and pts[k] == rpt, k


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 3])
def test_gpu_glue_own_share_unverified(mode):
    """A validator's own share is inserted unverified (hbbft start_decryption),
    so the combine cannot take its point from the verification's decoded-point
    table: an own share that does not decode gives HBG_E_INVALID_POINT (with
    the own sender ACCEPTED, as the oracle's outcome), and an own public key
    share that does not decode (its network shares all fail) still combines
    the trusted own share into the right plaintext.  A first call on other
    ciphertexts fills the context's scratch, so a stale table entry would show
    as a wrong plaintext.  On the per-share (0) and batched (3) schedules."""
    from hydrabadger_amd import _lib
    th = _th()
    sc, other = _case(), _case(seed=9)
    t, n = sc["t"], len(sc["pk_shares"])
    pks = [B.g1_compress(p) for p in sc["pk_shares"]]
    O = T.ARRIVAL_OWN
    enc = lambda c: th.Ciphertext(B.g1_compress(c.U), c.V, B.g2_compress(c.W))  # noqa: E731
    ctx = _lib.Context(0)
    try:
        _lib.check(_lib.lib().hbg_test_set_tdec_batched(ctx.h, mode))
        pts, st, _ = th.threshold_decrypt_batch(
            t, [enc(c) for c in other["cts"]], [B.g1_compress(p) for p in other["pk_shares"]],
            [[B.g1_compress(x) for x in row] for row in other["shares"]], None, ctx)
        assert list(st) == [0] * len(other["cts"]) and pts == other["msgs"]
        # (1) own share 2 of ct 0 undecodable; ct 1 the same list with a valid own share
        sh = [[B.g1_compress(x) for x in row] for row in sc["shares"]]
        junk = bytearray(sh[0][2]); junk[0] &= 0x7F
        sh[0][2] = bytes(junk)
        arr = [[O | 2, 0, 1, 3], [O | 2, 0, 1, 3], [O | 2, 0, 1, 3]]
        pts, st, oc = th.threshold_decrypt_batch(t, [enc(c) for c in sc["cts"]], pks, sh, arr, ctx)
        assert st[0] == _lib.HBG_E_INVALID_POINT and oc[0][2] == ACC
        for k in (1, 2):
            rst, rpt, roc = T.threshold_decrypt(t, sc["cts"][k], sc["pk_shares"], sc["shares"][k], arr[k])
            assert st[k] == rst == 0 and pts[k] == rpt == sc["msgs"][k] and list(oc[k]) == roc
        # (2) own pk share 4 undecodable: node 4's network shares fail, its own share is trusted
        bad_pks = list(pks)
        jp = bytearray(bad_pks[4]); jp[0] &= 0x7F
        bad_pks[4] = bytes(jp)
        sh = [[B.g1_compress(x) for x in row] for row in sc["shares"]]
        arr = [[0, O | 4, 1, 2], [O | 4, 5, 6, 3], [4, O | 4, 1, 2]]
        pts, st, oc = th.threshold_decrypt_batch(t, [enc(c) for c in sc["cts"]], bad_pks, sh, arr, ctx)
        for k in range(3):
            assert st[k] == 0 and pts[k] == sc["msgs"][k], k
            assert oc[k][4] == ACC, k
        assert list(oc[0]) == [ACC, ACC, IGN, NONE, ACC, NONE, NONE]
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_glue_random_epochs_match_oracle(seed):
    """16 nodes (t = 5), 12 ciphertexts: seeded arrival orders (some lists cut
    short), ~15 % of the shares corrupted with the three kinds, one
    ciphertext with fewer than t+1 valid arrivals."""
    th = _th()
    rng = random.Random(seed)
    sc = fx.scenario(16, 12, 48, seed=20 + seed)
    t, n, n_ct = sc["t"], 16, 12
    shares, arrivals = [], []
    for k in range(n_ct):
        row = []
        for i in range(n):
            row.append(_corrupt(rng.randrange(3), k, i, sc, rng) if rng.random() < 0.15 else sc["shares"][k][i])
        order = list(range(n))
        rng.shuffle(order)
        if k % 4 == 3:
            order = order[: rng.randrange(t + 1, n)]
        shares.append(row)
        arrivals.append(order)
    arrivals[5] = [i for i in arrivals[5]][: t]          # never enough
    cts = [th.Ciphertext(B.g1_compress(c.U), c.V, B.g2_compress(c.W)) for c in sc["cts"]]
    # senders missing from a cut arrival list never sent
    sent = [[x if i in set(arrivals[k]) else None for i, x in enumerate(shares[k])] for k in range(n_ct)]
    pts, st, oc = th.threshold_decrypt_batch(t, cts, [B.g1_compress(p) for p in sc["pk_shares"]],
                                             [[None if x is None else B.g1_compress(x) for x in row] for row in sent],
                                             arrivals)
    for k in range(n_ct):
        rst, rpt, roc = T.threshold_decrypt(t, sc["cts"][k], sc["pk_shares"], shares[k], arrivals[k])
        assert (int(st[k]), list(oc[k]), pts[k]) == (rst, roc, rpt), k
    assert int(st[5]) == T.E_NOT_ENOUGH_SHARES


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 4])
def test_gpu_glue_early_shares_and_repeats_match_oracle(seed):
    """HoneyBadger-style arrivals: the ciphertext marker at a seeded position
    (shares before it held unverified), ~20 % of the messages repeated
    (MultipleDecryptionShares), ~15 % of the shares corrupted."""
    th = _th()
    rng = random.Random(seed)
    sc = fx.scenario(16, 12, 48, seed=30 + seed)
    t, n, n_ct = sc["t"], 16, 12
    M = T.ARRIVAL_CIPHERTEXT
    shares, arrivals = [], []
    for k in range(n_ct):
        shares.append([_corrupt(rng.randrange(3), k, i, sc, rng) if rng.random() < 0.15 else sc["shares"][k][i]
                       for i in range(n)])
        order = list(range(n))
        rng.shuffle(order)
        order += [rng.randrange(n) for _ in range(rng.randrange(0, 5))]
        rng.shuffle(order)
        order.insert(rng.randrange(0, len(order) + 1), M)
        arrivals.append(order)
    cts = [th.Ciphertext(B.g1_compress(c.U), c.V, B.g2_compress(c.W)) for c in sc["cts"]]
    pts, st, oc = th.threshold_decrypt_batch(t, cts, [B.g1_compress(p) for p in sc["pk_shares"]],
                                             [[B.g1_compress(x) for x in row] for row in shares], arrivals)
    flags = 0
    for k in range(n_ct):
        rst, rpt, roc = T.threshold_decrypt(t, sc["cts"][k], sc["pk_shares"], shares[k], arrivals[k])
        assert (int(st[k]), list(oc[k]), pts[k]) == (rst, roc, rpt), k
        flags += sum(1 for x in roc if x & REP)
    assert flags > 0


@pytest.mark.gpu
def test_gpu_glue_device_mode_async():
    """Device tensors, HBG_ASYNC: same answers as the host-mode call."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hydrabadger_amd import _lib
    th = _th()
    sc = fx.scenario(16, 4, 64, seed=9)
    t, n, n_ct = sc["t"], 16, 4
    cts = [th.Ciphertext(B.g1_compress(c.U), c.V, B.g2_compress(c.W)) for c in sc["cts"]]
    U, V, off, W = th._ct_table(cts)
    pk = np.frombuffer(b"".join(B.g1_compress(p) for p in sc["pk_shares"]), np.uint8).copy()
    sh = np.frombuffer(b"".join(B.g1_compress(sc["shares"][k][i]) for k in range(n_ct) for i in range(n)),
                       np.uint8).copy().reshape(n_ct, n, 48)
    sh[2, 3] = sh[2, 4]
    dev = torch.device("cuda:0")
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    pt = torch.zeros(int(off[-1]), dtype=torch.uint8, device=dev)
    st = torch.zeros(n_ct, dtype=torch.int32, device=dev)
    oc = torch.zeros((n_ct, n), dtype=torch.uint8, device=dev)
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    th.threshold_decrypt_arrays(t, n, d(U), d(V), d(off.view(np.int64)), d(W), d(pk), d(sh), None, pt, st, oc,
                                ctx=ctx, device=True, asynchronous=True)
    ctx.sync()
    pts_h, st_h, oc_h = th.threshold_decrypt_batch(t, cts, [B.g1_compress(p) for p in sc["pk_shares"]],
                                                   [[sh[k, i].tobytes() for i in range(n)] for k in range(n_ct)])
    assert st.cpu().tolist() == st_h.tolist() == [0] * n_ct
    assert np.array_equal(oc.cpu().numpy(), oc_h)
    assert oc_h[2, 3] == FLT
    assert pt.cpu().numpy().tobytes() == b"".join(sc["msgs"])


@pytest.mark.gpu
def test_device_generated_epoch_and_driver():
    """hydrabadger_amd/tdec_workload.py (the bench's TDec inputs): key shares,
    distinct ciphertexts and shares made on the device match the oracle for
    a sample, and the driver's outcomes / plaintexts equal construction."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hydrabadger_amd import _lib, tdec_workload as tw
    th = _th()
    dev = torch.device("cuda:0")
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ep = tw.make_epoch(ctx, dev, n_ct=96, n_nodes=16, msg_len=200, bad_rate=0.08, seed=3)
    coeffs, sks = tw.keyset(16, ep.t, 3)
    assert ep.pk48[5].cpu().numpy().tobytes() == B.g1_compress(B.g1_mul(B.G1, sks[5]))
    assert ep.master_pk48.cpu().numpy().tobytes() == B.g1_compress(B.g1_mul(B.G1, coeffs[0]))
    assert len(set(map(bytes, ep.U.cpu().numpy()))) == 96                     # distinct ciphertexts
    k = 17
    ct = T.Ciphertext(B.g1_decompress(ep.U[k].cpu().numpy().tobytes()), ep.V[200 * k:200 * k + 200].cpu().numpy().tobytes(),
                      B.g2_decompress(ep.W[k].cpu().numpy().tobytes()))
    assert ct.verify()
    assert T.decrypt(ep.t, [(i, T.decrypt_share(sks[i], ct)) for i in range(ep.t + 1)], ct) == \
        ep.msgs[200 * k:200 * k + 200].cpu().numpy().tobytes()
    for (kk, ii) in list(zip(*np.nonzero(ep.bad)))[:6]:                       # replaced shares do not verify
        ck = T.Ciphertext(B.g1_decompress(ep.U[kk].cpu().numpy().tobytes()),
                          ep.V[200 * kk:200 * kk + 200].cpu().numpy().tobytes(),
                          B.g2_decompress(ep.W[kk].cpu().numpy().tobytes()))
        s = B.g1_decompress(ep.share48[kk, ii].cpu().numpy().tobytes())
        assert not T.verify_decryption_share(B.g1_mul(B.G1, sks[ii]), s, ck)
    assert set(np.unique(ep.kind[ep.bad])) == {0, 1, 2}
    pt = torch.zeros(96 * 200, dtype=torch.uint8, device=dev)
    st = torch.zeros(96, dtype=torch.int32, device=dev)
    oc = torch.zeros((96, 16), dtype=torch.uint8, device=dev)
    th.threshold_decrypt_arrays(ep.t, 16, ep.U, ep.V, ep.V_off, ep.W, ep.pk48, ep.share48, None, pt, st, oc,
                                ctx=ctx, device=True)
    assert st.cpu().tolist() == [0] * 96
    assert np.array_equal(oc.cpu().numpy(), tw.expected_outcomes(ep.bad, ep.t))
    assert torch.equal(pt, ep.msgs)


@pytest.mark.gpu
def test_configs3_size_threshold_decrypt_100k():
    """BASELINE.json configs[3] at full size: 100,000 distinct ciphertexts x 64
    shares (N = 64, t = 21, 1 % bad shares of the three kinds) through
    hbg_tdec_verify_shares and hbg_tdec_threshold_decrypt (device mode).  The
    round-2 grid-stride kernels faulted at >= 65,536 ciphertexts; this is the
    size that has to hold.  Checks: every share bit against construction,
    every outcome byte and plaintext against construction, and a sample of
    ciphertexts (every one holding a bad share among them) bit for bit against
    the C oracle's per-share verify_decryption_share and PublicKeySet::decrypt."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hydrabadger_amd import _lib, tdec_workload as tw
    from oracle import corb
    th = _th()
    dev = torch.device("cuda:0")
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    n_ct, N, L = 100_000, 64, 256
    ep = tw.make_epoch(ctx, dev, n_ct=n_ct, n_nodes=N, msg_len=L, bad_rate=0.01, seed=11)
    n = n_ct * N
    sct = torch.arange(n_ct, dtype=torch.int32, device=dev).repeat_interleave(N)
    spk = torch.arange(N, dtype=torch.int32, device=dev).repeat(n_ct)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    _lib.check(_lib.lib().hbg_tdec_verify_shares(ctx.h, n_ct, ep.U.data_ptr(), ep.V.data_ptr(), ep.V_off.data_ptr(),
                                                 ep.W.data_ptr(), N, ep.pk48.data_ptr(), n, ep.share48.data_ptr(),
                                                 sct.data_ptr(), spk.data_ptr(), ok.data_ptr(), _lib.HBG_DEVICE),
               "verify_decryption_share")
    okh = ok.cpu().numpy().reshape(n_ct, N).astype(bool)
    assert np.array_equal(okh, ~ep.bad)
    pt = torch.zeros(n_ct * L, dtype=torch.uint8, device=dev)
    st = torch.zeros(n_ct, dtype=torch.int32, device=dev)
    oc = torch.zeros((n_ct, N), dtype=torch.uint8, device=dev)
    th.threshold_decrypt_arrays(ep.t, N, ep.U, ep.V, ep.V_off, ep.W, ep.pk48, ep.share48, None, pt, st, oc,
                                ctx=ctx, device=True)
    assert st.cpu().tolist() == [0] * n_ct
    assert np.array_equal(oc.cpu().numpy(), tw.expected_outcomes(ep.bad, ep.t))
    assert torch.equal(pt, ep.msgs)
    # sampled oracle comparison: ciphertexts with a bad share, spread over the batch
    bad_rows = np.nonzero(ep.bad.any(axis=1))[0]
    sample = sorted(set(bad_rows[:: max(1, len(bad_rows) // 6)][:6].tolist() + [0, n_ct // 2, n_ct - 1]))
    U, V, W = ep.U.cpu().numpy(), ep.V.cpu().numpy(), ep.W.cpu().numpy()
    pk = [ep.pk48[i].cpu().numpy().tobytes() for i in range(N)]
    sh = ep.share48.cpu().numpy()
    cts = [(U[k].tobytes(), V[L * k:L * (k + 1)].tobytes(), W[k].tobytes()) for k in sample]
    items = [(sh[k, i].tobytes(), j, i) for j, k in enumerate(sample) for i in range(N)]
    ref = corb.verify_shares(cts, pk, items, threads=8).reshape(len(sample), N)
    assert np.array_equal(ref.astype(bool), okh[sample])
    sel = [[(i, sh[k, i].tobytes()) for i in range(N) if okh[k, i]][: ep.t + 1] for k in sample]
    pts, rst = corb.decrypt_batch(ep.t, cts, sel, threads=8)
    ph = pt.cpu().numpy()
    assert rst.tolist() == [0] * len(sample)
    assert pts == [ph[L * k:L * (k + 1)].tobytes() for k in sample]


# ------------------------------------------------------------------ a18 fixture (tests/golden/tdec_golden.json)
def _a18_fixture():
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tdec_golden.json")))
    sc = g["scenario"]
    M = T.ARRIVAL_CIPHERTEXT
    cases = []
    for c in g["threshold_decrypt"]["cases"]:
        ct = sc["cts"][c["ct"]]
        shares = [bytes.fromhex(x) for x in ct["shares"]]
        shares[c["bad_sender"]] = bytes.fromhex(c["bad_share"])
        own = T.ARRIVAL_OWN | g["threshold_decrypt"]["our_node"]
        arrival = [own if a == "own" else (M if a == "ct" else a) for a in c["arrival"]]
        cases.append((ct, shares, arrival, c))
    return sc, cases


def test_oracle_matches_a18_fixture():
    sc, cases = _a18_fixture()
    pks = [B.g1_decompress(bytes.fromhex(p)) for p in sc["pk_shares"]]
    for ct, shares, arrival, c in cases:
        cto = T.Ciphertext(B.g1_decompress(bytes.fromhex(ct["U"])), bytes.fromhex(ct["V"]),
                           B.g2_decompress(bytes.fromhex(ct["W"])))
        st, pt, oc = T.threshold_decrypt(sc["t"], cto, pks, [B.g1_decompress(s) for s in shares], arrival)
        assert (st, oc, None if pt is None else pt.hex()) == (c["status"], c["outcome"], c["plaintext"])


@pytest.mark.gpu
def test_gpu_glue_matches_a18_fixture():
    th = _th()
    sc, cases = _a18_fixture()
    cts = [th.Ciphertext(bytes.fromhex(ct["U"]), bytes.fromhex(ct["V"]), bytes.fromhex(ct["W"]))
           for ct, _, _, _ in cases]
    pts, st, oc = th.threshold_decrypt_batch(sc["t"], cts, [bytes.fromhex(p) for p in sc["pk_shares"]],
                                             [s for _, s, _, _ in cases], [a for _, _, a, _ in cases])
    for k, (_, _, _, c) in enumerate(cases):
        assert (int(st[k]), list(oc[k]), None if pts[k] is None else pts[k].hex()) == \
            (c["status"], c["outcome"], c["plaintext"]), k
