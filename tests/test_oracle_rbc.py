"""Pins the RBC oracle (CPU) against the known answers of SURVEY.md §8(c) and
the committed golden fixtures; cross-checks the numpy and C restatements.

KATs:  Backblaze JavaReedSolomon testOneEncode (RS 5+5), FIPS-202 SHA3-256
via hashlib (OpenSSL), rse structural properties (systematic top, any-D-rows
invertible).  Merkle tree shape has no external fixture: "parity unpinned"
 — it is checked here against its own stated invariants.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

from oracle import corc, gf256, merkle, rbc, synth

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_backblaze_kat():
    rs = gf256.ReedSolomon(5, 5)
    sh = np.zeros((10, 2), np.uint8)
    sh[:5] = [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]]
    rs.encode(sh)
    assert sh[5:].tolist() == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]
    c = sh.copy()
    c[5:] = 0
    corc.rs_encode(5, 5, c)
    assert np.array_equal(c, sh)


def test_gf_tables():
    assert gf256.gmul(3, 7) == 9 and gf256.gmul(0x80, 2) == 0x1D
    for a in range(1, 256):
        assert gf256.gmul(a, gf256.gdiv(1, a)) == 1
    assert gf256.gexp(0, 0) == 1 and gf256.gexp(0, 3) == 0


@pytest.mark.parametrize("D,Q", [(2, 2), (6, 10), (22, 42), (44, 84), (1, 1), (86, 170), (255, 1)])
def test_matrix_structure_and_c_match(D, Q):
    m = np.array(gf256.build_matrix(D, Q), np.uint8)
    assert np.array_equal(m[:D], np.eye(D, dtype=np.uint8))  # systematic
    assert np.array_equal(m, corc.build_matrix(D, Q))


def test_matrix_errors():
    with pytest.raises(gf256.TooFewDataShards):
        gf256.build_matrix(0, 3)
    with pytest.raises(gf256.TooFewParityShards):
        gf256.build_matrix(3, 0)
    with pytest.raises(gf256.TooManyShards):
        gf256.build_matrix(200, 57)


@pytest.mark.parametrize("n", [0, 1, 7, 8, 135, 136, 137, 200, 271, 272, 273, 1000, 5000])
def test_sha3_fips202(n):
    d = synth.synth_bytes(1, n, n)
    assert corc.sha3(d) == hashlib.sha3_256(d).digest() == merkle.sha3(d)


def test_sha3_empty_vector():
    assert merkle.sha3(b"").hex() == "a7ffc6f8bf1ed76651c14756a061d662f580ff4de43b49fa82d80a4b80f8434a"


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 7, 16, 33, 64, 128])
def test_merkle_invariants(N):
    vals = [synth.synth_bytes(1, N + i, 50) for i in range(N)]
    t = merkle.MerkleTree.from_vec(vals)
    assert len(t.flat_levels()) == merkle.num_nodes(N)
    for i in range(N):
        p = t.proof(i)
        assert p.validate(N)
        assert len(p.digests) <= merkle.depth(N)
        if N > 1:
            assert not merkle.Proof(p.value, p.index, p.digests, b"\0" * 32).validate(N)
    # odd promotion: the last node of an odd level is carried up unchanged
    if N == 5:
        assert t.levels[1][2] == t.levels[0][4] and t.levels[2][1] == t.levels[1][2]
    c = corc.merkle_levels(np.stack([np.frombuffer(v, np.uint8) for v in vals]))
    assert [bytes(x) for x in c] == t.flat_levels()


@pytest.mark.parametrize("N", [1, 2, 3, 4, 7, 16, 64, 128])
def test_rbc_roundtrip_numpy_vs_c(N):
    for P in [0, 1, 100, 3000]:
        pl = synth.payload(N * 100 + P, P)
        sh, tr = rbc.send_shards(pl, N)
        csh, clv = corc.rbc_encode_merkle(N, np.frombuffer(pl, np.uint8).copy())
        assert np.array_equal(sh, csh)
        assert [bytes(x) for x in clv] == tr.flat_levels()
        d, q = rbc.shard_counts(N)
        mask = synth.erasure_mask(N + P, N, q)
        lv = [sh[i].copy() if mask[i] else None for i in range(N)]
        assert rbc.decode_from_shards(lv, N, tr.root_hash) == pl
        c = sh.copy()
        c[[not m for m in mask]] = 0
        assert corc.rbc_decode(N, sh.shape[1], c, np.array(mask, np.uint8), tr.root_hash) == pl


def test_synth_c_matches_python():
    for tag, inst, n in [(1, 0, 100), (1, 5, 17), (2, 123456789, 64), (3, 2 ** 40, 9)]:
        assert corc.synth_bytes(tag, inst, n).tobytes() == synth.synth_bytes(tag, inst, n)
    m = synth.erasure_mask(3, 64, 42)
    assert sum(m) == 22


def _golden():
    with open(os.path.join(GOLDEN, "rbc_golden.json")) as f:
        return json.load(f)


def test_golden_fixtures_reproduce():
    """The committed fixtures (tests/golden/make_golden.py) still match the oracle."""
    g = _golden()
    assert g["backblaze"]["parity"] == [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]
    for case in g["send_shards"]:
        N, P, inst = case["N"], case["P"], case["instance"]
        pl = synth.payload(inst, P)
        assert hashlib.sha3_256(pl).hexdigest() == case["payload_sha3"]
        sh, tr = rbc.send_shards(pl, N)
        assert sh.shape[1] == case["L"]
        assert tr.root_hash.hex() == case["root"]
        assert hashlib.sha3_256(sh.tobytes()).hexdigest() == case["shards_sha3"]
        if "shards_hex" in case:
            assert sh.tobytes().hex() == case["shards_hex"]
        assert [d.hex() for d in tr.proof(case["proof_index"]).digests] == case["proof_digests"]
    for case in g["matrices"]:
        m = np.array(gf256.build_matrix(case["D"], case["Q"]), np.uint8)
        assert hashlib.sha3_256(m.tobytes()).hexdigest() == case["sha3"]
        assert m[case["D"]:case["D"] + 2].tolist() == case["first_parity_rows"]
