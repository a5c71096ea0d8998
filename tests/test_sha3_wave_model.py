"""Lane-program model of tdec_v_digest_wave (hydrabadger_amd/csrc/tdec_kernels.hip,
the bit-interleaved SHA3(V) wave sponge): 64 lanes, lane 2i + h holding the
even (h = 0) or odd (h = 1) bits of Keccak state word i, every cross-lane move
a dword gather from a per-lane source address.  The model computes the
kernel's per-lane constants (theta's column-x-1 / column-x+1 addresses, the
rho amount and the pi+chi source addresses with their half swap) with the
kernel's formulas and runs its round on Python ints, so the address and
rotation tables are checked against hashlib's SHA3-256 on the host; the GPU
tests check the kernel itself through W (test_gpu_bls_ops.py).
"""
from __future__ import annotations

import hashlib
import random

RHO = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]
RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000, 0x000000000000808B,
      0x0000000080000001, 0x8000000080008081, 0x8000000000008009, 0x000000000000008A, 0x0000000000000088,
      0x0000000080008009, 0x000000008000000A, 0x000000008000808B, 0x800000000000008B, 0x8000000000008089,
      0x8000000000008003, 0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
      0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
M32 = 0xFFFFFFFF


def even_bits(w: int) -> int:
    return sum(((w >> (2 * i)) & 1) << i for i in range(32))


def rotr32(v: int, s: int) -> int:  # v_alignbit(v, v, s)
    s &= 31
    return ((v >> s) | (v << (32 - s))) & M32 if s else v


def pisrc(X: int, Y: int) -> int:
    return (3 * (Y + 15 - 3 * X)) % 5 + 5 * X


def lane_constants():
    out = []
    for l in range(64):
        ls = l if l < 50 else l - 50
        i, h = ls >> 1, ls & 1
        x, y = i % 5, i // 5
        am = [2 * ((x + 4) % 5 + 5 * j) + h for j in range(5)]          # column x-1, half h
        ap = [2 * ((x + 1) % 5 + 5 * j) + (h ^ 1) for j in range(5)]    # column x+1, half 1-h
        r = RHO[i]
        amt = (((r + 1) // 2 if h else (r - 1) // 2) if r & 1 else r // 2)
        src = [pisrc((x + k) % 5, y) for k in range(3)]
        ab = [2 * s + (h ^ (RHO[s] & 1)) for s in src]
        out.append({"am": am, "ap": ap, "scp": 0 if h else 31, "srho": (32 - amt) & 31, "ab": ab})
    return out


LANES = lane_constants()


def permute(s: list[int]) -> list[int]:
    for rnd in range(24):
        d = []
        for c in LANES:
            cm = 0
            for a in c["am"]:
                cm ^= s[a]
            cp = 0
            for a in c["ap"]:
                cp ^= s[a]
            d.append(cm ^ rotr32(cp, c["scp"]))
        s = [s[l] ^ d[l] for l in range(64)]
        rv = [rotr32(s[l], LANES[l]["srho"]) for l in range(64)]
        ns = []
        for l, c in enumerate(LANES):
            b0, b1, b2 = (rv[a] for a in c["ab"])
            v = b0 ^ (~b1 & b2 & M32)
            if l == 0:
                v ^= even_bits(RC[rnd])
            elif l == 1:
                v ^= even_bits(RC[rnd] >> 1)
            ns.append(v)
        s = ns
    return s


def sha3_model(msg: bytes) -> bytes:
    m = bytearray(msg) + b"\x06"
    m += bytes(-len(m) % 136)
    m[-1] |= 0x80
    s = [0] * 64
    for b in range(len(m) // 136):
        blk = m[136 * b:136 * b + 136]
        for l in range(34):  # message lanes: 17 words x 2 halves
            w = int.from_bytes(blk[8 * (l >> 1):8 * (l >> 1) + 8], "little")
            s[l] ^= even_bits(w >> (l & 1))
        s = permute(s)
    out = b""
    for wd in range(4):  # lanes 0..7 re-interleaved
        e, o = s[2 * wd], s[2 * wd + 1]
        w = sum((((e >> k) & 1) << (2 * k)) | (((o >> k) & 1) << (2 * k + 1)) for k in range(32))
        out += w.to_bytes(8, "little")
    return out


def test_interleaved_wave_sponge_model_matches_hashlib():
    rng = random.Random(11)
    for n in (0, 1, 65, 135, 136, 137, 272, 300):
        m = bytes(rng.getrandbits(8) for _ in range(n))
        assert sha3_model(m) == hashlib.sha3_256(m).digest(), n


def test_gather_sources_are_a_permutation():
    """Every pi+chi first source is used by exactly one of the 50 real lanes
    (each source pre-rotates for a single destination)."""
    firsts = sorted(c["ab"][0] for c in LANES[:50])
    assert firsts == list(range(50))
