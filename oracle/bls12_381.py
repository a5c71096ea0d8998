"""BLS12-381 restatement (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Restates the zkcrypto ``pairing`` crate's bls12_381 module [EXT, version
unpinned: 0.14-0.16 share these formulas] as threshold_crypto uses it
(SURVEY.md §8(a) a11-a17):

* Fq (p, 381 bit), Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3-(u+1)),
  Fq12 = Fq6[w]/(w^2-v); Fr (r, 255 bit);
* G1: y^2 = x^3 + 4 over Fq; G2: y^2 = x^3 + 4(u+1) over Fq2;
* optimal-ate Miller loop over |x| (x = -0xd201000000010000) with the
  crate's G2Prepared (Algorithms 26/27 of eprint 2010/354, homogeneous
  projective) line coefficients and ``mul_by_014``; the crate's
  final-exponentiation addition chain (exp_by_x);
* zcash compressed encodings (48 B G1, 96 B G2: flag bits 7 compressed,
  6 infinity, 5 y-lexicographically-largest; Fq2 as c1 || c0).

Constants are checked in tests/test_oracle_tdec.py (generator on curve,
r*G = O, p and r from x, compression of the G1 generator).  The pairing is
pinned by bilinearity / non-degeneracy and by equality with the plain
exponentiation f^((p^12-1)/r) cubed (the crate's chain computes e^3).
"""
from __future__ import annotations

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
BLS_X = 0xD201000000010000  # |x|; x is negative
BLS_X_IS_NEGATIVE = True

G1_X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1_Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1
G2_X = (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E)
G2_Y = (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE)

# G2 cofactor used by the crate's scale_by_cofactor (pairing 0.14 G2Affine)
G2_COFACTOR = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5
G1_COFACTOR = 0x396C8C005555E1568C00AAAB0000AAAB

R_MONT = 1 << 384  # Fq Montgomery radix (6 x 64-bit limbs)
R_MONT_INV = pow(R_MONT, -1, P)


# --------------------------------------------------------------------------- Fq2
def f2(a0, a1=0):
    return (a0 % P, a1 % P)


F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    return ((t0 - t1) % P, ((a[0] + a[1]) * (b[0] + b[1]) - t0 - t1) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    t = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
    return (a[0] * t % P, (-a[1]) * t % P)


def f2_mul_xi(a):
    """(a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u"""
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)


def f2_pow(a, e):
    r = F2_ONE
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_sqr(a)
        e >>= 1
    return r


def f2_frob(a, k=1):
    return a if k % 2 == 0 else f2_conj(a)


def fq_gt(a, b):
    return a > b


def f2_gt(a, b):
    """Fq2 Ord of the crate: compare c1 first, then c0 (canonical integers)."""
    if a[1] != b[1]:
        return a[1] > b[1]
    return a[0] > b[0]


def fq_sqrt(a):
    """p = 3 mod 4: a^((p+1)/4); None when a is not a square."""
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a % P else None


def f2_sqrt(a):
    """Algorithm 9 of eprint 2012/685 (the crate's Fq2::sqrt); any root is
    fine for callers here because they pick by lexicographic order."""
    if a == F2_ZERO:
        return F2_ZERO
    a1 = f2_pow(a, (P - 3) // 4)
    alpha = f2_mul(f2_sqr(a1), a)
    a0 = f2_mul(f2_frob(alpha), alpha)
    if a0 == (P - 1, 0):
        return None
    a1 = f2_mul(a1, a)
    if alpha == (P - 1, 0):
        return f2_mul(a1, (0, 1))
    b = f2_pow(f2_add(alpha, F2_ONE), (P - 1) // 2)
    return f2_mul(a1, b)


# --------------------------------------------------------------------------- Fq6 / Fq12
def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(f2_neg(x) for x in a)


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0, t1, t2 = f2_mul(a0, b0), f2_mul(a1, b1), f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_mul(f2_add(a1, a2), f2_add(b1, b2)), f2_add(t1, t2))))
    c1 = f2_add(f2_sub(f2_mul(f2_add(a0, a1), f2_add(b0, b1)), f2_add(t0, t1)), f2_mul_xi(t2))
    c2 = f2_add(f2_sub(f2_mul(f2_add(a0, a2), f2_add(b0, b2)), f2_add(t0, t2)), t1)
    return (c0, c1, c2)


def f6_mul_by_v(a):
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_xi(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0, t1 = f6_mul(a0, b0), f6_mul(a1, b1)
    c1 = f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), f6_add(t0, t1))
    c0 = f6_add(t0, f6_mul_by_v(t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_inv(f6_sub(f6_mul(a0, a0), f6_mul_by_v(f6_mul(a1, a1))))
    return (f6_mul(a0, t), f6_neg(f6_mul(a1, t)))


def f12_pow(a, e):
    r = F12_ONE
    while e:
        if e & 1:
            r = f12_mul(r, a)
        a = f12_sqr(a)
        e >>= 1
    return r


XI = (1, 1)
# Frobenius coefficients: gamma_{k,j} = xi^(j*(p^k-1)/6)
_G6_1 = [f2_pow(XI, (P ** k - 1) // 3) for k in range(12)]        # for v
_G6_2 = [f2_pow(XI, 2 * (P ** k - 1) // 3) for k in range(12)]    # for v^2
_G12 = [f2_pow(XI, (P ** k - 1) // 6) for k in range(12)]         # for w


def f6_frob(a, k):
    return (f2_frob(a[0], k), f2_mul(f2_frob(a[1], k), _G6_1[k % 12]), f2_mul(f2_frob(a[2], k), _G6_2[k % 12]))


def f12_frob(a, k):
    c0 = f6_frob(a[0], k)
    c1 = f6_frob(a[1], k)
    g = _G12[k % 12]
    return (c0, tuple(f2_mul(x, g) for x in c1))


def f12_mul_by_014(f, c0, c1, c4):
    """f * (c0 + c1 v + c4 v w)  (the crate's sparse line product)."""
    line = ((c0, c1, F2_ZERO), (F2_ZERO, c4, F2_ZERO))
    return f12_mul(f, line)


# --------------------------------------------------------------------------- curves
# points: affine (x, y) or None for infinity; Jacobian internally.
B1 = 4
B2 = (4, 4)


def g1_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g2_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


class _F1:
    add, sub, mul, sqr, neg = (lambda a, b: (a + b) % P), (lambda a, b: (a - b) % P), (lambda a, b: a * b % P), \
        (lambda a: a * a % P), (lambda a: (-a) % P)
    zero, one = 0, 1

    @staticmethod
    def inv(a):
        return pow(a, P - 2, P)

    @staticmethod
    def small(a, k):
        return a * k % P


class _F2:
    add, sub, mul, sqr, neg, inv = f2_add, f2_sub, f2_mul, f2_sqr, f2_neg, f2_inv
    zero, one = F2_ZERO, F2_ONE

    @staticmethod
    def small(a, k):
        return f2_muls(a, k)


def _jac_double(F, p):
    if p is None:
        return None
    X, Y, Z = p
    if Y == F.zero:
        return None
    A = F.sqr(X)
    Bq = F.sqr(Y)
    C = F.sqr(Bq)
    D = F.small(F.sub(F.sub(F.sqr(F.add(X, Bq)), A), C), 2)
    E = F.small(A, 3)
    Fv = F.sqr(E)
    X3 = F.sub(Fv, F.small(D, 2))
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), F.small(C, 8))
    Z3 = F.small(F.mul(Y, Z), 2)
    return (X3, Y3, Z3)


def _jac_add(F, p, q):
    if p is None:
        return q
    if q is None:
        return p
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    Z1Z1, Z2Z2 = F.sqr(Z1), F.sqr(Z2)
    U1, U2 = F.mul(X1, Z2Z2), F.mul(X2, Z1Z1)
    S1, S2 = F.mul(F.mul(Y1, Z2), Z2Z2), F.mul(F.mul(Y2, Z1), Z1Z1)
    if U1 == U2:
        return _jac_double(F, p) if S1 == S2 else None
    H = F.sub(U2, U1)
    I = F.sqr(F.small(H, 2))
    J = F.mul(H, I)
    r = F.small(F.sub(S2, S1), 2)
    V = F.mul(U1, I)
    X3 = F.sub(F.sub(F.sqr(r), J), F.small(V, 2))
    Y3 = F.sub(F.mul(r, F.sub(V, X3)), F.small(F.mul(S1, J), 2))
    Z3 = F.mul(F.sub(F.sub(F.sqr(F.add(Z1, Z2)), Z1Z1), Z2Z2), H)
    return (X3, Y3, Z3)


def _to_jac(F, pt):
    return None if pt is None else (pt[0], pt[1], F.one)


def _to_aff(F, p):
    if p is None:
        return None
    X, Y, Z = p
    zi = F.inv(Z)
    zi2 = F.sqr(zi)
    return (F.mul(X, zi2), F.mul(Y, F.mul(zi2, zi)))


def _mul(F, pt, k):
    acc = None
    q = _to_jac(F, pt)
    for bit in bin(k)[2:] if k > 0 else "":
        acc = _jac_double(F, acc)
        if bit == "1":
            acc = _jac_add(F, acc, q)
    return _to_aff(F, acc)


def g1_mul(pt, k):
    return _mul(_F1, pt, k)


def g2_mul(pt, k):
    return _mul(_F2, pt, k)


def g1_add(a, b):
    return _to_aff(_F1, _jac_add(_F1, _to_jac(_F1, a), _to_jac(_F1, b)))


def g2_add(a, b):
    return _to_aff(_F2, _jac_add(_F2, _to_jac(_F2, a), _to_jac(_F2, b)))


def g1_neg(a):
    return None if a is None else (a[0], (-a[1]) % P)


def g2_neg(a):
    return None if a is None else (a[0], f2_neg(a[1]))


G1 = (G1_X, G1_Y)
G2 = (G2_X, G2_Y)


# --------------------------------------------------------------------------- zcash encodings
def g1_compress(pt) -> bytes:
    if pt is None:
        out = bytearray(48)
        out[0] = 0xC0
        return bytes(out)
    x, y = pt
    out = bytearray(x.to_bytes(48, "big"))
    out[0] |= 0x80
    if y > (P - y) % P:
        out[0] |= 0x20
    return bytes(out)


def g1_decompress(b: bytes):
    if len(b) != 48 or not (b[0] & 0x80):
        raise ValueError("not a compressed G1 point")
    if b[0] & 0x40:
        if b[0] & 0x3F or any(b[1:]):
            raise ValueError("bad infinity encoding")
        return None
    greatest = bool(b[0] & 0x20)
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    if x >= P:
        raise ValueError("x not in field")
    y = fq_sqrt((x * x * x + B1) % P)
    if y is None:
        raise ValueError("not on curve")
    ny = (P - y) % P
    y = max(y, ny) if greatest else min(y, ny)
    pt = (x, y)
    if g1_mul(pt, R) is not None:
        raise ValueError("not in subgroup")
    return pt


def g2_compress(pt) -> bytes:
    if pt is None:
        out = bytearray(96)
        out[0] = 0xC0
        return bytes(out)
    x, y = pt
    out = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    out[0] |= 0x80
    if f2_gt(y, f2_neg(y)):
        out[0] |= 0x20
    return bytes(out)


def g2_decompress(b: bytes):
    if len(b) != 96 or not (b[0] & 0x80):
        raise ValueError("not a compressed G2 point")
    if b[0] & 0x40:
        # the crate: mask the two top flag bits, everything left must be zero
        if b[0] & 0x3F or any(b[1:]):
            raise ValueError("bad infinity encoding")
        return None
    greatest = bool(b[0] & 0x20)
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:], "big")
    if x0 >= P or x1 >= P:
        raise ValueError("x not in field")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise ValueError("not on curve")
    ny = f2_neg(y)
    if f2_gt(y, ny) != greatest:
        y = ny
    pt = (x, y)
    if g2_mul(pt, R) is not None:
        raise ValueError("not in subgroup")
    return pt


# --------------------------------------------------------------------------- pairing
def _doubling_step(r):
    """Algorithm 26 of eprint 2010/354 as in the crate's G2Prepared (Jacobian r)."""
    rx, ry, rz = r
    tmp0 = f2_sqr(rx)
    tmp1 = f2_sqr(ry)
    tmp2 = f2_sqr(tmp1)
    tmp3 = f2_sub(f2_sub(f2_sqr(f2_add(tmp1, rx)), tmp0), tmp2)
    tmp3 = f2_add(tmp3, tmp3)
    tmp4 = f2_add(f2_add(tmp0, tmp0), tmp0)
    tmp6 = f2_add(rx, tmp4)
    tmp5 = f2_sqr(tmp4)
    zsquared = f2_sqr(rz)
    nx = f2_sub(f2_sub(tmp5, tmp3), tmp3)
    nz = f2_sub(f2_sub(f2_sqr(f2_add(rz, ry)), tmp1), zsquared)
    ny = f2_mul(f2_sub(tmp3, nx), tmp4)
    tmp2 = f2_muls(tmp2, 8)
    ny = f2_sub(ny, tmp2)
    tmp3 = f2_neg(f2_muls(f2_mul(tmp4, zsquared), 2))
    tmp6 = f2_sub(f2_sub(f2_sqr(tmp6), tmp0), tmp5)
    tmp1 = f2_muls(tmp1, 4)
    tmp6 = f2_sub(tmp6, tmp1)
    tmp0 = f2_muls(f2_mul(nz, zsquared), 2)
    return (nx, ny, nz), (tmp0, tmp3, tmp6)


def _addition_step(r, q):
    """Algorithm 27 of eprint 2010/354 as in the crate's G2Prepared."""
    rx, ry, rz = r
    qx, qy = q
    zsquared = f2_sqr(rz)
    ysquared = f2_sqr(qy)
    t0 = f2_mul(zsquared, qx)
    t1 = f2_mul(f2_sub(f2_sub(f2_sqr(f2_add(qy, rz)), ysquared), zsquared), zsquared)
    t2 = f2_sub(t0, rx)
    t3 = f2_sqr(t2)
    t4 = f2_muls(t3, 4)
    t5 = f2_mul(t4, t2)
    t6 = f2_sub(f2_sub(t1, ry), ry)
    t9 = f2_mul(t6, qx)
    t7 = f2_mul(t4, rx)
    nx = f2_sub(f2_sub(f2_sub(f2_sqr(t6), t5), t7), t7)
    nz = f2_sub(f2_sub(f2_sqr(f2_add(rz, t2)), zsquared), t3)
    t10 = f2_add(qy, nz)
    t8 = f2_mul(f2_sub(t7, nx), t6)
    t0 = f2_muls(f2_mul(ry, t5), 2)
    ny = f2_sub(t8, t0)
    t10 = f2_sub(f2_sqr(t10), ysquared)
    ztsquared = f2_sqr(nz)
    t10 = f2_sub(t10, ztsquared)
    t9 = f2_sub(f2_muls(t9, 2), t10)
    t10 = f2_muls(nz, 2)
    t6 = f2_neg(t6)
    t1 = f2_muls(t6, 2)
    return (nx, ny, nz), (t10, t1, t9)


def _x_bits():
    bits = bin(BLS_X >> 1)[2:]
    return bits[1:]  # the crate skips up to and including the leading one


def g2_prepare(q):
    """G2Prepared::from_affine: list of (c0, c1, c2) Fq2 line coefficients."""
    if q is None:
        return None
    coeffs = []
    r = (q[0], q[1], F2_ONE)
    for bit in _x_bits():
        r, c = _doubling_step(r)
        coeffs.append(c)
        if bit == "1":
            r, c = _addition_step(r, q)
            coeffs.append(c)
    r, c = _doubling_step(r)
    coeffs.append(c)
    return coeffs


def _ell(f, coeffs, p):
    c0, c1, c2 = coeffs
    c0 = f2_muls(c0, p[1])
    c1 = f2_muls(c1, p[0])
    return f12_mul_by_014(f, c2, c1, c0)


def miller_loop(pairs):
    """pairs: [(G1 affine, G2Prepared)]; the crate's Bls12::miller_loop."""
    live = [(p, iter(qc)) for p, qc in pairs if p is not None and qc is not None]
    f = F12_ONE
    for bit in _x_bits():
        for p, it in live:
            f = _ell(f, next(it), p)
        if bit == "1":
            for p, it in live:
                f = _ell(f, next(it), p)
        f = f12_sqr(f)
    for p, it in live:
        f = _ell(f, next(it), p)
    if BLS_X_IS_NEGATIVE:
        f = f12_conj(f)
    return f


def _exp_by_x(f):
    f = f12_pow(f, BLS_X)
    return f12_conj(f) if BLS_X_IS_NEGATIVE else f


def final_exponentiation(r):
    """The crate's final_exponentiation (easy part + exp_by_x chain)."""
    f1 = f12_conj(r)
    f2_ = f12_inv(r)
    r = f12_mul(f1, f2_)
    f2_ = r
    r = f12_frob(r, 2)
    r = f12_mul(r, f2_)
    y0 = f12_sqr(r)
    y1 = _exp_by_x(y0)
    # x >>= 1 (for the exponent only)
    y2 = f12_pow(y1, BLS_X >> 1)
    y2 = f12_conj(y2)
    y3 = f12_conj(r)
    y1 = f12_mul(y1, y3)
    y1 = f12_conj(y1)
    y1 = f12_mul(y1, y2)
    y2 = _exp_by_x(y1)
    y3 = _exp_by_x(y2)
    y1 = f12_conj(y1)
    y3 = f12_mul(y3, y1)
    y1 = f12_conj(y1)
    y1 = f12_frob(y1, 3)
    y2 = f12_frob(y2, 2)
    y1 = f12_mul(y1, y2)
    y2 = _exp_by_x(y3)
    y2 = f12_mul(y2, y0)
    y2 = f12_mul(y2, r)
    y1 = f12_mul(y1, y2)
    y2 = f12_frob(y3, 1)
    y1 = f12_mul(y1, y2)
    return y1


def final_exponentiation_plain(f):
    return f12_pow(f, (P ** 12 - 1) // R)


def pairing(p, q):
    return final_exponentiation(miller_loop([(p, g2_prepare(q))]))


def pairing_check(pairs) -> bool:
    """prod e(P_i, Q_i) == 1 via one multi-Miller loop + one final exp."""
    return final_exponentiation(miller_loop([(p, g2_prepare(q)) for p, q in pairs])) == F12_ONE


# --------------------------------------------------------------------------- Montgomery views (rand sampling)
def fq_from_mont_repr(repr_int: int) -> int:
    """The crate stores Fq in Montgomery form: Fq(repr) has value repr * R^-1."""
    return repr_int * R_MONT_INV % P


def g2_scale_by_cofactor(pt):
    return g2_mul(pt, G2_COFACTOR)


def g2_get_point_from_x(x, greatest):
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        return None
    ny = f2_neg(y)
    # the crate: y if (y < negy) ^ greatest else negy
    return (x, y if (f2_gt(ny, y)) ^ greatest else ny)
