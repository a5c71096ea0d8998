/* bls_oracle.c — C restatement of threshold_crypto's ThresholdDecrypt path
 * (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).
 *
 * The same algorithm as oracle/bls12_381.py + oracle/tcrypto.py (pairing crate
 * bls12_381 [EXT], threshold_crypto 0.3-era [EXT]),
 * written the way the reference crates run it on a CPU so that bench.py can
 * time a fair host baseline ("port") and tests can check the GPU at sizes the
 * Python oracle is too slow for:
 *
 *  * Fq: 6 x 64-bit limbs, Montgomery R = 2^384 (the crate's domain and limb
 *    size), CIOS multiplication; Fr: 4 x 64-bit, R = 2^256.
 *  * Fq2/Fq6/Fq12 tower, G2Prepared (eprint 2010/354 Alg. 26/27),
 *    Miller loop with the crate's sparse mul_by_014, the crate's
 *    final-exponentiation chain (exp_by_x by square-and-multiply).
 *  * Decoding checks subgroup membership by [r]P == O, as the crate's
 *    `into_affine` does.
 *  * PublicKeyShare::verify_decryption_share exactly as threshold_crypto:
 *    H = hash_g1_g2(U, V) per call, then pairing(share, H) == pairing(pk_i, W)
 *    — two full pairings (two final exponentiations) per share.
 *  * PublicKeySet::decrypt: Lagrange at 0 over the first t+1 shares (one Fr
 *    inversion per coefficient), per-share scalar multiplication, sum,
 *    xor_with_hash.
 *
 * Pinned in tests/test_oracle_tdec.py against the Python oracle and the
 * committed golden fixtures (tests/golden/tdec_*.json).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t l[6]; } fp;
typedef struct { fp c0, c1; } fp2;
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
typedef struct { uint64_t l[4]; } fr;

#include "bls_consts_c.h"

void orc_sha3_256(const uint8_t *in, uint64_t len, uint8_t out[32]); /* rbc_oracle.c */

/* ------------------------------------------------------------------ Fq */
static inline int geq_n(const uint64_t *a, const uint64_t *m, int n) {
    for (int i = n - 1; i >= 0; --i) {
        if (a[i] != m[i]) return a[i] > m[i];
    }
    return 1;
}
static inline void sub_n(uint64_t *a, const uint64_t *m, int n) {
    u128 br = 0;
    for (int i = 0; i < n; ++i) {
        u128 t = (u128)a[i] - m[i] - br;
        a[i] = (uint64_t)t;
        br = (t >> 64) ? 1 : 0;
    }
}
/* CIOS Montgomery product, n limbs (n <= 6), result < m */
static inline __attribute__((always_inline)) void mont_mul_n(uint64_t *r, const uint64_t *a, const uint64_t *b, const uint64_t *m, uint64_t minv, int n) {
    uint64_t t[8] = {0};
    for (int i = 0; i < n; ++i) {
        u128 c = 0;
        for (int j = 0; j < n; ++j) {
            c += (u128)a[j] * b[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        c += t[n];
        t[n] = (uint64_t)c;
        t[n + 1] = (uint64_t)(c >> 64);
        const uint64_t q = t[0] * minv;
        c = (u128)q * m[0] + t[0];
        c >>= 64;
        for (int j = 1; j < n; ++j) {
            c += (u128)q * m[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[n];
        t[n - 1] = (uint64_t)c;
        t[n] = t[n + 1] + (uint64_t)(c >> 64);
    }
    if (t[n] || geq_n(t, m, n)) sub_n(t, m, n);
    memcpy(r, t, 8 * n);
}

/* The crate's Fq::mul_assign: 6x6 schoolbook into 12 limbs (mac_with_carry),
 * then mont_reduce — fully unrolled by the compiler. */
static inline uint64_t mac(uint64_t a, uint64_t b, uint64_t c, uint64_t *carry) {
    u128 t = (u128)b * c + a + *carry;
    *carry = (uint64_t)(t >> 64);
    return (uint64_t)t;
}
static inline uint64_t adc(uint64_t a, uint64_t b, uint64_t *carry) {
    u128 t = (u128)a + b + *carry;
    *carry = (uint64_t)(t >> 64);
    return (uint64_t)t;
}
static inline fp fp_mul(fp a, fp b) {
    uint64_t t[12] = {0};
    for (int i = 0; i < 6; ++i) {
        uint64_t c = 0;
        for (int j = 0; j < 6; ++j) t[i + j] = mac(t[i + j], a.l[i], b.l[j], &c);
        t[i + 6] = c;
    }
    uint64_t c2 = 0;
    for (int i = 0; i < 6; ++i) {
        const uint64_t k = t[i] * kPInv;
        uint64_t c = 0;
        (void)mac(t[i], k, kP[0], &c);
        for (int j = 1; j < 6; ++j) t[i + j] = mac(t[i + j], k, kP[j], &c);
        t[i + 6] = adc(t[i + 6], c2, &c);
        c2 = c;
    }
    fp r;
    for (int i = 0; i < 6; ++i) r.l[i] = t[6 + i];
    if (geq_n(r.l, kP, 6)) sub_n(r.l, kP, 6);
    return r;
}
static inline fp fp_sqr(fp a) { return fp_mul(a, a); }
static inline fp fp_add(fp a, fp b) {
    fp r;
    u128 c = 0;
    for (int i = 0; i < 6; ++i) { c += (u128)a.l[i] + b.l[i]; r.l[i] = (uint64_t)c; c >>= 64; }
    if (c || geq_n(r.l, kP, 6)) sub_n(r.l, kP, 6);
    return r;
}
static inline fp fp_sub(fp a, fp b) {
    fp r;
    u128 br = 0;
    for (int i = 0; i < 6; ++i) { u128 t = (u128)a.l[i] - b.l[i] - br; r.l[i] = (uint64_t)t; br = (t >> 64) ? 1 : 0; }
    if (br) {
        u128 c = 0;
        for (int i = 0; i < 6; ++i) { c += (u128)r.l[i] + kP[i]; r.l[i] = (uint64_t)c; c >>= 64; }
    }
    return r;
}
static const fp FP_ZERO = {{0, 0, 0, 0, 0, 0}};
static inline fp fp_neg(fp a) { return fp_sub(FP_ZERO, a); }
static inline fp fp_dbl(fp a) { return fp_add(a, a); }
static inline int fp_is_zero(fp a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3] | a.l[4] | a.l[5]) == 0; }
static inline int fp_eq(fp a, fp b) { return memcmp(&a, &b, sizeof a) == 0; }
static fp fp_pow(fp a, const uint64_t *e, int n) {
    fp r = kOneQ;
    int started = 0;
    for (int i = 64 * n - 1; i >= 0; --i) {
        if (started) r = fp_sqr(r);
        if ((e[i >> 6] >> (i & 63)) & 1) { r = started ? fp_mul(r, a) : a; started = 1; }
    }
    return r;
}
static inline fp fp_inv(fp a) { return fp_pow(a, kExpInv, 6); }
static fp fp_from_canon(const uint64_t c[6]) { fp t; memcpy(t.l, c, 48); fp r2; memcpy(r2.l, kR2q, 48); return fp_mul(t, r2); }
static void fp_to_canon(fp a, uint64_t out[6]) { fp one = {{1, 0, 0, 0, 0, 0}}; fp r = fp_mul(a, one); memcpy(out, r.l, 48); }
static int canon_gt(const uint64_t *a, const uint64_t *b) {
    for (int i = 5; i >= 0; --i) if (a[i] != b[i]) return a[i] > b[i];
    return 0;
}
static int fp_gt(fp a, fp b) { uint64_t x[6], y[6]; fp_to_canon(a, x); fp_to_canon(b, y); return canon_gt(x, y); }
static int be48_to_canon(const uint8_t *b, uint64_t out[6], uint8_t top_mask) {
    for (int i = 0; i < 6; ++i) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) {
            uint8_t byte = b[8 * (5 - i) + j];
            if (i == 5 && j == 0) byte &= top_mask;
            w = (w << 8) | byte;
        }
        out[i] = w;
    }
    return !geq_n(out, kP, 6); /* 1 iff < p */
}
static void canon_to_be48(const uint64_t c[6], uint8_t *b) {
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 8; ++j) b[8 * (5 - i) + j] = (uint8_t)(c[i] >> (8 * (7 - j)));
}

/* ------------------------------------------------------------------ Fq2 */
static const fp2 FP2_ZERO = {{{0}}, {{0}}};
static inline fp2 fp2_one(void) { fp2 r = {kOneQ, FP_ZERO}; return r; }
static inline fp2 fp2_add(fp2 a, fp2 b) { fp2 r = {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; return r; }
static inline fp2 fp2_sub(fp2 a, fp2 b) { fp2 r = {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; return r; }
static inline fp2 fp2_neg(fp2 a) { fp2 r = {fp_neg(a.c0), fp_neg(a.c1)}; return r; }
static inline fp2 fp2_dbl(fp2 a) { return fp2_add(a, a); }
static inline fp2 fp2_mul(fp2 a, fp2 b) {
    fp t0 = fp_mul(a.c0, b.c0), t1 = fp_mul(a.c1, b.c1);
    fp2 r = {fp_sub(t0, t1), fp_sub(fp_sub(fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1)), t0), t1)};
    return r;
}
static inline fp2 fp2_sqr(fp2 a) {
    fp2 r = {fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1)), fp_dbl(fp_mul(a.c0, a.c1))};
    return r;
}
static inline fp2 fp2_muls(fp2 a, fp s) { fp2 r = {fp_mul(a.c0, s), fp_mul(a.c1, s)}; return r; }
static inline fp2 fp2_conj(fp2 a) { fp2 r = {a.c0, fp_neg(a.c1)}; return r; }
static inline fp2 fp2_mul_xi(fp2 a) { fp2 r = {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; return r; }
static inline int fp2_is_zero(fp2 a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
static inline int fp2_eq(fp2 a, fp2 b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
static fp2 fp2_inv(fp2 a) {
    fp t = fp_inv(fp_add(fp_sqr(a.c0), fp_sqr(a.c1)));
    fp2 r = {fp_mul(a.c0, t), fp_neg(fp_mul(a.c1, t))};
    return r;
}
static fp2 fp2_pow(fp2 a, const uint64_t *e, int n) {
    fp2 r = fp2_one();
    int started = 0;
    for (int i = 64 * n - 1; i >= 0; --i) {
        if (started) r = fp2_sqr(r);
        if ((e[i >> 6] >> (i & 63)) & 1) { r = started ? fp2_mul(r, a) : a; started = 1; }
    }
    return r;
}
static int fp2_gt(fp2 a, fp2 b) { /* the crate's Ord: c1 first, then c0 */
    if (!fp_eq(a.c1, b.c1)) return fp_gt(a.c1, b.c1);
    return fp_gt(a.c0, b.c0);
}
/* Algorithm 9 of eprint 2012/685 (the crate's Fq2::sqrt); returns 0 if none */
static int fp2_sqrt(fp2 a, fp2 *out) {
    if (fp2_is_zero(a)) { *out = FP2_ZERO; return 1; }
    fp2 a1 = fp2_pow(a, kExpP34, 6);
    fp2 alpha = fp2_mul(fp2_sqr(a1), a);
    fp2 a0 = fp2_mul(fp2_conj(alpha), alpha);
    fp2 m1 = {fp_neg(kOneQ), FP_ZERO};
    if (fp2_eq(a0, m1)) return 0;
    a1 = fp2_mul(a1, a);
    if (fp2_eq(alpha, m1)) {
        fp2 u = {FP_ZERO, kOneQ};
        *out = fp2_mul(a1, u);
        return 1;
    }
    fp2 b = fp2_pow(fp2_add(alpha, fp2_one()), kExpP12, 6);
    *out = fp2_mul(a1, b);
    return 1;
}

/* ------------------------------------------------------------------ Fq6 / Fq12 */
static inline fp6 fp6_add(fp6 a, fp6 b) { fp6 r = {fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; return r; }
static inline fp6 fp6_sub(fp6 a, fp6 b) { fp6 r = {fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; return r; }
static inline fp6 fp6_neg(fp6 a) { fp6 r = {fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; return r; }
static fp6 fp6_mul(fp6 a, fp6 b) {
    fp2 t0 = fp2_mul(a.c0, b.c0), t1 = fp2_mul(a.c1, b.c1), t2 = fp2_mul(a.c2, b.c2);
    fp6 r;
    r.c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), fp2_add(t1, t2))));
    r.c1 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
    r.c2 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), fp2_add(t0, t2)), t1);
    return r;
}
static inline fp6 fp6_mul_by_v(fp6 a) { fp6 r = {fp2_mul_xi(a.c2), a.c0, a.c1}; return r; }
static fp6 fp6_mul_by_01(fp6 a, fp2 c0, fp2 c1) {
    fp2 aa = fp2_mul(a.c0, c0), bb = fp2_mul(a.c1, c1);
    fp6 r;
    r.c0 = fp2_add(fp2_mul_xi(fp2_mul(a.c2, c1)), aa);
    r.c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(c0, c1), fp2_add(a.c0, a.c1)), aa), bb);
    r.c2 = fp2_add(fp2_mul(a.c2, c0), bb);
    return r;
}
static fp6 fp6_mul_by_1(fp6 a, fp2 c1) {
    fp6 r = {fp2_mul_xi(fp2_mul(a.c2, c1)), fp2_mul(a.c0, c1), fp2_mul(a.c1, c1)};
    return r;
}
static fp6 fp6_inv(fp6 a) {
    fp2 c0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
    fp2 c1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
    fp2 c2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
    fp2 t = fp2_add(fp2_mul(a.c0, c0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, c1), fp2_mul(a.c1, c2))));
    fp2 ti = fp2_inv(t);
    fp6 r = {fp2_mul(c0, ti), fp2_mul(c1, ti), fp2_mul(c2, ti)};
    return r;
}
static fp12 fp12_one(void) {
    fp12 r;
    memset(&r, 0, sizeof r);
    r.c0.c0.c0 = kOneQ;
    return r;
}
static fp12 fp12_mul(fp12 a, fp12 b) {
    fp6 t0 = fp6_mul(a.c0, b.c0), t1 = fp6_mul(a.c1, b.c1);
    fp12 r;
    r.c1 = fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), fp6_add(t0, t1));
    r.c0 = fp6_add(t0, fp6_mul_by_v(t1));
    return r;
}
static fp12 fp12_sqr(fp12 a) { /* the crate's complex squaring */
    fp6 ab = fp6_mul(a.c0, a.c1);
    fp6 c0c1 = fp6_add(a.c0, a.c1);
    fp6 c0 = fp6_add(fp6_mul_by_v(a.c1), a.c0);
    c0 = fp6_sub(fp6_sub(fp6_mul(c0, c0c1), ab), fp6_mul_by_v(ab));
    fp12 r = {c0, fp6_add(ab, ab)};
    return r;
}
static inline fp12 fp12_conj(fp12 a) { fp12 r = {a.c0, fp6_neg(a.c1)}; return r; }
static fp12 fp12_inv(fp12 a) {
    fp6 t = fp6_inv(fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_by_v(fp6_mul(a.c1, a.c1))));
    fp12 r = {fp6_mul(a.c0, t), fp6_neg(fp6_mul(a.c1, t))};
    return r;
}
static fp12 fp12_frob(fp12 a, int k) {
    const fp2 *g61 = k == 1 ? &kG61_1 : k == 2 ? &kG61_2 : &kG61_3;
    const fp2 *g62 = k == 1 ? &kG62_1 : k == 2 ? &kG62_2 : &kG62_3;
    const fp2 *g12 = k == 1 ? &kG12_1 : k == 2 ? &kG12_2 : &kG12_3;
    fp2 (*fr)(fp2) = (k & 1) ? fp2_conj : NULL;
#define FR(x) (fr ? fr(x) : (x))
    fp12 r;
    r.c0.c0 = FR(a.c0.c0);
    r.c0.c1 = fp2_mul(FR(a.c0.c1), *g61);
    r.c0.c2 = fp2_mul(FR(a.c0.c2), *g62);
    r.c1.c0 = fp2_mul(FR(a.c1.c0), *g12);
    r.c1.c1 = fp2_mul(fp2_mul(FR(a.c1.c1), *g61), *g12);
    r.c1.c2 = fp2_mul(fp2_mul(FR(a.c1.c2), *g62), *g12);
#undef FR
    return r;
}
static fp12 fp12_mul_by_014(fp12 f, fp2 c0, fp2 c1, fp2 c4) {
    fp6 aa = fp6_mul_by_01(f.c0, c0, c1);
    fp6 bb = fp6_mul_by_1(f.c1, c4);
    fp2 o = fp2_add(c1, c4);
    fp12 r;
    r.c1 = fp6_sub(fp6_sub(fp6_mul_by_01(fp6_add(f.c1, f.c0), c0, o), aa), bb);
    r.c0 = fp6_add(fp6_mul_by_v(bb), aa);
    return r;
}
static int fp12_is_one(fp12 a) {
    fp12 o = fp12_one();
    return memcmp(&a, &o, sizeof a) == 0;
}
static fp12 fp12_pow_u64(fp12 a, uint64_t e) {
    fp12 r = fp12_one();
    int started = 0;
    for (int i = 63; i >= 0; --i) {
        if (started) r = fp12_sqr(r);
        if ((e >> i) & 1) { r = started ? fp12_mul(r, a) : a; started = 1; }
    }
    return r;
}

/* ------------------------------------------------------------------ curves (Jacobian, Z == 0 <=> O) */
#define BLS_X 0xd201000000010000ull
typedef struct { fp x, y, z; } g1;
typedef struct { fp2 x, y, z; } g2;

static g1 g1_dbl(g1 p) {
    if (fp_is_zero(p.z) || fp_is_zero(p.y)) { g1 o = {kOneQ, kOneQ, FP_ZERO}; return o; }
    fp A = fp_sqr(p.x), B = fp_sqr(p.y), C = fp_sqr(B);
    fp D = fp_dbl(fp_sub(fp_sub(fp_sqr(fp_add(p.x, B)), A), C));
    fp E = fp_add(fp_dbl(A), A), F = fp_sqr(E);
    g1 r;
    r.x = fp_sub(F, fp_dbl(D));
    r.y = fp_sub(fp_mul(E, fp_sub(D, r.x)), fp_dbl(fp_dbl(fp_dbl(C))));
    r.z = fp_dbl(fp_mul(p.y, p.z));
    return r;
}
static g1 g1_add(g1 p, g1 q) {
    if (fp_is_zero(p.z)) return q;
    if (fp_is_zero(q.z)) return p;
    fp Z1Z1 = fp_sqr(p.z), Z2Z2 = fp_sqr(q.z);
    fp U1 = fp_mul(p.x, Z2Z2), U2 = fp_mul(q.x, Z1Z1);
    fp S1 = fp_mul(fp_mul(p.y, q.z), Z2Z2), S2 = fp_mul(fp_mul(q.y, p.z), Z1Z1);
    if (fp_eq(U1, U2)) {
        if (fp_eq(S1, S2)) return g1_dbl(p);
        g1 o = {kOneQ, kOneQ, FP_ZERO};
        return o;
    }
    fp H = fp_sub(U2, U1), I = fp_sqr(fp_dbl(H)), J = fp_mul(H, I);
    fp rr = fp_dbl(fp_sub(S2, S1)), V = fp_mul(U1, I);
    g1 r;
    r.x = fp_sub(fp_sub(fp_sqr(rr), J), fp_dbl(V));
    r.y = fp_sub(fp_mul(rr, fp_sub(V, r.x)), fp_dbl(fp_mul(S1, J)));
    r.z = fp_mul(fp_sub(fp_sub(fp_sqr(fp_add(p.z, q.z)), Z1Z1), Z2Z2), H);
    return r;
}
static g1 g1_mul(g1 p, const uint64_t *k, int n) {
    g1 r = {kOneQ, kOneQ, FP_ZERO};
    for (int i = 64 * n - 1; i >= 0; --i) {
        r = g1_dbl(r);
        if ((k[i >> 6] >> (i & 63)) & 1) r = g1_add(r, p);
    }
    return r;
}
static int g1_to_affine(g1 p, fp *x, fp *y) {
    if (fp_is_zero(p.z)) return 0;
    fp zi = fp_inv(p.z), zi2 = fp_sqr(zi);
    *x = fp_mul(p.x, zi2);
    *y = fp_mul(p.y, fp_mul(zi2, zi));
    return 1;
}
static g2 g2_dbl(g2 p) {
    if (fp2_is_zero(p.z) || fp2_is_zero(p.y)) { g2 o = {fp2_one(), fp2_one(), FP2_ZERO}; return o; }
    fp2 A = fp2_sqr(p.x), B = fp2_sqr(p.y), C = fp2_sqr(B);
    fp2 D = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.x, B)), A), C));
    fp2 E = fp2_add(fp2_dbl(A), A), F = fp2_sqr(E);
    g2 r;
    r.x = fp2_sub(F, fp2_dbl(D));
    r.y = fp2_sub(fp2_mul(E, fp2_sub(D, r.x)), fp2_dbl(fp2_dbl(fp2_dbl(C))));
    r.z = fp2_dbl(fp2_mul(p.y, p.z));
    return r;
}
static g2 g2_add(g2 p, g2 q) {
    if (fp2_is_zero(p.z)) return q;
    if (fp2_is_zero(q.z)) return p;
    fp2 Z1Z1 = fp2_sqr(p.z), Z2Z2 = fp2_sqr(q.z);
    fp2 U1 = fp2_mul(p.x, Z2Z2), U2 = fp2_mul(q.x, Z1Z1);
    fp2 S1 = fp2_mul(fp2_mul(p.y, q.z), Z2Z2), S2 = fp2_mul(fp2_mul(q.y, p.z), Z1Z1);
    if (fp2_eq(U1, U2)) {
        if (fp2_eq(S1, S2)) return g2_dbl(p);
        g2 o = {fp2_one(), fp2_one(), FP2_ZERO};
        return o;
    }
    fp2 H = fp2_sub(U2, U1), I = fp2_sqr(fp2_dbl(H)), J = fp2_mul(H, I);
    fp2 rr = fp2_dbl(fp2_sub(S2, S1)), V = fp2_mul(U1, I);
    g2 r;
    r.x = fp2_sub(fp2_sub(fp2_sqr(rr), J), fp2_dbl(V));
    r.y = fp2_sub(fp2_mul(rr, fp2_sub(V, r.x)), fp2_dbl(fp2_mul(S1, J)));
    r.z = fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.z, q.z)), Z1Z1), Z2Z2), H);
    return r;
}
static g2 g2_mul(g2 p, const uint64_t *k, int n) {
    g2 r = {fp2_one(), fp2_one(), FP2_ZERO};
    for (int i = 64 * n - 1; i >= 0; --i) {
        r = g2_dbl(r);
        if ((k[i >> 6] >> (i & 63)) & 1) r = g2_add(r, p);
    }
    return r;
}
static int g2_to_affine(g2 p, fp2 *x, fp2 *y) {
    if (fp2_is_zero(p.z)) return 0;
    fp2 zi = fp2_inv(p.z), zi2 = fp2_sqr(zi);
    *x = fp2_mul(p.x, zi2);
    *y = fp2_mul(p.y, fp2_mul(zi2, zi));
    return 1;
}

/* zcash encodings.  Return 1 ok (inf set for the identity), 0 invalid. */
static int g1_decompress(const uint8_t *b, fp *x, fp *y, int *inf, int check_subgroup) {
    *inf = 0;
    if (!(b[0] & 0x80)) return 0;
    if (b[0] & 0x40) {
        if (b[0] & 0x3F) return 0;
        for (int i = 1; i < 48; ++i) if (b[i]) return 0;
        *inf = 1;
        return 1;
    }
    uint64_t c[6];
    if (!be48_to_canon(b, c, 0x1F)) return 0;
    *x = fp_from_canon(c);
    fp rhs = fp_add(fp_mul(fp_sqr(*x), *x), kFour);
    fp s = fp_pow(rhs, kExpSqrt, 6);
    if (!fp_eq(fp_sqr(s), rhs)) return 0;
    fp ns = fp_neg(s);
    const int greatest = (b[0] & 0x20) != 0;
    *y = (fp_gt(s, ns) == greatest) ? s : ns;
    if (!check_subgroup) return 1;
    g1 p = {*x, *y, kOneQ};
    g1 t = g1_mul(p, kR, 4);
    return fp_is_zero(t.z);
}
static void g1_compress(fp x, fp y, int inf, uint8_t *b) {
    if (inf) { memset(b, 0, 48); b[0] = 0xC0; return; }
    uint64_t c[6];
    fp_to_canon(x, c);
    canon_to_be48(c, b);
    b[0] |= 0x80;
    if (fp_gt(y, fp_neg(y))) b[0] |= 0x20;
}
static int g2_decompress(const uint8_t *b, fp2 *x, fp2 *y, int *inf) {
    *inf = 0;
    if (!(b[0] & 0x80)) return 0;
    if (b[0] & 0x40) {
        if (b[0] & 0x3F) return 0;
        for (int i = 1; i < 96; ++i) if (b[i]) return 0;
        *inf = 1;
        return 1;
    }
    uint64_t c1[6], c0[6];
    if (!be48_to_canon(b, c1, 0x1F)) return 0;
    if (!be48_to_canon(b + 48, c0, 0xFF)) return 0;
    x->c0 = fp_from_canon(c0);
    x->c1 = fp_from_canon(c1);
    fp2 b2 = {kFour, kFour};
    fp2 s;
    if (!fp2_sqrt(fp2_add(fp2_mul(fp2_sqr(*x), *x), b2), &s)) return 0;
    fp2 ns = fp2_neg(s);
    const int greatest = (b[0] & 0x20) != 0;
    *y = (fp2_gt(s, ns) != greatest) ? ns : s;
    g2 p = {*x, *y, fp2_one()};
    g2 t = g2_mul(p, kR, 4);
    return fp2_is_zero(t.z);
}

/* ------------------------------------------------------------------ pairing */
typedef struct { fp2 c0, c1, c2; } line;
#define N_LINES 68
static line doubling_step(g2 *r) {
    fp2 tmp0 = fp2_sqr(r->x), tmp1 = fp2_sqr(r->y), tmp2 = fp2_sqr(tmp1);
    fp2 tmp3 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(tmp1, r->x)), tmp0), tmp2);
    tmp3 = fp2_dbl(tmp3);
    fp2 tmp4 = fp2_add(fp2_dbl(tmp0), tmp0);
    fp2 tmp6 = fp2_add(r->x, tmp4);
    fp2 tmp5 = fp2_sqr(tmp4);
    fp2 zsq = fp2_sqr(r->z);
    g2 n;
    n.x = fp2_sub(fp2_sub(tmp5, tmp3), tmp3);
    n.z = fp2_sub(fp2_sub(fp2_sqr(fp2_add(r->z, r->y)), tmp1), zsq);
    n.y = fp2_mul(fp2_sub(tmp3, n.x), tmp4);
    tmp2 = fp2_dbl(fp2_dbl(fp2_dbl(tmp2)));
    n.y = fp2_sub(n.y, tmp2);
    tmp3 = fp2_neg(fp2_dbl(fp2_mul(tmp4, zsq)));
    tmp6 = fp2_sub(fp2_sub(fp2_sqr(tmp6), tmp0), tmp5);
    tmp1 = fp2_dbl(fp2_dbl(tmp1));
    tmp6 = fp2_sub(tmp6, tmp1);
    tmp0 = fp2_dbl(fp2_mul(n.z, zsq));
    *r = n;
    line c = {tmp0, tmp3, tmp6};
    return c;
}
static line addition_step(g2 *r, fp2 qx, fp2 qy) {
    fp2 zsq = fp2_sqr(r->z), ysq = fp2_sqr(qy);
    fp2 t0 = fp2_mul(zsq, qx);
    fp2 t1 = fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(qy, r->z)), ysq), zsq), zsq);
    fp2 t2 = fp2_sub(t0, r->x);
    fp2 t3 = fp2_sqr(t2);
    fp2 t4 = fp2_dbl(fp2_dbl(t3));
    fp2 t5 = fp2_mul(t4, t2);
    fp2 t6 = fp2_sub(fp2_sub(t1, r->y), r->y);
    fp2 t9 = fp2_mul(t6, qx);
    fp2 t7 = fp2_mul(t4, r->x);
    g2 n;
    n.x = fp2_sub(fp2_sub(fp2_sub(fp2_sqr(t6), t5), t7), t7);
    n.z = fp2_sub(fp2_sub(fp2_sqr(fp2_add(r->z, t2)), zsq), t3);
    fp2 t10 = fp2_add(qy, n.z);
    fp2 t8 = fp2_mul(fp2_sub(t7, n.x), t6);
    t0 = fp2_dbl(fp2_mul(r->y, t5));
    n.y = fp2_sub(t8, t0);
    t10 = fp2_sub(fp2_sqr(t10), ysq);
    fp2 ztsq = fp2_sqr(n.z);
    t10 = fp2_sub(t10, ztsq);
    t9 = fp2_sub(fp2_dbl(t9), t10);
    t10 = fp2_dbl(n.z);
    t6 = fp2_neg(t6);
    t1 = fp2_dbl(t6);
    *r = n;
    line c = {t10, t1, t9};
    return c;
}
static void g2_prepare(fp2 qx, fp2 qy, line *out) {
    g2 r = {qx, qy, fp2_one()};
    int k = 0;
    const uint64_t xh = BLS_X >> 1;
    for (int i = 61; i >= 0; --i) {
        out[k++] = doubling_step(&r);
        if ((xh >> i) & 1) out[k++] = addition_step(&r, qx, qy);
    }
    out[k++] = doubling_step(&r);
}
static fp12 ell(fp12 f, const line *c, fp px, fp py) {
    return fp12_mul_by_014(f, c->c2, fp2_muls(c->c1, px), fp2_muls(c->c0, py));
}
/* Miller loop over up to two (G1 affine, prepared G2) pairs */
static fp12 miller_loop(int np, const fp *px, const fp *py, line *const *lines) {
    fp12 f = fp12_one();
    int k = 0;
    const uint64_t xh = BLS_X >> 1;
    for (int i = 61; i >= 0; --i) {
        for (int j = 0; j < np; ++j) f = ell(f, &lines[j][k], px[j], py[j]);
        ++k;
        if ((xh >> i) & 1) {
            for (int j = 0; j < np; ++j) f = ell(f, &lines[j][k], px[j], py[j]);
            ++k;
        }
        f = fp12_sqr(f);
    }
    for (int j = 0; j < np; ++j) f = ell(f, &lines[j][k], px[j], py[j]);
    return fp12_conj(f);
}
static fp12 exp_by_x(fp12 f) { return fp12_conj(fp12_pow_u64(f, BLS_X)); }
static fp12 final_exponentiation(fp12 r) {
    fp12 f1 = fp12_conj(r), f2 = fp12_inv(r);
    r = fp12_mul(f1, f2);
    f2 = r;
    r = fp12_mul(fp12_frob(r, 2), f2);
    fp12 y0 = fp12_sqr(r);
    fp12 y1 = exp_by_x(y0);
    fp12 y2 = fp12_conj(fp12_pow_u64(y1, BLS_X >> 1));
    fp12 y3 = fp12_conj(r);
    y1 = fp12_conj(fp12_mul(y1, y3));
    y1 = fp12_mul(y1, y2);
    y2 = exp_by_x(y1);
    y3 = exp_by_x(y2);
    y1 = fp12_conj(y1);
    y3 = fp12_mul(y3, y1);
    y1 = fp12_conj(y1);
    y1 = fp12_frob(y1, 3);
    y2 = fp12_frob(y2, 2);
    y1 = fp12_mul(y1, y2);
    y2 = exp_by_x(y3);
    y2 = fp12_mul(y2, y0);
    y2 = fp12_mul(y2, r);
    y1 = fp12_mul(y1, y2);
    y2 = fp12_frob(y3, 1);
    return fp12_mul(y1, y2);
}
/* e(P, Q) as the crate's Engine::pairing (identity -> 1) */
static fp12 pairing(fp px, fp py, int p_inf, fp2 qx, fp2 qy, int q_inf) {
    if (p_inf || q_inf) return fp12_one();
    line *ln = (line *)malloc(sizeof(line) * N_LINES);
    g2_prepare(qx, qy, ln);
    line *const ls[1] = {ln};
    fp12 f = final_exponentiation(miller_loop(1, &px, &py, ls));
    free(ln);
    return f;
}

/* ------------------------------------------------------------------ ChaCha20 / hash_g2 */
typedef struct { uint32_t key[8]; uint64_t ctr; uint32_t buf[16]; int idx; } chacha;
#define ROTL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))
#define QR(a, b, c, d) a += b; d = ROTL(d ^ a, 16); c += d; b = ROTL(b ^ c, 12); a += b; d = ROTL(d ^ a, 8); c += d; b = ROTL(b ^ c, 7);
static void chacha_init(chacha *s, const uint8_t seed[32]) {
    for (int i = 0; i < 8; ++i) s->key[i] = (uint32_t)seed[4 * i] | (uint32_t)seed[4 * i + 1] << 8 | (uint32_t)seed[4 * i + 2] << 16 | (uint32_t)seed[4 * i + 3] << 24;
    s->ctr = 0;
    s->idx = 16;
}
static uint32_t chacha_u32(chacha *s) {
    if (s->idx >= 16) {
        uint32_t st[16] = {0x61707865, 0x3320646E, 0x79622D32, 0x6B206574};
        memcpy(st + 4, s->key, 32);
        st[12] = (uint32_t)s->ctr;
        st[13] = (uint32_t)(s->ctr >> 32);
        st[14] = st[15] = 0;
        uint32_t w[16];
        memcpy(w, st, 64);
        for (int r = 0; r < 10; ++r) {
            QR(w[0], w[4], w[8], w[12]) QR(w[1], w[5], w[9], w[13]) QR(w[2], w[6], w[10], w[14]) QR(w[3], w[7], w[11], w[15])
            QR(w[0], w[5], w[10], w[15]) QR(w[1], w[6], w[11], w[12]) QR(w[2], w[7], w[8], w[13]) QR(w[3], w[4], w[9], w[14])
        }
        for (int i = 0; i < 16; ++i) s->buf[i] = w[i] + st[i];
        s->ctr++;
        s->idx = 0;
    }
    return s->buf[s->idx++];
}
static uint64_t chacha_u64(chacha *s) { uint64_t lo = chacha_u32(s); return lo | (uint64_t)chacha_u32(s) << 32; }
/* ff_derive Rand for Fq: 6 LE u64, top masked by 3 shave bits, reject >= p,
 * the limbs ARE the Montgomery representation */
static fp rand_fq(chacha *s) {
    for (;;) {
        fp r;
        for (int i = 0; i < 6; ++i) r.l[i] = chacha_u64(s);
        r.l[5] &= 0xFFFFFFFFFFFFFFFFull >> 3;
        if (!geq_n(r.l, kP, 6)) return r;
    }
}
static void hash_g2_seed(const uint8_t seed[32], fp2 *hx, fp2 *hy) {
    chacha s;
    chacha_init(&s, seed);
    fp2 b2 = {kFour, kFour};
    for (;;) {
        fp2 x = {rand_fq(&s), rand_fq(&s)};
        const int greatest = (chacha_u32(&s) & 1) != 0;
        fp2 y;
        if (!fp2_sqrt(fp2_add(fp2_mul(fp2_sqr(x), x), b2), &y)) continue;
        fp2 ny = fp2_neg(y);
        fp2 yy = (fp2_gt(ny, y) != greatest) ? y : ny;
        g2 p = {x, yy, fp2_one()};
        g2 q = g2_mul(p, kCofG2, 8);
        if (g2_to_affine(q, hx, hy)) return;
    }
}
static void hash_g1_g2(const uint8_t U48[48], const uint8_t *V, uint64_t vlen, fp2 *hx, fp2 *hy) {
    uint8_t m[64 + 48], seed[32];
    uint64_t ml;
    if (vlen > 64) { orc_sha3_256(V, vlen, m); ml = 32; }
    else { memcpy(m, V, vlen); ml = vlen; }
    memcpy(m + ml, U48, 48);
    orc_sha3_256(m, ml + 48, seed);
    hash_g2_seed(seed, hx, hy);
}

/* ------------------------------------------------------------------ Fr */
static fr fr_mul(fr a, fr b) { fr r; mont_mul_n(r.l, a.l, b.l, kR, kRInv, 4); return r; }
static fr fr_from_u64(uint64_t v) { fr t = {{v, 0, 0, 0}}, r2; memcpy(r2.l, kR2r, 32); return fr_mul(t, r2); }
static fr fr_sub(fr a, fr b) {
    fr r;
    u128 br = 0;
    for (int i = 0; i < 4; ++i) { u128 t = (u128)a.l[i] - b.l[i] - br; r.l[i] = (uint64_t)t; br = (t >> 64) ? 1 : 0; }
    if (br) { u128 c = 0; for (int i = 0; i < 4; ++i) { c += (u128)r.l[i] + kR[i]; r.l[i] = (uint64_t)c; c >>= 64; } }
    return r;
}
static fr fr_inv(fr a) {
    fr r;
    memcpy(r.l, kRMontOne, 32);
    int started = 0;
    for (int i = 255; i >= 0; --i) {
        if (started) r = fr_mul(r, r);
        if ((kExpRInv[i >> 6] >> (i & 63)) & 1) { r = started ? fr_mul(r, a) : a; started = 1; }
    }
    return r;
}
static int fr_is_zero(fr a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0; }

/* ------------------------------------------------------------------ threshold_crypto surfaces */
/* PublicKeyShare::verify_decryption_share(share, Ciphertext(U, V, W)): the
 * share and key are decoded (with the crate's subgroup checks) first, as
 * message deserialisation does in hbbft.  1 valid, 0 invalid. */
/* Decoded operands: a ciphertext and the key shares are parsed once (as a
 * node holds them in memory); each share is parsed when its message arrives. */
typedef struct { fp x, y; int inf, ok; } g1dec;
typedef struct { fp2 x, y; int inf, ok; } g2dec;

static int verify_decoded(const uint8_t share48[48], const g1dec *pk, const uint8_t U48[48], const g1dec *u,
                          const uint8_t *V, uint64_t vlen, const g2dec *w) {
    fp sx, sy;
    int si;
    if (!pk->ok || !u->ok || !w->ok) return 0;
    if (!g1_decompress(share48, &sx, &sy, &si, 1)) return 0;
    fp2 hx, hy;
    hash_g1_g2(U48, V, vlen, &hx, &hy);               /* recomputed per call, as the crate does */
    fp12 a = pairing(sx, sy, si, hx, hy, 0);
    fp12 b = pairing(pk->x, pk->y, pk->inf, w->x, w->y, w->inf);
    return memcmp(&a, &b, sizeof a) == 0;
}

int orb_verify_share(const uint8_t pk48[48], const uint8_t share48[48], const uint8_t U48[48], const uint8_t *V,
                     uint64_t vlen, const uint8_t W96[96]) {
    g1dec pk, u;
    g2dec w;
    pk.ok = g1_decompress(pk48, &pk.x, &pk.y, &pk.inf, 1);
    u.ok = g1_decompress(U48, &u.x, &u.y, &u.inf, 1);
    w.ok = g2_decompress(W96, &w.x, &w.y, &w.inf);
    return verify_decoded(share48, &pk, U48, &u, V, vlen, &w);
}

/* Ciphertext::verify: e(G1, W) == e(U, H) */
int orb_ct_verify(const uint8_t U48[48], const uint8_t *V, uint64_t vlen, const uint8_t W96[96]) {
    fp ux, uy;
    fp2 wx, wy, hx, hy;
    int ui, wi;
    if (!g1_decompress(U48, &ux, &uy, &ui, 1) || !g2_decompress(W96, &wx, &wy, &wi)) return 0;
    hash_g1_g2(U48, V, vlen, &hx, &hy);
    fp12 a = pairing(kG1x, kG1y, 0, wx, wy, wi);
    fp12 b = pairing(ux, uy, ui, hx, hy, 0);
    return memcmp(&a, &b, sizeof a) == 0;
}

/* PublicKeySet::decrypt over the first t+1 (index, share) items.
 * 0 ok, -21 DuplicateEntry, -22 undecodable share. */
int orb_decrypt(uint32_t t, const uint32_t *idx, const uint8_t *shares48, const uint8_t *V, uint64_t vlen,
                uint8_t *out) {
    const uint32_t m = t + 1;
    for (uint32_t i = 0; i < m; ++i)
        for (uint32_t j = i + 1; j < m; ++j)
            if (idx[i] == idx[j]) return -21;
    g1 acc = {kOneQ, kOneQ, FP_ZERO};
    for (uint32_t i = 0; i < m; ++i) {
        fp x, y;
        int inf;
        /* shares reach decrypt already parsed (and verified): no second subgroup check */
        if (!g1_decompress(shares48 + 48ull * i, &x, &y, &inf, 0)) return -22;
        fr num = fr_from_u64(1), den = fr_from_u64(1);
        const fr xi = fr_from_u64((uint64_t)idx[i] + 1);
        for (uint32_t j = 0; j < m; ++j) {
            if (j == i) continue;
            const fr xj = fr_from_u64((uint64_t)idx[j] + 1);
            num = fr_mul(num, xj);
            den = fr_mul(den, fr_sub(xj, xi));
        }
        if (fr_is_zero(den)) return -21;
        fr l = fr_mul(num, fr_inv(den));
        fr one = {{1, 0, 0, 0}};
        l = fr_mul(l, one); /* canonical */
        if (inf) continue;
        g1 p = {x, y, kOneQ};
        acc = g1_add(acc, g1_mul(p, l.l, 4));
    }
    fp gx, gy;
    const int inf = !g1_to_affine(acc, &gx, &gy);
    uint8_t cg[48], seed[32];
    g1_compress(gx, gy, inf, cg);
    orc_sha3_256(cg, 48, seed);
    chacha s;
    chacha_init(&s, seed);
    for (uint64_t i = 0; i < vlen; ++i) out[i] = V[i] ^ (uint8_t)chacha_u32(&s);
    return 0;
}

/* ------------------------------------------------------------------ threaded batch drivers (CPU baseline) */
typedef struct {
    uint64_t lo, hi;
    const uint8_t *pk48, *share48, *U48, *V, *W96;
    const uint64_t *V_off;
    const uint32_t *share_ct, *share_pk;
    uint8_t *ok;
    uint32_t t;
    const uint32_t *idx;
    uint8_t *out;
    int32_t *status;
    g1dec *pkd, *ud;
    g2dec *wd;
    uint64_t n_pk;
} job;

static void *decode_worker(void *arg) { /* items [0, n_ct) ciphertexts, [n_ct, n_ct + n_pk) keys */
    job *j = (job *)arg;
    for (uint64_t k = j->lo; k < j->hi; ++k) {
        if (k < j->n_pk) {
            g1dec *d = &j->pkd[k];
            d->ok = g1_decompress(j->pk48 + 48ull * k, &d->x, &d->y, &d->inf, 1);
        } else {
            const uint64_t c = k - j->n_pk;
            j->ud[c].ok = g1_decompress(j->U48 + 48ull * c, &j->ud[c].x, &j->ud[c].y, &j->ud[c].inf, 1);
            j->wd[c].ok = g2_decompress(j->W96 + 96ull * c, &j->wd[c].x, &j->wd[c].y, &j->wd[c].inf);
        }
    }
    return NULL;
}
static void *verify_worker(void *arg) {
    job *j = (job *)arg;
    for (uint64_t k = j->lo; k < j->hi; ++k) {
        const uint32_t c = j->share_ct[k], p = j->share_pk[k];
        j->ok[k] = (uint8_t)verify_decoded(j->share48 + 48ull * k, &j->pkd[p], j->U48 + 48ull * c, &j->ud[c],
                                           j->V + j->V_off[c], j->V_off[c + 1] - j->V_off[c], &j->wd[c]);
    }
    return NULL;
}
static void *decrypt_worker(void *arg) {
    job *j = (job *)arg;
    const uint32_t m = j->t + 1;
    for (uint64_t k = j->lo; k < j->hi; ++k)
        j->status[k] = orb_decrypt(j->t, j->idx + (uint64_t)k * m, j->share48 + 48ull * m * k, j->V + j->V_off[k],
                                   j->V_off[k + 1] - j->V_off[k], j->out + j->V_off[k]);
    return NULL;
}
static void run_jobs(int threads, uint64_t n, job proto, void *(*fn)(void *)) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    job jobs[256];
    for (int i = 0; i < threads; ++i) {
        jobs[i] = proto;
        jobs[i].lo = n * i / threads;
        jobs[i].hi = n * (i + 1) / threads;
        pthread_create(&th[i], NULL, fn, &jobs[i]);
    }
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
}

/* verify_decryption_share for n shares (share k of ciphertext share_ct[k]
 * under key share_pk[k]): ciphertexts and keys decoded once, then one
 * contiguous block of shares per thread. */
void orb_verify_shares_batch(int threads, uint64_t n_ct, const uint8_t *U48, const uint8_t *V, const uint64_t *V_off,
                             const uint8_t *W96, uint64_t n_pk, const uint8_t *pk48, uint64_t n, const uint8_t *share48,
                             const uint32_t *share_ct, const uint32_t *share_pk, uint8_t *ok) {
    job p;
    memset(&p, 0, sizeof p);
    p.U48 = U48; p.V = V; p.V_off = V_off; p.W96 = W96; p.pk48 = pk48;
    p.share48 = share48; p.share_ct = share_ct; p.share_pk = share_pk; p.ok = ok;
    p.pkd = (g1dec *)calloc(n_pk ? n_pk : 1, sizeof(g1dec));
    p.ud = (g1dec *)calloc(n_ct ? n_ct : 1, sizeof(g1dec));
    p.wd = (g2dec *)calloc(n_ct ? n_ct : 1, sizeof(g2dec));
    p.n_pk = n_pk;
    run_jobs(threads, n_pk + n_ct, p, decode_worker);
    run_jobs(threads, n, p, verify_worker);
    free(p.pkd);
    free(p.ud);
    free(p.wd);
}

void orb_decrypt_batch(int threads, uint32_t t, uint64_t n, const uint8_t *share48, const uint32_t *idx,
                       const uint8_t *V, const uint64_t *V_off, uint8_t *out, int32_t *status) {
    job p;
    memset(&p, 0, sizeof p);
    p.t = t; p.share48 = share48; p.idx = idx; p.V = V; p.V_off = V_off; p.out = out; p.status = status;
    run_jobs(threads, n, p, decrypt_worker);
}
