// gf256.h — GF(2^8) arithmetic for gfx950 (host constexpr + device SWAR).
//
// Restates reed-solomon-erasure `galois_8` + `build_matrix` [EXT]
// (SURVEY.md §8(a) a1/a3/a10): polynomial 0x11D, generator 2, coding matrix
// M = V * inv(V[0..D]) with V[r][c] = r^c (0^0 = 1).
//
// Device representation: 4 consecutive byte positions of a shard in one
// 32-bit VGPR.  A product c*w is linear over GF(2): c*w = XOR over set bits i
// of c of (alpha^i * w), alpha = 2.  `xtime` computes alpha*w for 4 packed
// bytes; the 8 powers alpha^i*w of a data word are shared by every output row.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace hbg {

// ------------------------------------------------------------- constexpr tables
struct GfTables {
    uint8_t log[256];
    uint8_t exp[510];
};

constexpr GfTables make_gf_tables() {
    GfTables t{};
    unsigned b = 1;
    for (int l = 0; l < 255; ++l) {
        t.log[b] = (uint8_t)l;
        t.exp[l] = (uint8_t)b;
        t.exp[l + 255] = (uint8_t)b;
        b <<= 1;
        if (b >= 256) b ^= 0x11D;
    }
    return t;
}
inline constexpr GfTables kGf = make_gf_tables();

constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
    return (a == 0 || b == 0) ? 0 : kGf.exp[kGf.log[a] + kGf.log[b]];
}
constexpr uint8_t gf_inv(uint8_t a) { return kGf.exp[(255 - kGf.log[a]) % 255]; }
constexpr uint8_t gf_pow(uint8_t a, int n) {
    return n == 0 ? 1 : (a == 0 ? 0 : kGf.exp[(kGf.log[a] * n) % 255]);
}

// Gauss-Jordan inverse of an n x n row-major matrix (n <= 256).  Returns
// false when singular.  `aug` is caller scratch of n*2n bytes.
constexpr bool gf_invert(const uint8_t* m, int n, uint8_t* out, uint8_t* aug) {
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < 2 * n; ++c) aug[r * 2 * n + c] = c < n ? m[r * n + c] : (uint8_t)(c - n == r);
    for (int r = 0; r < n; ++r) {
        uint8_t* row = aug + r * 2 * n;
        if (row[r] == 0) {
            for (int rb = r + 1; rb < n; ++rb) {
                uint8_t* o = aug + rb * 2 * n;
                if (o[r]) {
                    for (int c = 0; c < 2 * n; ++c) {
                        uint8_t t = row[c];
                        row[c] = o[c];
                        o[c] = t;
                    }
                    break;
                }
            }
        }
        if (row[r] == 0) return false;
        if (row[r] != 1) {
            const uint8_t s = gf_inv(row[r]);
            for (int c = 0; c < 2 * n; ++c) row[c] = gf_mul(s, row[c]);
        }
        for (int rb = 0; rb < n; ++rb) {
            if (rb == r) continue;
            uint8_t* o = aug + rb * 2 * n;
            const uint8_t s = o[r];
            if (s)
                for (int c = 0; c < 2 * n; ++c) o[c] ^= gf_mul(s, row[c]);
        }
    }
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) out[r * n + c] = aug[r * 2 * n + n + c];
    return true;
}

// Parity rows M[D..D+Q) of the coding matrix, computed at compile time for
// the specialised kernels (rse build_matrix, restated).
template <int D, int Q>
struct ParityMatrix {
    uint8_t m[Q][D];
};

template <int D, int Q>
constexpr ParityMatrix<D, Q> make_parity_matrix() {
    ParityMatrix<D, Q> pm{};
    uint8_t top[D * D] = {};
    uint8_t inv[D * D] = {};
    uint8_t aug[D * 2 * D] = {};
    for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) top[r * D + c] = gf_pow((uint8_t)r, c);
    gf_invert(top, D, inv, aug);
    for (int k = 0; k < Q; ++k)
        for (int c = 0; c < D; ++c) {
            uint8_t acc = 0;
            for (int t = 0; t < D; ++t) acc ^= gf_mul(gf_pow((uint8_t)(D + k), t), inv[t * D + c]);
            pm.m[k][c] = acc;
        }
    return pm;
}

template <int D, int Q>
inline constexpr ParityMatrix<D, Q> kParity = make_parity_matrix<D, Q>();

// ------------------------------------------------------------- device SWAR
// alpha * w for 4 packed GF(2^8) bytes (xtime, reduction by 0x1D).
__device__ __forceinline__ uint32_t xtime4(uint32_t w) {
    const uint32_t h = w & 0x80808080u;
    const uint32_t mask = (h << 1) - (h >> 7);  // 0xFF in every byte whose top bit is set
    return ((w << 1) & 0xFEFEFEFEu) ^ (mask & 0x1D1D1D1Du);
}

struct Pow8 {
    uint32_t p[8];
};

__device__ __forceinline__ Pow8 powers(uint32_t w) {
    Pow8 r;
    r.p[0] = w;
#pragma unroll
    for (int i = 1; i < 8; ++i) r.p[i] = xtime4(r.p[i - 1]);
    return r;
}

struct BitList {
    int n;
    int b[8];
};
constexpr BitList bit_list(uint8_t c) {
    BitList r{};
    for (int i = 0; i < 8; ++i)
        if ((c >> i) & 1) r.b[r.n++] = i;
    return r;
}

__device__ __forceinline__ uint32_t xor3u(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc ^ (c * w) for a compile-time coefficient c: XOR of the set-bit powers,
// folded two at a time into v_bitop3 (xor3): ceil(popcount(c)/2) VALU ops.
template <uint8_t C>
__device__ __forceinline__ uint32_t cmul_acc(uint32_t acc, const Pow8& P) {
    constexpr BitList bl = bit_list(C);
#pragma unroll
    for (int i = 0; i + 1 < bl.n; i += 2) acc = xor3u(acc, P.p[bl.b[i]], P.p[bl.b[i + 1]]);
    if constexpr (bl.n & 1) acc ^= P.p[bl.b[bl.n - 1]];
    return acc;
}

// ------------------------------------------------------------- split-nibble form
// c*w = Lo[c & 15] ^ Hi[c >> 4] with Lo[m] = XOR_{i in m} alpha^i w and
// Hi[m] = XOR_{i in m} alpha^(4+i) w (the GPU analogue of rse's PSHUFB
// low/high nibble tables, but over the 8 SWAR powers of one data word).
// xtime via v_perm: the reduction byte (0x1D or 0) is selected by each
// byte's top bit, so one xtime = lshr, and, perm, lshl, bitop3.
__device__ __forceinline__ uint32_t xtime4p(uint32_t w) {
    const uint32_t sel = (w >> 7) & 0x01010101u;               // 0/1 per byte
    const uint32_t red = __builtin_amdgcn_perm(0u, 0x00001D00u, sel);  // byte -> 0x00 / 0x1D
    return __builtin_amdgcn_bitop3_b32(w << 1, 0xFEFEFEFEu, red, 0x6A);  // (a & b) ^ c
}

// One nibble table: T[m] for m in 1..15 from the four powers q0..q3 (T[0] unused).
// Entries are computed lazily by the compiler: only those a column's
// compile-time coefficients reference survive dead-code elimination.
struct NibTab {
    uint32_t t[16];
};

__device__ __forceinline__ NibTab nib_table(uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3) {
    NibTab r;
    r.t[0] = 0u;
    r.t[1] = q0;
    r.t[2] = q1;
    r.t[4] = q2;
    r.t[8] = q3;
    r.t[3] = q0 ^ q1;
    r.t[5] = q0 ^ q2;
    r.t[6] = q1 ^ q2;
    r.t[9] = q0 ^ q3;
    r.t[10] = q1 ^ q3;
    r.t[12] = q2 ^ q3;
    r.t[7] = xor3u(q0, q1, q2);
    r.t[11] = xor3u(q0, q1, q3);
    r.t[13] = xor3u(q0, q2, q3);
    r.t[14] = xor3u(q1, q2, q3);
    r.t[15] = r.t[3] ^ r.t[12];
    return r;
}

struct NibPair {
    NibTab lo, hi;
};

__device__ __forceinline__ NibPair nib_tables(uint32_t w) {
    const uint32_t p1 = xtime4p(w), p2 = xtime4p(p1), p3 = xtime4p(p2), p4 = xtime4p(p3);
    const uint32_t p5 = xtime4p(p4), p6 = xtime4p(p5), p7 = xtime4p(p6);
    return {nib_table(w, p1, p2, p3), nib_table(p4, p5, p6, p7)};
}

// acc ^ (C * w) for a compile-time coefficient: one bitop3 (or xor) per pair.
template <uint8_t C>
__device__ __forceinline__ uint32_t nib_mac(uint32_t acc, const NibPair& T) {
    constexpr int lo = C & 15, hi = C >> 4;
    if constexpr (lo && hi) return xor3u(acc, T.lo.t[lo], T.hi.t[hi]);
    else if constexpr (lo) return acc ^ T.lo.t[lo];
    else if constexpr (hi) return acc ^ T.hi.t[hi];
    else return acc;
}

// c * w for a run-time (wave-uniform) coefficient.
__device__ __forceinline__ uint32_t rmul(uint32_t c, const Pow8& P) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= P.p[i] & (0u - ((c >> i) & 1u));
    return r;
}

}  // namespace hbg
