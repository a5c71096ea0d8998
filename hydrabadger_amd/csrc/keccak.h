// keccak.h — Keccak-f[1600] / SHA3-256 for gfx950, one sponge state per work-item.
//
// Restates tiny-keccak `sha3_256` [EXT] (FIPS-202: rate 136, capacity 512,
// pad 0x06..0x80) as hbbft's MerkleTree uses it.
//
// gfx950 mapping: every 64-bit lane is a (lo, hi) pair of 32-bit VGPRs.
//   theta parity      v_bitop3_b32 (xor3)          2 ops per 32-bit column half
//   rotl64            v_alignbit_b32 x2            (rot by 32: register swap, free)
//   theta apply       xor3(a, C[x-1], rotl1(C[x+1])) — D never materialised
//   chi               v_bitop3_b32 a ^ (~b & c)    1 op per word
// => 180 VALU ops per round, 4320 per permutation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbg {

struct u64p {
    uint32_t lo, hi;
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// rotl64 by compile-time N (0 < N < 64)
template <int N>
__device__ __forceinline__ u64p rotl(u64p v) {
    if constexpr (N == 0) {
        return v;
    } else if constexpr (N == 32) {
        return {v.hi, v.lo};
    } else if constexpr (N < 32) {
        return {__builtin_amdgcn_alignbit(v.lo, v.hi, 32 - N), __builtin_amdgcn_alignbit(v.hi, v.lo, 32 - N)};
    } else {
        return {__builtin_amdgcn_alignbit(v.hi, v.lo, 64 - N), __builtin_amdgcn_alignbit(v.lo, v.hi, 64 - N)};
    }
}

__constant__ static const uint32_t kKeccakRC[48] = {
    0x00000001u, 0x00000000u, 0x00008082u, 0x00000000u, 0x0000808au, 0x80000000u, 0x80008000u, 0x80000000u,
    0x0000808bu, 0x00000000u, 0x80000001u, 0x00000000u, 0x80008081u, 0x80000000u, 0x00008009u, 0x80000000u,
    0x0000008au, 0x00000000u, 0x00000088u, 0x00000000u, 0x80008009u, 0x00000000u, 0x8000000au, 0x00000000u,
    0x8000808bu, 0x00000000u, 0x0000008bu, 0x80000000u, 0x00008089u, 0x80000000u, 0x00008003u, 0x80000000u,
    0x00008002u, 0x80000000u, 0x00000080u, 0x80000000u, 0x0000800au, 0x00000000u, 0x8000000au, 0x80000000u,
    0x80008081u, 0x80000000u, 0x00008080u, 0x80000000u, 0x80000001u, 0x00000000u, 0x80008008u, 0x80000000u};

// One theta-rho-pi-chi-iota round.  Lane index = x + 5y.
// B[y + 5*((2x+3y)%5)] = rotl(A[x+5y] ^ D[x], r[x+5y])
#define HBG_THETA_RHO(x, y, r, dst)                                                   \
    {                                                                                  \
        u64p t{xor3(a[(x) + 5 * (y)].lo, C[((x) + 4) % 5].lo, E[((x) + 1) % 5].lo),   \
               xor3(a[(x) + 5 * (y)].hi, C[((x) + 4) % 5].hi, E[((x) + 1) % 5].hi)};  \
        b[dst] = rotl<r>(t);                                                           \
    }

__device__ __forceinline__ void keccak_round(u64p (&a)[25], uint32_t rc_lo, uint32_t rc_hi) {
    u64p C[5], E[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) {
        C[x].lo = xor3(xor3(a[x].lo, a[x + 5].lo, a[x + 10].lo), a[x + 15].lo, a[x + 20].lo);
        C[x].hi = xor3(xor3(a[x].hi, a[x + 5].hi, a[x + 10].hi), a[x + 15].hi, a[x + 20].hi);
    }
#pragma unroll
    for (int x = 0; x < 5; ++x) E[x] = rotl<1>(C[x]);
    // rho offsets r[x+5y]:
    //  y=0: 0 1 62 28 27 | y=1: 36 44 6 55 20 | y=2: 3 10 43 25 39
    //  y=3: 41 45 15 21 8 | y=4: 18 2 61 56 14
    HBG_THETA_RHO(0, 0, 0, 0)
    HBG_THETA_RHO(1, 0, 1, 10)
    HBG_THETA_RHO(2, 0, 62, 20)
    HBG_THETA_RHO(3, 0, 28, 5)
    HBG_THETA_RHO(4, 0, 27, 15)
    HBG_THETA_RHO(0, 1, 36, 16)
    HBG_THETA_RHO(1, 1, 44, 1)
    HBG_THETA_RHO(2, 1, 6, 11)
    HBG_THETA_RHO(3, 1, 55, 21)
    HBG_THETA_RHO(4, 1, 20, 6)
    HBG_THETA_RHO(0, 2, 3, 7)
    HBG_THETA_RHO(1, 2, 10, 17)
    HBG_THETA_RHO(2, 2, 43, 2)
    HBG_THETA_RHO(3, 2, 25, 12)
    HBG_THETA_RHO(4, 2, 39, 22)
    HBG_THETA_RHO(0, 3, 41, 23)
    HBG_THETA_RHO(1, 3, 45, 8)
    HBG_THETA_RHO(2, 3, 15, 18)
    HBG_THETA_RHO(3, 3, 21, 3)
    HBG_THETA_RHO(4, 3, 8, 13)
    HBG_THETA_RHO(0, 4, 18, 14)
    HBG_THETA_RHO(1, 4, 2, 24)
    HBG_THETA_RHO(2, 4, 61, 9)
    HBG_THETA_RHO(3, 4, 56, 19)
    HBG_THETA_RHO(4, 4, 14, 4)
#pragma unroll
    for (int y = 0; y < 5; ++y) {
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            const u64p p = b[x + 5 * y], q = b[(x + 1) % 5 + 5 * y], s = b[(x + 2) % 5 + 5 * y];
            a[x + 5 * y].lo = p.lo ^ (~q.lo & s.lo);
            a[x + 5 * y].hi = p.hi ^ (~q.hi & s.hi);
        }
    }
    a[0].lo ^= rc_lo;
    a[0].hi ^= rc_hi;
}
#undef HBG_THETA_RHO

__device__ __forceinline__ void keccak_f(u64p (&a)[25]) {
#pragma unroll 2
    for (int r = 0; r < 24; ++r) keccak_round(a, kKeccakRC[2 * r], kKeccakRC[2 * r + 1]);
}

// IMPL 0: compiler-scheduled C round; 1: bank-allocated asm (keccak_asm.h)
template <int IMPL>
__device__ __forceinline__ void perm(u64p (&a)[25]);
template <>
__device__ __forceinline__ void perm<0>(u64p (&a)[25]) {
    keccak_f(a);
}

__device__ __forceinline__ void keccak_zero(u64p (&a)[25]) {
#pragma unroll
    for (int i = 0; i < 25; ++i) a[i] = {0u, 0u};
}

// SHA3-256 of a 64-byte message (left digest || right digest): hbbft hash_pair.
template <int IMPL = 0>
__device__ __forceinline__ void sha3_pair(const uint32_t (&l)[8], const uint32_t (&r)[8], uint32_t (&out)[8]) {
    u64p a[25];
    keccak_zero(a);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = {l[2 * i], l[2 * i + 1]};
        a[4 + i] = {r[2 * i], r[2 * i + 1]};
    }
    a[8].lo = 0x06u;
    a[16].hi = 0x80000000u;
    perm<IMPL>(a);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        out[2 * i] = a[i].lo;
        out[2 * i + 1] = a[i].hi;
    }
}

// SHA3-256 of `len` bytes at an 8-byte-aligned device address.  Reads only
// bytes [0, round_up(len, 8)) — callers guarantee that range is mapped.
// All lanes of a wave should pass the same `len` (the block loop is then
// wave-uniform); `p` may differ per lane.  PREFETCH: the next block's loads
// go out before this block's permutation (+31 VGPRs: merkle_build 19.8 vs
// 21.4 ms at N = 64; merkle_validate, at 4 -> 3 waves per SIMD, 6 % slower).
template <int IMPL = 0, bool PREFETCH = false>
__device__ __forceinline__ void sha3_256_aligned8(const uint8_t* __restrict__ p, uint64_t len,
                                                  uint32_t (&out)[8]) {
    u64p a[25];
    keccak_zero(a);
    const uint64_t nfull = len / 136;
    const uint2* q = reinterpret_cast<const uint2*>(p);
    uint2 w[17];
    if (PREFETCH && nfull) {
#pragma unroll
        for (int i = 0; i < 17; ++i) w[i] = q[i];
    }
    for (uint64_t blk = 0; blk < nfull; ++blk) {
        if (!PREFETCH) {
#pragma unroll
            for (int i = 0; i < 17; ++i) w[i] = q[i];
        }
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            a[i].lo ^= w[i].x;
            a[i].hi ^= w[i].y;
        }
        q += 17;
        if (PREFETCH && blk + 1 < nfull) {
#pragma unroll
            for (int i = 0; i < 17; ++i) w[i] = q[i];
        }
        perm<IMPL>(a);
    }
    // final (possibly empty) block with FIPS-202 SHA3 padding
    const uint32_t rem = (uint32_t)(len - nfull * 136);
#pragma unroll
    for (int i = 0; i < 17; ++i) {
        uint2 w = {0u, 0u};
        if ((uint32_t)(8 * i) < rem) {
            w = q[i];
            const uint32_t left = rem - 8 * i;  // bytes of this word that are message
            if (left < 8) {
                // keep `left` low bytes
                const uint64_t m = (left == 0) ? 0ull : (~0ull >> (64 - 8 * left));
                w.x &= (uint32_t)m;
                w.y &= (uint32_t)(m >> 32);
            }
        }
        a[i].lo ^= w.x;
        a[i].hi ^= w.y;
    }
    // 0x06 at byte rem, 0x80 at byte 135
    {
        const uint32_t wi = rem >> 3, sh = (rem & 7) * 8;
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            if ((uint32_t)i == wi) {
                if (sh < 32) a[i].lo ^= 0x06u << sh;
                else a[i].hi ^= 0x06u << (sh - 32);
            }
        }
        a[16].hi ^= 0x80000000u;
    }
    perm<IMPL>(a);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        out[2 * i] = a[i].lo;
        out[2 * i + 1] = a[i].hi;
    }
}

// ---- two-lane sponge: one Keccak state on a lane pair (2k, 2k + 1) -------
// Lane half h = lane & 1 holds the h-th 32-bit half of every 64-bit word, so a
// state is 25 VGPRs a lane.  A 64-bit rotation needs the partner's half (one
// DPP quad_perm [1,0,3,2] move) and one v_alignbit — the same instruction for
// both halves.  Per round and lane: 120 VALU (29 v_alignbit) against the
// one-lane round's 180 (58): a wave of 32 sponges takes ~0.63 of the time of a
// wave of 64, so merkle_build runs a launch's partial last wave generation
// this way (more waves, each shorter: launch_merkle_build).
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);  // quad_perm [1, 0, 3, 2]
}

// the own half of rotl64(w, N), given the own half of w
template <int N>
__device__ __forceinline__ uint32_t rotl_half(uint32_t own) {
    if constexpr (N == 0) {
        return own;
    } else {
        const uint32_t p = pair_swap(own);
        if constexpr (N == 32) return p;
        else if constexpr (N < 32) return __builtin_amdgcn_alignbit(own, p, 32 - N);
        else return __builtin_amdgcn_alignbit(p, own, 64 - N);
    }
}

#define HBG_THETA_RHO_HALF(x, y, r, dst) \
    b[dst] = rotl_half<r>(xor3(a[(x) + 5 * (y)], C[((x) + 4) % 5], E[((x) + 1) % 5]));

__device__ __forceinline__ void keccak_round_half(uint32_t (&a)[25], uint32_t rc) {
    uint32_t C[5], E[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) C[x] = xor3(xor3(a[x], a[x + 5], a[x + 10]), a[x + 15], a[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; ++x) E[x] = rotl_half<1>(C[x]);
    HBG_THETA_RHO_HALF(0, 0, 0, 0)
    HBG_THETA_RHO_HALF(1, 0, 1, 10)
    HBG_THETA_RHO_HALF(2, 0, 62, 20)
    HBG_THETA_RHO_HALF(3, 0, 28, 5)
    HBG_THETA_RHO_HALF(4, 0, 27, 15)
    HBG_THETA_RHO_HALF(0, 1, 36, 16)
    HBG_THETA_RHO_HALF(1, 1, 44, 1)
    HBG_THETA_RHO_HALF(2, 1, 6, 11)
    HBG_THETA_RHO_HALF(3, 1, 55, 21)
    HBG_THETA_RHO_HALF(4, 1, 20, 6)
    HBG_THETA_RHO_HALF(0, 2, 3, 7)
    HBG_THETA_RHO_HALF(1, 2, 10, 17)
    HBG_THETA_RHO_HALF(2, 2, 43, 2)
    HBG_THETA_RHO_HALF(3, 2, 25, 12)
    HBG_THETA_RHO_HALF(4, 2, 39, 22)
    HBG_THETA_RHO_HALF(0, 3, 41, 23)
    HBG_THETA_RHO_HALF(1, 3, 45, 8)
    HBG_THETA_RHO_HALF(2, 3, 15, 18)
    HBG_THETA_RHO_HALF(3, 3, 21, 3)
    HBG_THETA_RHO_HALF(4, 3, 8, 13)
    HBG_THETA_RHO_HALF(0, 4, 18, 14)
    HBG_THETA_RHO_HALF(1, 4, 2, 24)
    HBG_THETA_RHO_HALF(2, 4, 61, 9)
    HBG_THETA_RHO_HALF(3, 4, 56, 19)
    HBG_THETA_RHO_HALF(4, 4, 14, 4)
#pragma unroll
    for (int y = 0; y < 5; ++y) {
#pragma unroll
        for (int x = 0; x < 5; ++x)
            a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    }
    a[0] ^= rc;
}
#undef HBG_THETA_RHO_HALF

__device__ __forceinline__ void keccak_f_half(uint32_t (&a)[25], uint32_t half) {
#pragma unroll 2
    for (int r = 0; r < 24; ++r) keccak_round_half(a, half ? kKeccakRC[2 * r + 1] : kKeccakRC[2 * r]);
}

// SHA3-256 of `len` bytes at an 8-byte-aligned device address by a lane pair:
// both lanes pass the same p and len, half = lane & 1; out = this lane's halves
// of the digest's four 64-bit words (digest word 2i + half).  Every lane of the
// wave runs the permutations (the DPP moves read the partner lane): pairs
// without a sponge pass len = 0 and discard the result.  Reads as
// sha3_256_aligned8.
template <bool PREFETCH = false>
__device__ __forceinline__ void sha3_256_aligned8_pair(const uint8_t* __restrict__ p, uint64_t len, uint32_t half,
                                                       uint32_t (&out)[4]) {
    uint32_t a[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) a[i] = 0u;
    const uint64_t nfull = len / 136;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p) + half;
    uint32_t w[17];
    if (PREFETCH && nfull) {
#pragma unroll
        for (int i = 0; i < 17; ++i) w[i] = q[2 * i];
    }
    for (uint64_t blk = 0; blk < nfull; ++blk) {
        if (!PREFETCH) {
#pragma unroll
            for (int i = 0; i < 17; ++i) w[i] = q[2 * i];
        }
#pragma unroll
        for (int i = 0; i < 17; ++i) a[i] ^= w[i];
        q += 34;
        if (PREFETCH && blk + 1 < nfull) {
#pragma unroll
            for (int i = 0; i < 17; ++i) w[i] = q[2 * i];
        }
        keccak_f_half(a, half);
    }
    const uint32_t rem = (uint32_t)(len - nfull * 136);
#pragma unroll
    for (int i = 0; i < 17; ++i) {
        const int32_t left = (int32_t)rem - (int32_t)(8 * i + 4 * half);  // message bytes in this half-word
        if (left > 0) {
            uint32_t v = q[2 * i];
            if (left < 4) v &= (1u << (8 * left)) - 1u;
            a[i] ^= v;
        }
    }
    {
        const uint32_t wi = rem >> 3, sh = (rem & 7) * 8;
        const uint32_t hh = sh < 32 ? 0u : 1u;
#pragma unroll
        for (int i = 0; i < 17; ++i)
            if ((uint32_t)i == wi && hh == half) a[i] ^= 0x06u << (sh & 31u);
        if (half) a[16] ^= 0x80000000u;
    }
    keccak_f_half(a, half);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = a[i];
}

}  // namespace hbg
