// tdec_kernels.hip — gfx950 kernels for hbbft's ThresholdDecrypt path (family 3).
//
// Restates threshold_crypto [EXT] as hbbft's ThresholdDecrypt drives it
// (reached from /root/reference/src/hydrabadger/
// state.rs:486-487):
//   tdec_ct_decode      per ciphertext: decompress + subgroup-check U (G1) and
//                       W (G2) -> the ciphertext's status (what the leaves need)
//   tdec_ct_prepare(_w) H = hash_g1_g2(U, V) (SHA3 -> ChaChaRng -> try-and-
//                       increment -> cofactor), G2Prepared lines of H and W
//                       (second stream, overlapped with the share leaves)
//   tdec_pk_prepare     PublicKeyShare table: decompress + subgroup check
//   tdec_verify_shares  PublicKeyShare::verify_decryption_share for every share:
//                       e(S_i, H) * e(-PK_i, W) == 1 (one 2-pair Miller loop +
//                       one final exponentiation per work-item)
//   tdec_ct_verify      Ciphertext::verify: e(G1, W) * e(-U, H) == 1
//   tdec_combine        PublicKeySet::decrypt: interpolate the first t+1 shares
//                       at 0 (Lagrange over Fr) + xor_with_hash
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <stdint.h>

#include "bls.h"
#include "dev_err.h"
#include "grid.h"
#include "keccak.h"
#include "keccak_asm.h"
#include "tdec_kernels.h"

#include <hipcub/hipcub.hpp>

namespace hbg {
namespace bls {

// Occupancy contract for every TDec kernel: the tower arithmetic is a deep
// non-inlined call graph whose callees otherwise take the whole 512-entry
// unified register file (256 VGPRs + AGPR spill space = 1 wave/SIMD).  Capping
// every kernel (and so, via attribute propagation, every callee) at
// HBG_TDEC_WPE waves per SIMD trades a few scratch spills for latency hiding.
#ifndef HBG_TDEC_WPE
#define HBG_TDEC_WPE 2
#endif
#define TDEC_KERNEL __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HBG_TDEC_WPE)))
// Pairing and G2 kernels (a Miller loop + final exponentiation, or G2 point
// arithmetic, per lane): one wave per SIMD in both builds.  The
// register-resident Fp12 tower (bls.h) keeps a line evaluation's ~450 live
// values in the 256 VGPRs + 256 AGPRs a lone wave owns, and Fp2 products are
// three interleaved Montgomery chains (hbg_fpmul3), so a lone wave still
// issues back to back.  G1-only kernels stay at HBG_TDEC_WPE.
#define TDEC_WAVE1_KERNEL __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1)))

#define BD __device__ __forceinline__

// Work count of a grid-stride round read on the device (no host round trip
// between the group-testing rounds): min(*n_dev, cap), or cap without n_dev.
BD uint64_t dev_count(const uint32_t* n_dev, uint64_t cap) {
    if (!n_dev) return cap;
    const uint64_t v = *n_dev;
    return v < cap ? v : cap;
}
BD uint64_t grid_lane() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }

// Diagnostic builds only (-DHBG_DEBUG_CHECKS, tools/diag_tdec.py): range checks
// on the batched verifier's indices that print and skip instead of faulting.
#ifdef HBG_DEBUG_CHECKS
__device__ uint64_t g_dbg[4];  // n shares, nb_max, n_ct + 1, n_pk + 1
#define HBG_DBG_RANGE(v, bound, what)                                                                   \
    (((uint64_t)(v) < (uint64_t)(bound))                                                                \
         ? true                                                                                         \
         : (printf("hbg range: %s = %llu >= %llu (%s:%d)\n", what, (unsigned long long)(v),              \
                   (unsigned long long)(bound), __FILE__, __LINE__),                                    \
            false))
#else
#define HBG_DBG_RANGE(v, bound, what) true
#endif

// ------------------------------------------------------------------ SHA3-256 over bytes
BD void sha3_bytes(const uint8_t* p, uint32_t len, uint8_t out[32]) {
    u64p a[25];
    keccak_zero(a);
    uint32_t pos = 0;
    while (true) {
        const uint32_t take = (len - pos) >= 136 ? 136 : (len - pos);
        uint8_t blk[136];
        for (uint32_t i = 0; i < 136; ++i) blk[i] = i < take ? p[pos + i] : 0;
        const bool last = take < 136;
        if (last) {
            blk[take] ^= 0x06;
            blk[135] ^= 0x80;
        }
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                lo |= (uint32_t)blk[8 * i + b] << (8 * b);
                hi |= (uint32_t)blk[8 * i + 4 + b] << (8 * b);
            }
            a[i].lo ^= lo;
            a[i].hi ^= hi;
        }
        keccak_f(a);
        pos += take;
        if (last) break;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            out[8 * i + b] = (uint8_t)(a[i].lo >> (8 * b));
            out[8 * i + 4 + b] = (uint8_t)(a[i].hi >> (8 * b));
        }
    }
}

// ------------------------------------------------------------------ ChaCha20 (rand_chacha layout)
BD uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
// the byte rotations as one full-rate v_perm_b32 (v_alignbit, the compiler's
// rotate, issues at half rate on gfx950)
BD uint32_t rotl16p(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x01000302u); }
BD uint32_t rotl8p(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x02010003u); }

#define QR(a, b, c, d)            \
    a += b;                       \
    d = rotl16p(d ^ a);           \
    c += d;                       \
    b = rotl32(b ^ c, 12);        \
    a += b;                       \
    d = rotl8p(d ^ a);            \
    c += d;                       \
    b = rotl32(b ^ c, 7);

BD void chacha_block(const uint32_t key[8], uint32_t counter, uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646Eu, 0x79622D32u, 0x6B206574u, key[0], key[1], key[2], key[3],
                      key[4],      key[5],      key[6],      key[7],      counter, 0u,     0u,     0u};
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = s[i];
    for (int r = 0; r < 10; ++r) {
        QR(w[0], w[4], w[8], w[12]);
        QR(w[1], w[5], w[9], w[13]);
        QR(w[2], w[6], w[10], w[14]);
        QR(w[3], w[7], w[11], w[15]);
        QR(w[0], w[5], w[10], w[15]);
        QR(w[1], w[6], w[11], w[12]);
        QR(w[2], w[7], w[8], w[13]);
        QR(w[3], w[4], w[9], w[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = w[i] + s[i];
}
#undef QR

struct ChaChaRng {
    uint32_t key[8];
    uint32_t buf[16];
    uint32_t counter, idx;
    BD void init(const uint8_t seed[32]) {
        for (int i = 0; i < 8; ++i)
            key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) | ((uint32_t)seed[4 * i + 2] << 16) |
                     ((uint32_t)seed[4 * i + 3] << 24);
        counter = 0;
        idx = 16;
    }
    BD uint32_t next_u32() {
        if (idx >= 16) {
            chacha_block(key, counter, buf);
            ++counter;
            idx = 0;
        }
        return buf[idx++];
    }
};

// ------------------------------------------------------------------ long messages (a13, a16)
// xor_with_hash's keystream and hash_g1_g2's SHA3(V) for contributions of any
// length (in HoneyBadger V is the whole serialised contribution):
//  * the keystream is seekable by block counter: a 256-thread workgroup per
//    item (items strided over a capped grid, so the item count sets no grid
//    limit), threads over its ChaCha20 blocks; block c covers output bytes
//    [16c, 16c + 16) (rand's `Standard` u8 is the low byte of each next_u32);
//  * SHA3(V) reads V a dword at a time (aligned loads + v_alignbyte) into the
//    bank-allocated Keccak round (keccak_asm.h), one lane per item.
// Both replace byte-serial loops of one lane in the kernels that call them.
__global__ __launch_bounds__(256) void tdec_keystream_xor(uint64_t n, const uint8_t* __restrict__ seeds,
                                                          const uint8_t* __restrict__ in,
                                                          const uint64_t* __restrict__ off, uint8_t* __restrict__ out,
                                                          const int32_t* __restrict__ status) {
    for (uint64_t k = blockIdx.x; k < n; k += gridDim.x) {
    if (status && status[k] != 0) continue;  // no output for a failed item (its bytes stay untouched)
    uint32_t key[8];
    const uint8_t* sd = seeds + 32 * k;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        key[i] = (uint32_t)sd[4 * i] | ((uint32_t)sd[4 * i + 1] << 8) | ((uint32_t)sd[4 * i + 2] << 16) |
                 ((uint32_t)sd[4 * i + 3] << 24);
    const uint64_t o = off[k], len = off[k + 1] - o;
    const uint64_t nb = (len + 15) / 16;
    const bool vec = (((uintptr_t)(in + o) | (uintptr_t)(out + o)) & 15u) == 0;
    for (uint64_t c = threadIdx.x; c < nb; c += blockDim.x) {
        uint32_t w[16];
        chacha_block(key, (uint32_t)c, w);
        const uint64_t b0 = 16 * c;
        if (vec && b0 + 16 <= len) {  // one 16-B load and store: the keystream is each word's low byte
            uint32_t ks[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                ks[i] = __builtin_amdgcn_perm(w[4 * i + 1], w[4 * i], 0x0c0c0400u) |
                        __builtin_amdgcn_perm(w[4 * i + 3], w[4 * i + 2], 0x04000c0cu);
            const uint4 v = *reinterpret_cast<const uint4*>(in + o + b0);
            *reinterpret_cast<uint4*>(out + o + b0) = make_uint4(v.x ^ ks[0], v.y ^ ks[1], v.z ^ ks[2], v.w ^ ks[3]);
            continue;
        }
#pragma unroll
        for (int b = 0; b < 16; ++b)
            if (b0 + b < len) out[o + b0 + b] = in[o + b0 + b] ^ (uint8_t)(w[b] & 0xFFu);
    }
    }
}

// SHA3-256 of len bytes at p (any alignment).  An aligned dword holding at
// least one message byte is always readable.
__device__ __forceinline__ void sha3_long(const uint8_t* p, uint64_t len, uint8_t* out) {
    u64p a[25];
    keccak_zero(a);
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
    // the next block's loads are issued before this block's permutation (one
    // lane per message at one wave per SIMD: nothing else hides their latency)
    const uint64_t nfull = len / 136;
    uint32_t nw[35];
    auto load = [&](uint64_t blk) {
        const uint32_t* qb = q + blk * 34;
#pragma unroll
        for (int j = 0; j < 34; ++j) nw[j] = qb[j];
        nw[34] = sh ? qb[34] : 0u;
    };
    if (nfull) load(0);
    for (uint64_t blk = 0; blk < nfull; ++blk) {
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            a[i].lo ^= __builtin_amdgcn_alignbyte(nw[2 * i + 1], nw[2 * i], sh);
            a[i].hi ^= __builtin_amdgcn_alignbyte(nw[2 * i + 2], nw[2 * i + 1], sh);
        }
        if (blk + 1 < nfull) load(blk + 1);
        perm<1>(a);
    }
    const uint64_t pos = nfull * 136;
    const uint32_t rem = (uint32_t)(len - pos);  // < 136 bytes + FIPS-202 padding
    uint32_t w[34];
#pragma unroll
    for (int j = 0; j < 34; ++j) w[j] = 0u;
    for (uint32_t i = 0; i < rem; ++i) {
        const uint32_t b = p[pos + i];
#pragma unroll
        for (int j = 0; j < 34; ++j)
            if ((i >> 2) == (uint32_t)j) w[j] |= b << (8 * (i & 3));
    }
#pragma unroll
    for (int j = 0; j < 34; ++j) {
        if ((rem >> 2) == (uint32_t)j) w[j] ^= 0x06u << (8 * (rem & 3));
    }
    w[33] ^= 0x80000000u;
#pragma unroll
    for (int i = 0; i < 17; ++i) {
        a[i].lo ^= w[2 * i];
        a[i].hi ^= w[2 * i + 1];
    }
    perm<1>(a);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            out[8 * i + b] = (uint8_t)(a[i].lo >> (8 * b));
            out[8 * i + 4 + b] = (uint8_t)(a[i].hi >> (8 * b));
        }
    }
}

// dig[k] = SHA3(V_k) for every item with |V_k| > 64 (hash_g1_g2's message
// digest); shorter items are hashed inline by the caller.
__global__ __launch_bounds__(64) void tdec_v_digest(uint64_t n, const uint8_t* __restrict__ V,
                                                    const uint64_t* __restrict__ off, uint8_t* __restrict__ dig) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint64_t o = off[k], len = off[k + 1] - o;
    if (len > 64) sha3_long(V + o, len, dig + 32 * k);
}

// Low-latency SHA3-256 of one long message per WAVE (few items, MiB-sized V:
// the configs[4] epoch hashes 128 contributions of 1 MiB, where one lane per
// item leaves the GPU idle and each sponge is 7,710 dependent permutations).
// Lane l < 25 holds state word l = x + 5y as (lo, hi); a round is
//   theta  column parity from the 4 other lanes of the column, then C[x-1]
//          and C[x+1] from the neighbour lanes (ds_bpermute gathers),
//   rho    each lane rotates its own word by its own offset (64-bit shifts),
//   pi+chi each lane gathers the rotated words of its pi source and of the
//          sources of (x+1, y), (x+2, y) and applies chi,
//   iota   lane 0 only (a lane mask ANDed with the round constant),
// ~35 VALU + 18 cross-lane gathers (three dependent gather stages) per round
// instead of the 190-instruction round of one lane: 4.4 us per permutation
// against 8.8 (gathering C[x-1] and C[x+1] from the 10 lanes of the two
// columns in ONE stage, 26 gathers per round, measured slower:
// profiles/r03n/theta_ab.txt).  Blocks are absorbed by lanes 0..16 (8 message bytes
// each, the next block's dwords prefetched during the current permutation).
constexpr uint8_t kRhoOff[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39,
                                 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
__device__ __forceinline__ uint32_t lane_get(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}

__global__ __launch_bounds__(64) void tdec_v_digest_wave64(uint64_t n, const uint8_t* __restrict__ V,
                                                           const uint64_t* __restrict__ off,
                                                           uint8_t* __restrict__ dig) {
    const uint64_t k = blockIdx.x;
    if (k >= n) return;
    const uint64_t o = off[k], len = off[k + 1] - o;
    if (len <= 64) return;  // hashed inline by hash_g1_g2_msg's caller
    const uint32_t l = threadIdx.x, ls = l < 25 ? l : l % 25;
    const uint32_t x = ls % 5, y = ls / 5;
    uint32_t col[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j] = x + 5 * ((y + 1 + j) % 5);
    const uint32_t cm1 = (x + 4) % 5 + 5 * y, cp1 = (x + 1) % 5 + 5 * y;
    // B[X][Y] = rho(A[x][y]) with X = y, Y = 2x + 3y: the source of (X, Y) is
    // x = 3 (Y - 3X) mod 5, y = X
    auto pisrc = [](uint32_t X, uint32_t Y) { return (3 * (Y + 15 - 3 * X)) % 5 + 5 * X; };
    const uint32_t s0 = pisrc(x, y), s1 = pisrc((x + 1) % 5, y), s2 = pisrc((x + 2) % 5, y);
    const uint32_t r = kRhoOff[ls], rr = (64 - r) & 63;
    const uint32_t lane0 = l == 0 ? 0xFFFFFFFFu : 0u;
    uint32_t lo = 0, hi = 0;
    auto permute = [&]() {
        for (int rnd = 0; rnd < 24; ++rnd) {
            uint32_t clo = lo, chi = hi;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                clo ^= lane_get(lo, col[j]);
                chi ^= lane_get(hi, col[j]);
            }
            const uint32_t mlo = lane_get(clo, cm1), mhi = lane_get(chi, cm1);
            const uint32_t plo = lane_get(clo, cp1), phi = lane_get(chi, cp1);
            lo = __builtin_amdgcn_bitop3_b32(lo, mlo, __builtin_amdgcn_alignbit(plo, phi, 31), 0x96);
            hi = __builtin_amdgcn_bitop3_b32(hi, mhi, __builtin_amdgcn_alignbit(phi, plo, 31), 0x96);
            uint64_t w = ((uint64_t)hi << 32) | lo;
            w = (w << r) | (w >> rr);
            const uint32_t wlo = (uint32_t)w, whi = (uint32_t)(w >> 32);
            const uint32_t b0l = lane_get(wlo, s0), b0h = lane_get(whi, s0);
            const uint32_t b1l = lane_get(wlo, s1), b1h = lane_get(whi, s1);
            const uint32_t b2l = lane_get(wlo, s2), b2h = lane_get(whi, s2);
            lo = __builtin_amdgcn_bitop3_b32(b0l, b1l, b2l, 0xd2) ^ (lane0 & kKeccakRC[2 * rnd]);
            hi = __builtin_amdgcn_bitop3_b32(b0h, b1h, b2h, 0xd2) ^ (lane0 & kKeccakRC[2 * rnd + 1]);
        }
    };
    const uint8_t* p = V + o;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
    const bool msg_lane = l < 17;
    const uint32_t li = msg_lane ? l : 0u;
    const uint64_t nfull = len / 136;
    // lane li's 8 bytes of block b: dwords 34 b + 2 li .. + 2 of the aligned view
    // (the third only when the message is unaligned: the dword holding byte
    // 136 b + 8 li + 7 is readable because that byte is a message byte)
    uint32_t d0 = 0, d1 = 0, d2 = 0;
    auto fetch = [&](uint64_t b) {
        const uint32_t* qb = q + 34 * b + 2 * li;
        d0 = qb[0];
        d1 = qb[1];
        d2 = sh ? qb[2] : 0u;
    };
    if (nfull) fetch(0);
    for (uint64_t b = 0; b < nfull; ++b) {
        const uint32_t wl = __builtin_amdgcn_alignbyte(d1, d0, sh), wh = __builtin_amdgcn_alignbyte(d2, d1, sh);
        if (msg_lane) {
            lo ^= wl;
            hi ^= wh;
        }
        if (b + 1 < nfull) fetch(b + 1);  // in flight during this permutation
        permute();
    }
    // final block: bytes [136 nfull, len) + FIPS-202 padding 0x06 .. 0x80
    const uint32_t rem = (uint32_t)(len - 136 * nfull);
    uint32_t wl = 0, wh = 0;
    if (msg_lane) {
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t pos = 8 * li + i;
            uint32_t byte = pos < rem ? (uint32_t)p[136 * nfull + pos] : 0u;
            if (pos == rem) byte ^= 0x06u;
            if (pos == 135) byte ^= 0x80u;
            if (i < 4) wl |= byte << (8 * i);
            else wh |= byte << (8 * (i - 4));
        }
        lo ^= wl;
        hi ^= wh;
    }
    permute();
    if (l < 4) {
        uint8_t* d = dig + 32 * k + 8 * l;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            d[b] = (uint8_t)(lo >> (8 * b));
            d[4 + b] = (uint8_t)(hi >> (8 * b));
        }
    }
}

// Round 4: the same wave sponge on BIT-INTERLEAVED 32-bit halves, one half
// per lane (lane 2i + h holds the even (h = 0) or odd (h = 1) bits of state
// word i, the standard 32-bit Keccak representation).  A 64-bit rotation by
// r is then a 32-bit rotation of one half — by r/2 when r is even, and by
// (r±1)/2 of the OTHER half when r is odd — so every cross-lane move is one
// ds_bpermute of one dword instead of two: per round 4 (column parity) + 2
// (C[x-1], rotl(C[x+1], 1)) + 3 (pi sources of chi) gathers in three
// dependent stages and 7 VALU, against 18 gathers and ~35 VALU for the
// (lo, hi)-per-lane sponge above.  The odd-r half swap is folded into the
// gather addresses: a source lane pre-rotates its half by the amount its one
// pi destination needs, and a destination of half h reads half h ^ (r & 1).
// Message words are de-interleaved on absorption (prepared for the next block
// in the middle of the current permutation) and re-interleaved for the
// digest.
constexpr uint64_t kKeccakRC64[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
constexpr uint32_t even_bits64(uint64_t w) {
    uint32_t r = 0;
    for (int i = 0; i < 32; ++i) r |= (uint32_t)((w >> (2 * i)) & 1u) << i;
    return r;
}
__device__ __forceinline__ uint32_t compress_even32(uint32_t x) {  // bits 0, 2, .., 30 -> 0 .. 15
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    return (x | (x >> 8)) & 0x0000FFFFu;
}
__device__ __forceinline__ uint32_t spread_even16(uint32_t x) {  // bits 0 .. 15 -> 0, 2, .., 30
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    return (x | (x << 1)) & 0x55555555u;
}
__device__ __forceinline__ uint32_t bperm(uint32_t addr, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)v);
}

template <bool kTwoStage>
__global__ __launch_bounds__(64) void tdec_v_digest_wave(uint64_t n, const uint8_t* __restrict__ V,
                                                         const uint64_t* __restrict__ off,
                                                         uint8_t* __restrict__ dig) {
    const uint64_t k = blockIdx.x;
    if (k >= n) return;
    const uint64_t o = off[k], len = off[k + 1] - o;
    if (len <= 64) return;  // hashed inline by hash_g1_g2_msg's caller
    // lanes 50..63 shadow lanes 0..13 (never read, never absorb or store)
    const uint32_t l = threadIdx.x, ls = l < 50 ? l : l - 50;
    const uint32_t i = ls >> 1, h = ls & 1u, x = i % 5, y = i / 5;
    auto addr = [](uint32_t word, uint32_t half) { return (2 * word + half) << 2; };
    uint32_t acol[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acol[j] = addr(x + 5 * ((y + 1 + j) % 5), h);
    // D[x] = C[x-1] ^ rotl64(C[x+1], 1): even half = C[x-1].e ^ rotl32(C[x+1].o, 1), odd = C[x-1].o ^ C[x+1].e
    const uint32_t acm = addr((x + 4) % 5 + 5 * y, h), acp = addr((x + 1) % 5 + 5 * y, h ^ 1u);
    // kTwoStage: D from the 5 + 5 words of columns x-1 and x+1 in ONE gather
    // stage (C[x] itself is never needed): 13 gathers in two dependent stages
    uint32_t am5[5], ap5[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        am5[j] = addr((x + 4) % 5 + 5 * j, h);
        ap5[j] = addr((x + 1) % 5 + 5 * j, h ^ 1u);
    }
    const uint32_t scp = h ? 0u : 31u;
    const uint32_t r = kRhoOff[i];
    const uint32_t amt = (r & 1u) ? (h ? (r + 1) / 2 : (r - 1) / 2) : r / 2;
    const uint32_t srho = (32u - amt) & 31u;  // alignbit(v, v, s) = rotr32(v, s)
    auto pisrc = [](uint32_t X, uint32_t Y) { return (3 * (Y + 15 - 3 * X)) % 5 + 5 * X; };
    auto srcaddr = [&](uint32_t X, uint32_t Y) {
        const uint32_t s = pisrc(X, Y);
        return addr(s, h ^ (kRhoOff[s] & 1u));
    };
    const uint32_t ab0 = srcaddr(x, y), ab1 = srcaddr((x + 1) % 5, y), ab2 = srcaddr((x + 2) % 5, y);
    const uint32_t m_e = l == 0 ? 0xFFFFFFFFu : 0u, m_o = l == 1 ? 0xFFFFFFFFu : 0u;
    const bool msg_lane = l < 34;
    const uint32_t li = msg_lane ? i : 0u;
    const uint8_t* p = V + o;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
    const uint64_t nfull = len / 136;
    uint32_t d0 = 0, d1 = 0, d2 = 0, nxt = 0;
    auto fetch = [&](uint64_t b) {
        const uint32_t* qb = q + 34 * b + 2 * li;
        d0 = qb[0];
        d1 = qb[1];
        d2 = sh ? qb[2] : 0u;
    };
    // this lane's interleaved half of the 64-bit message word (wl, wh)
    auto half_of = [&](uint32_t wl, uint32_t wh) {
        const uint32_t v = compress_even32(wl >> h) | (compress_even32(wh >> h) << 16);
        return msg_lane ? v : 0u;
    };
    auto prepare = [&]() {
        nxt = half_of(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh));
    };
    uint32_t s = 0;
    auto permute = [&](bool hook) {
#pragma unroll
        for (int rnd = 0; rnd < 24; ++rnd) {
            if constexpr (kTwoStage) {
                uint32_t m[5], q5[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) m[j] = bperm(am5[j], s);
#pragma unroll
                for (int j = 0; j < 5; ++j) q5[j] = bperm(ap5[j], s);
                const uint32_t cm = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(m[0], m[1], m[2], 0x96),
                                                                m[3], m[4], 0x96);
                const uint32_t cp = __builtin_amdgcn_bitop3_b32(
                    __builtin_amdgcn_bitop3_b32(q5[0], q5[1], q5[2], 0x96), q5[3], q5[4], 0x96);
                s = __builtin_amdgcn_bitop3_b32(s, cm, __builtin_amdgcn_alignbit(cp, cp, scp), 0x96);
            } else {
                const uint32_t g0 = bperm(acol[0], s), g1 = bperm(acol[1], s);
                const uint32_t g2 = bperm(acol[2], s), g3 = bperm(acol[3], s);
                const uint32_t c =
                    __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(s, g0, g1, 0x96), g2, g3, 0x96);
                const uint32_t cm = bperm(acm, c), cp = bperm(acp, c);
                s = __builtin_amdgcn_bitop3_b32(s, cm, __builtin_amdgcn_alignbit(cp, cp, scp), 0x96);
            }
            const uint32_t rv = __builtin_amdgcn_alignbit(s, s, srho);
            const uint32_t b0 = bperm(ab0, rv), b1 = bperm(ab1, rv), b2 = bperm(ab2, rv);
            constexpr uint32_t kE[24] = {
                even_bits64(kKeccakRC64[0]), even_bits64(kKeccakRC64[1]), even_bits64(kKeccakRC64[2]),
                even_bits64(kKeccakRC64[3]), even_bits64(kKeccakRC64[4]), even_bits64(kKeccakRC64[5]),
                even_bits64(kKeccakRC64[6]), even_bits64(kKeccakRC64[7]), even_bits64(kKeccakRC64[8]),
                even_bits64(kKeccakRC64[9]), even_bits64(kKeccakRC64[10]), even_bits64(kKeccakRC64[11]),
                even_bits64(kKeccakRC64[12]), even_bits64(kKeccakRC64[13]), even_bits64(kKeccakRC64[14]),
                even_bits64(kKeccakRC64[15]), even_bits64(kKeccakRC64[16]), even_bits64(kKeccakRC64[17]),
                even_bits64(kKeccakRC64[18]), even_bits64(kKeccakRC64[19]), even_bits64(kKeccakRC64[20]),
                even_bits64(kKeccakRC64[21]), even_bits64(kKeccakRC64[22]), even_bits64(kKeccakRC64[23])};
            constexpr uint32_t kO[24] = {
                even_bits64(kKeccakRC64[0] >> 1), even_bits64(kKeccakRC64[1] >> 1), even_bits64(kKeccakRC64[2] >> 1),
                even_bits64(kKeccakRC64[3] >> 1), even_bits64(kKeccakRC64[4] >> 1), even_bits64(kKeccakRC64[5] >> 1),
                even_bits64(kKeccakRC64[6] >> 1), even_bits64(kKeccakRC64[7] >> 1), even_bits64(kKeccakRC64[8] >> 1),
                even_bits64(kKeccakRC64[9] >> 1), even_bits64(kKeccakRC64[10] >> 1),
                even_bits64(kKeccakRC64[11] >> 1), even_bits64(kKeccakRC64[12] >> 1),
                even_bits64(kKeccakRC64[13] >> 1), even_bits64(kKeccakRC64[14] >> 1),
                even_bits64(kKeccakRC64[15] >> 1), even_bits64(kKeccakRC64[16] >> 1),
                even_bits64(kKeccakRC64[17] >> 1), even_bits64(kKeccakRC64[18] >> 1),
                even_bits64(kKeccakRC64[19] >> 1), even_bits64(kKeccakRC64[20] >> 1),
                even_bits64(kKeccakRC64[21] >> 1), even_bits64(kKeccakRC64[22] >> 1),
                even_bits64(kKeccakRC64[23] >> 1)};
            s = __builtin_amdgcn_bitop3_b32(b0, b1, b2, 0xd2) ^ (m_e & kE[rnd]) ^ (m_o & kO[rnd]);
            if (hook && rnd == 11) prepare();  // the next block's dwords have long arrived
        }
    };
    if (nfull) {
        fetch(0);
        prepare();
    }
    for (uint64_t b = 0; b < nfull; ++b) {
        s ^= nxt;
        const bool more = b + 1 < nfull;
        if (more) fetch(b + 1);  // in flight during this permutation
        permute(more);
    }
    // final block: bytes [136 nfull, len) + FIPS-202 padding 0x06 .. 0x80
    const uint32_t rem = (uint32_t)(len - 136 * nfull);
    uint32_t wl = 0, wh = 0;
    if (msg_lane) {
        for (uint32_t t = 0; t < 8; ++t) {
            const uint32_t pos = 8 * li + t;
            uint32_t byte = pos < rem ? (uint32_t)p[136 * nfull + pos] : 0u;
            if (pos == rem) byte ^= 0x06u;
            if (pos == 135) byte ^= 0x80u;
            if (t < 4) wl |= byte << (8 * t);
            else wh |= byte << (8 * (t - 4));
        }
    }
    s ^= half_of(wl, wh);
    permute(false);
    // digest: words 0..3 = lanes 0..7; lane 2w + h writes bytes 8w + 4h .. + 3
    const uint32_t partner = bperm((l ^ 1u) << 2, s);
    const uint32_t e = h ? partner : s, od = h ? s : partner;
    const uint32_t es = h ? e >> 16 : e, os = h ? od >> 16 : od;
    const uint32_t w32 = spread_even16(es) | (spread_even16(os) << 1);
    if (l < 8) {
        uint8_t* d = dig + 32 * k + 4 * l;
#pragma unroll
        for (int b = 0; b < 4; ++b) d[b] = (uint8_t)(w32 >> (8 * b));
    }
}

// hash_g1_g2's message m = (|V| > 64 ? SHA3(V) : V) || compress(U); returns
// |m| (dig: tdec_v_digest's output for this item).
BD uint32_t hash_g1_g2_msg(const uint8_t* V, uint64_t len, const uint8_t* dig, const uint8_t* u48,
                           uint8_t (&m)[64 + 48]) {
    uint32_t mlen;
    if (len > 64) {
        for (int i = 0; i < 32; ++i) m[i] = dig[i];
        mlen = 32;
    } else {
        for (uint32_t i = 0; i < len; ++i) m[i] = V[i];
        mlen = (uint32_t)len;
    }
    for (int i = 0; i < 48; ++i) m[mlen + i] = u48[i];
    return mlen + 48;
}

// ------------------------------------------------------------------ hash_g1_g2
// ff_derive Rand for Fq: 6 x next_u64 (LE), top limb masked by 3 shave bits,
// rejected unless < p, taken as a Montgomery representation.  Our Montgomery
// form of that value IS the repr (same R = 2^384).
// Bounded: each try succeeds with probability p / 2^381 > 0.8, so 64 failed
// tries (probability < 2^-148) never happen; the bound only guarantees that
// every wave terminates.
BD Fp rand_fq(ChaChaRng& rng) {
    Fp r;
    for (int tries = 0; tries < 64; ++tries) {
#pragma unroll
        for (int i = 0; i < 12; ++i) r[i] = rng.next_u32();
        r[11] &= 0x1FFFFFFFu;
        if (fp_raw_lt_p(r)) return r;
    }
    return fp_zero();
}

// ---- G2 cofactor clearing (the crate's scale_by_cofactor: [h2]P, h2 the 507-bit
// G2 cofactor), computed without a 507-bit double-and-add:
//  * Budroni-Pintore: [h_eff]P = [x^2-x-1]P + [x-1]psi(P) + psi^2(2P) with
//    h_eff = 3(x^2-1) h2 — an endomorphism identity on all of E'(Fp2);
//  * [h2]P = [c]([h_eff]P), c = (3(x^2-1))^-1 mod r, because [h2]P has order r
//    and [r h2] kills E'(Fp2);
//  * on G2 psi acts as [x], and c = d0(1 + x + 2x^2 + 2x^3) - x^2 + x^4 with
//    d0 = 0x460055555555aaab, so [c]Q = [d0](1 + psi + 2psi^2 + 2psi^3)Q
//    + psi^4(Q) - psi^2(Q).
// 191 G2 doublings + ~45 additions instead of 506 + ~250 (derivation checked
// against the plain multiplication in tests/test_gpu_tdec.py).
constexpr uint64_t kCofD0 = 0x460055555555aaabull;

BD G2 g2_add_v(const G2& p, const G2& q) {
    if (fp2_is_zero(p.z)) return q;
    if (fp2_is_zero(q.z)) return p;
    const Fp2 Z1Z1 = fp2_sqr(p.z), Z2Z2 = fp2_sqr(q.z);
    const Fp2 U1 = fp2_mul(p.x, Z2Z2), U2 = fp2_mul(q.x, Z1Z1);
    const Fp2 S1 = fp2_mul(fp2_mul(p.y, q.z), Z2Z2), S2 = fp2_mul(fp2_mul(q.y, p.z), Z1Z1);
    const Fp2 H = fp2_sub(U2, U1);
    const Fp2 rr = fp2_dbl(fp2_sub(S2, S1));
    if (fp2_is_zero(H)) {
        if (fp2_is_zero(rr)) return g2_dbl(p);
        return {fp2_one(), fp2_one(), fp2_zero()};
    }
    const Fp2 I = fp2_sqr(fp2_dbl(H));
    const Fp2 J = fp2_mul(H, I);
    const Fp2 V = fp2_mul(U1, I);
    G2 r;
    r.x = fp2_sub(fp2_sub(fp2_sqr(rr), J), fp2_dbl(V));
    r.y = fp2_sub(fp2_mul(rr, fp2_sub(V, r.x)), fp2_dbl(fp2_mul(S1, J)));
    r.z = fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.z, q.z)), Z1Z1), Z2Z2), H);
    return r;
}
__device__ __noinline__ void g2_add_p(G2* r, const G2* p, const G2* q) { *r = g2_add_v(*p, *q); }
BD G2 g2_add(const G2& p, const G2& q) {
    G2 r;
    g2_add_p(&r, &p, &q);
    return r;
}
BD G2 g2_neg(const G2& p) { return {p.x, fp2_neg(p.y), p.z}; }
// psi(X, Y, Z) = (conj(X) cx, conj(Y) cy, conj(Z)) in Jacobian coordinates
BD G2 g2_psi(const G2& p) {
    return {fp2_mul(fp2_conj(p.x), fp2_const(kPsiX)), fp2_mul(fp2_conj(p.y), fp2_const(kPsiY)), fp2_conj(p.z)};
}
// [k]P for Jacobian P = (X, Y, Z), Z != 0: on the isomorphic curve
// y^2 = x^3 + b' Z^6 ((x, y) -> (x Z^2, y Z^3)) P is the affine (X, Y), so the
// loop runs mixed additions and the result maps back as (X', Y', Z' Z)
BD G2 g2_mul_u64_jac(const G2& p, uint64_t k) {
    const G2 r = g2_mul_u64(p.x, p.y, k);
    return {r.x, r.y, fp2_mul(r.z, p.z)};
}

BD G2 g2_scale_by_cofactor(const Fp2& px, const Fp2& py) {
    const G2 P = {px, py, fp2_one()};
    const G2 nP = g2_neg(P);
    const G2 t1 = g2_neg(g2_mul_u64(px, py, kBlsX));  // [x]P   (x < 0)
    const G2 t2 = g2_neg(g2_mul_u64_jac(t1, kBlsX));   // [x^2]P
    G2 q = g2_add(g2_add(t2, g2_neg(t1)), nP);          // [x^2 - x - 1]P
    q = g2_add(q, g2_psi(g2_add(t1, nP)));              // + psi([x - 1]P)
    q = g2_add(q, g2_psi(g2_psi(g2_dbl(P))));           // + psi^2(2P)  = [h_eff]P
    const G2 s1 = g2_add(q, g2_psi(q));                 // (1 + psi)Q
    const G2 t = g2_add(s1, g2_dbl(g2_psi(g2_psi(s1)))); // (1 + psi + 2psi^2 + 2psi^3)Q
    const G2 q2 = g2_psi(g2_psi(q));
    const G2 q4 = g2_psi(g2_psi(q2));
    return g2_add(g2_mul_u64_jac(t, kCofD0), g2_add(q4, g2_neg(q2)));
}

// ---- quadratic-residue test for the try-and-increment search
// Legendre symbol (a | p) by the binary Jacobi algorithm on the raw limbs.
// A Montgomery value is a R with R = 2^384 a square, so (aR | p) = (a | p).
// ~1k limb operations instead of the ~1.4k field multiplications of a failed
// Fq2::sqrt; returns 1 (square), -1 (non-square) or 0 (a == 0).
BD int fp_legendre(const Fp& a_in) {
    Fp a = a_in, n = fp_const(kP);
    int t = 1;
    for (int guard = 0; guard < 4096; ++guard) {
        bool zero = true;
#pragma unroll
        for (int i = 0; i < 12; ++i) zero &= a[i] == 0u;
        if (zero) break;
        while (a[0] == 0u) {  // whole-limb shift: 32 bits, an even count (no sign change)
#pragma unroll
            for (int i = 0; i < 11; ++i) a[i] = a[i + 1];
            a[11] = 0u;
        }
        const uint32_t z = __builtin_ctz(a[0]);
        if (z) {
#pragma unroll
            for (int i = 0; i < 11; ++i) a[i] = __builtin_amdgcn_alignbit(a[i + 1], a[i], z);
            a[11] >>= z;
            const uint32_t r8 = n[0] & 7u;
            if ((z & 1u) && (r8 == 3u || r8 == 5u)) t = -t;
        }
        // a odd: make a >= n (swap, quadratic reciprocity), then a -= n (even)
        uint32_t br = 0;
#pragma unroll
        for (int i = 0; i < 12; ++i) (void)__builtin_subc(a[i], n[i], br, &br);
        if (br) {
            const Fp tmp = a;
            a = n;
            n = tmp;
            if ((a[0] & 3u) == 3u && (n[0] & 3u) == 3u) t = -t;
        }
        br = 0;
#pragma unroll
        for (int i = 0; i < 12; ++i) a[i] = __builtin_subc(a[i], n[i], br, &br);
    }
    bool one = n[0] == 1u;
#pragma unroll
    for (int i = 1; i < 12; ++i) one &= n[i] == 0u;
    return one ? t : 0;
}
// a in Fq2 is a square iff its norm a0^2 + a1^2 is a square in Fq (p = 3 mod 4)
BD bool fp2_is_square(const Fp2& a) { return fp_legendre(fp_add(fp_sqr(a.c0), fp_sqr(a.c1))) >= 0; }

// hash_g2(digest_input) given its 32-byte SHA3 digest as the ChaCha seed.
// Two phases so a wave clears the cofactor ONCE: lanes find their curve point
// after a different number of tries (geometric, p = 1/2), so a cofactor
// multiplication inside the try loop would run once per distinct exit
// iteration of the wave (~4-6x).  Candidates are screened with the cheap
// Legendre test; the square root is taken once.  Same point, same RNG stream
// as the crate.
BD G2A hash_g2_from_seed(const uint8_t seed[32]) {
    ChaChaRng rng;
    rng.init(seed);
    const Fp2 b2 = {fp_const(kB2), fp_const(kB2)};
    // ~half of all x give a curve point; 128 failures (< 2^-128) never happen —
    // the bounds only guarantee termination.
    for (int round = 0; round < 4; ++round) {
        Fp2 x = fp2_zero(), yy = fp2_zero();
        bool found = false, gr = false;
        for (int tries = 0; tries < 128 && !found; ++tries) {
            Fp2 xt;
            xt.c0 = rand_fq(rng);
            xt.c1 = rand_fq(rng);
            const bool greatest = (rng.next_u32() & 1u) != 0;
            if (!fp2_is_square(fp2_add(fp2_mul(fp2_sqr(xt), xt), b2))) continue;
            x = xt;
            gr = greatest;
            found = true;
        }
        if (!found) break;
        bool ok;
        const Fp2 y = fp2_sqrt(fp2_add(fp2_mul(fp2_sqr(x), x), b2), ok);  // ok: x^3 + b is a square
        const Fp2 ny = fp2_neg(y);
        // the crate: y if (y < negy) ^ greatest else negy
        yy = (fp2_gt(ny, y) != gr) ? y : ny;
        const G2A h = g2_to_affine(g2_scale_by_cofactor(x, yy));
        if (!h.inf) return h;  // an identity after clearing: the crate draws again
    }
    return {fp2_zero(), fp2_zero(), true};
}

// ------------------------------------------------------------------ G2Prepared
// coeff layout per point: [68][c0.c0, c0.c1, c1.c0, c1.c1, c2.c0, c2.c1][12 u32]
BD void store_fp(uint32_t* dst, const Fp& a) {
#pragma unroll
    for (int i = 0; i < 12; ++i) dst[i] = a[i];
}
BD Fp load_fp(const uint32_t* src) {
    Fp r;
#pragma unroll
    for (int i = 0; i < 12; ++i) r[i] = src[i];
    return r;
}
BD void store_line(uint32_t* dst, const LineCoeff& c) {
    store_fp(dst + 0, c.c0.c0);
    store_fp(dst + 12, c.c0.c1);
    store_fp(dst + 24, c.c1.c0);
    store_fp(dst + 36, c.c1.c1);
    store_fp(dst + 48, c.c2.c0);
    store_fp(dst + 60, c.c2.c1);
}
BD LineCoeff load_line(const uint32_t* src) {
    LineCoeff c;
    c.c0 = {load_fp(src + 0), load_fp(src + 12)};
    c.c1 = {load_fp(src + 24), load_fp(src + 36)};
    c.c2 = {load_fp(src + 48), load_fp(src + 60)};
    return c;
}

// |x| >> 1 = 0x6900800000008000: the 62 bits below its leading one drive the loop.
constexpr uint64_t kXHalf = kBlsX >> 1;

BD void g2_prepare(const Fp2& qx, const Fp2& qy, uint32_t* out) {
    G2 r = {qx, qy, fp2_one()};
    int k = 0;
    for (int i = 61; i >= 0; --i) {
        store_line(out + 72 * k++, g2_doubling_step(r));
        if ((kXHalf >> i) & 1ull) store_line(out + 72 * k++, g2_addition_step(r, qx, qy));
    }
    store_line(out + 72 * k, g2_doubling_step(r));
}

// Miller loop over two pairs with prepared lines (the crate's miller_loop),
// register-resident (bls.h: the Fp12 tower inlined down to fp_mul / fp_sqr).
// The crate's order — for each bit i = 61..0 of |x|>>1 below its top: the
// doubling line, the addition line when the bit is set, then f^2; last the
// final doubling line — is flattened into one loop over the 68 lines with
// "f^2 after line k" from a constant schedule, and the two pairs into an
// inner loop, so the kernel holds ONE inlined line evaluation and ONE
// squaring (code size: the body is ~80 multiplication call sites).  A pair is
// skipped when its G1 or G2 point is the identity.
struct MillerSched {
    uint32_t w[3];
};
constexpr MillerSched miller_sched() {
    MillerSched s{{0u, 0u, 0u}};
    int k = 0;
    for (int i = 61; i >= 0; --i) {
        ++k;                              // doubling line
        if ((kXHalf >> i) & 1ull) ++k;    // addition line
        s.w[(k - 1) >> 5] |= 1u << ((k - 1) & 31);  // f^2 after line k - 1
    }
    return s;
}
constexpr MillerSched kMillerSqr = miller_sched();
static_assert(kMillerSqr.w[2] >> 3 == 0, "68 lines: f^2 never follows the last one");

// JAC: pair j's G1 point is Jacobian (X, Y, Z), passed as (a, b, z) =
// (XZ, Y, Z^3): each line value at (X/Z^2, Y/Z^3) is taken times Z^3
// (c2 Z^3 + c1 XZ + c0 Y), an Fp factor that the final exponentiation maps
// to 1 ((p - 1) divides (p^12 - 1) / r) — no inversion for a conversion to
// affine.  Otherwise (a, b) = affine (x, y) and z is unused.
//
// The accumulator f lives in LDS, not in registers: 72 u64 words per lane,
// word w of lane l at f[64 w + l] (a wave's ds_read_b64 of one word is 512
// contiguous bytes: conflict-free), 36 KiB per one-wave workgroup, so four
// such waves per CU fit in its 160 KiB.  A line evaluation or a squaring
// reads the halves it needs when it needs them (a compiler fence between the
// phases forces the re-read instead of keeping a loaded half live), so at
// most ~3 Fp6 plus the multiplication window are in registers.  With f in
// registers (round 4) the 144 words of f beside those temporaries overflowed
// 256 VGPRs + 256 AGPRs: ~5 KB of scratch reloads per Miller step per lane,
// ~450 KB per pairing check (profiles/r05 PMC), the pairing kernels' traffic.
BD void lds_fence() { asm volatile("" ::: "memory"); }
BD Fp lds_fp(const uint64_t* f, int i) {
    Fp r;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const uint64_t v = f[64 * (6 * i + k)];
        r[2 * k] = (uint32_t)v;
        r[2 * k + 1] = (uint32_t)(v >> 32);
    }
    return r;
}
BD void lds_st_fp(uint64_t* f, int i, const Fp& a) {
#pragma unroll
    for (int k = 0; k < 6; ++k) f[64 * (6 * i + k)] = (uint64_t)a[2 * k] | ((uint64_t)a[2 * k + 1] << 32);
}
BD Fp6 lds_fp6(const uint64_t* f, int h) {
    return {{lds_fp(f, 6 * h), lds_fp(f, 6 * h + 1)},
            {lds_fp(f, 6 * h + 2), lds_fp(f, 6 * h + 3)},
            {lds_fp(f, 6 * h + 4), lds_fp(f, 6 * h + 5)}};
}
BD void lds_st_fp6(uint64_t* f, int h, const Fp6& a) {
    lds_st_fp(f, 6 * h, a.c0.c0);
    lds_st_fp(f, 6 * h + 1, a.c0.c1);
    lds_st_fp(f, 6 * h + 2, a.c1.c0);
    lds_st_fp(f, 6 * h + 3, a.c1.c1);
    lds_st_fp(f, 6 * h + 4, a.c2.c0);
    lds_st_fp(f, 6 * h + 5, a.c2.c1);
}
// f *= (c0 + c1 v + c4 v w): fp12_mul_by_014_v on the LDS accumulator
BD void lds_mul_by_014(uint64_t* f, const Fp2& c0, const Fp2& c1, const Fp2& c4) {
    const Fp6 aa = fp6_mul_by_01(lds_fp6(f, 0), c0, c1);
    lds_fence();
    const Fp6 bb = fp6_mul_by_1(lds_fp6(f, 1), c4);
    lds_fence();
    const Fp6 t = fp6_mul_by_01(fp6_add(lds_fp6(f, 1), lds_fp6(f, 0)), c0, fp2_add(c1, c4));
    lds_fence();
    lds_st_fp6(f, 1, fp6_sub(fp6_sub(t, aa), bb));
    lds_st_fp6(f, 0, fp6_add(fp6_mul_by_v(bb), aa));
    lds_fence();
}
// f = f^2: fp12_sqr_v on the LDS accumulator
BD void lds_sqr(uint64_t* f) {
    const Fp6 ab = fp6_mul(lds_fp6(f, 0), lds_fp6(f, 1));
    lds_fence();
    const Fp6 s = fp6_mul(fp6_add(fp6_mul_by_v(lds_fp6(f, 1)), lds_fp6(f, 0)), fp6_add(lds_fp6(f, 0), lds_fp6(f, 1)));
    lds_fence();
    lds_st_fp6(f, 0, fp6_sub(fp6_sub(s, ab), fp6_mul_by_v(ab)));
    lds_st_fp6(f, 1, fp6_add(ab, ab));
    lds_fence();
}

template <bool JAC>
BD Fp12 miller_loop2(const uint32_t* c1, const Fp& a1, const Fp& b1, const Fp& z1, bool use1, const uint32_t* c2,
                     const Fp& a2, const Fp& b2, const Fp& z2, bool use2) {
    // one accumulator per lane, lane-strided: correct for workgroups of at most
    // 64 lanes.  Every caller is a TDEC_KERNEL / TDEC_WAVE1_KERNEL, whose
    // __launch_bounds__(64) makes a larger launch fail at launch time; the
    // diagnostic build also traps here.
    __shared__ uint64_t f_lds[72 * 64];
#ifdef HBG_DEBUG_CHECKS
    if (blockDim.x * blockDim.y * blockDim.z > 64) __builtin_trap();
#endif
    uint64_t* f = f_lds + threadIdx.x;
    lds_st_fp6(f, 0, fp6_one());
    lds_st_fp6(f, 1, fp6_zero());
    lds_fence();
#pragma unroll 1
    for (int k = 0; k < kMillerSteps; ++k) {
#pragma unroll 1
        for (int j = 0; j < 2; ++j) {
            if (j ? use2 : use1) {
                const LineCoeff c = load_line((j ? c2 : c1) + 72 * k);
                const Fp a = j ? a2 : a1, b = j ? b2 : b1;
                if constexpr (JAC) {
                    const Fp z = j ? z2 : z1;
                    lds_mul_by_014(f, fp2_mul_fp(c.c2, z), fp2_mul_fp(c.c1, a), fp2_mul_fp(c.c0, b));
                } else {
                    lds_mul_by_014(f, c.c2, fp2_mul_fp(c.c1, a), fp2_mul_fp(c.c0, b));
                }
            }
        }
        if ((kMillerSqr.w[k >> 5] >> (k & 31)) & 1u) lds_sqr(f);
    }
    return fp12_conj({lds_fp6(f, 0), lds_fp6(f, 1)});
}

// one pairing check: prod e(P_i, Q_i) == 1 over the two prepared pairs
// (miller_loop2's LDS accumulator: callable only from kernels of <= 64 lanes
// a workgroup — the TDEC kernel macros' __launch_bounds__(64))
BD bool pairing_check2(const uint32_t* c1, const Fp& p1x, const Fp& p1y, bool use1, const uint32_t* c2,
                       const Fp& p2x, const Fp& p2y, bool use2) {
    Fp12 f = miller_loop2<false>(c1, p1x, p1y, p1y, use1, c2, p2x, p2y, p2y, use2);
    final_exponentiation(&f);
    return fp12_is_one(f);
}

// e(P1, Q1) e(P2, Q2) in GT for Jacobian P1, P2 (an identity point: its pair is
// skipped; <= 64-lane workgroups, as pairing_check2)
BD Fp12 pairing_value2_jac(const uint32_t* c1, const G1& p1, const uint32_t* c2, const G1& p2, bool use2) {
    const bool u1 = !fp_is_zero(p1.z), u2 = use2 && !fp_is_zero(p2.z);
    const Fp z1 = fp_sqr(p1.z), z2 = fp_sqr(p2.z);
    Fp12 f = miller_loop2<true>(c1, fp_mul(p1.x, p1.z), p1.y, fp_mul(z1, p1.z), u1, c2, fp_mul(p2.x, p2.z), p2.y,
                                fp_mul(z2, p2.z), u2);
    final_exponentiation(&f);
    return f;
}

// ------------------------------------------------------------------ kernels
// Ciphertext preparation (round 5): tdec_ct_decode — U decoded with its
// subgroup check: U's affine record and U's status, all that the share leaves
// read; H = hash_g1_g2(U, V) (SHA3(V) for |V| > 64, try-and-increment,
// cofactor clearing) and its G2Prepared lines (tdec_ct_prepare); on the
// second stream, beside H and the share leaves, W decoded with its subgroup
// check (the final status: U's, else W's) and its lines (tdec_ct_prepare_w),
// which only the check rounds and Ciphertext::verify read, after the
// caller's wait for them.
TDEC_KERNEL void tdec_ct_decode(uint32_t n, const uint8_t* __restrict__ U48, uint32_t* __restrict__ ct_u,
                                int32_t* __restrict__ u_status) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    G1A u;
    const bool u_ok = g1_decompress(U48 + 48ull * k, u, true);
    uint32_t* cu = ct_u + 32ull * k;
    store_fp(cu, u.x);
    store_fp(cu + 12, u.y);
    cu[24] = u.inf ? 1u : 0u;
    u_status[k] = u_ok ? 0 : HBG_E_INVALID_POINT;
}

// W: decode + subgroup check, the ciphertext's final status, W's lines
BD void ct_w_body(uint32_t k, const uint8_t* __restrict__ W96, uint32_t* __restrict__ ct_u,
                  const int32_t* __restrict__ u_status, int32_t* __restrict__ ct_status, uint32_t* __restrict__ coefW) {
    G2A w;
    const bool w_ok = g2_decompress(W96 + 96ull * k, w, true);
    ct_u[32ull * k + 25] = w.inf ? 1u : 0u;
    const int32_t us = u_status[k];
    const int32_t st = us != 0 ? us : (w_ok ? 0 : HBG_E_INVALID_POINT);
    ct_status[k] = st;
    if (st == 0 && !w.inf) g2_prepare(w.x, w.y, coefW + (uint64_t)k * 72 * kMillerSteps);
}
TDEC_WAVE1_KERNEL void tdec_ct_prepare_w(uint32_t n, const uint8_t* __restrict__ W96, uint32_t* __restrict__ ct_u,
                                         const int32_t* __restrict__ u_status, int32_t* __restrict__ ct_status,
                                         uint32_t* __restrict__ coefW) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) ct_w_body(k, W96, ct_u, u_status, ct_status, coefW);
}

// H = hash_g1_g2(U, V) and its G2Prepared lines, for the ciphertexts whose U
// decodes (status: U's; a ciphertext whose W fails too gets an unused H).
// vdig: SHA3(V) of the items with |V| > 64 (tdec_v_digest), or null: hashed
// here, one lane per item.
BD void ct_h_body(uint32_t k, const uint8_t* __restrict__ U48, const uint8_t* __restrict__ V,
                  const uint64_t* __restrict__ V_off, const uint8_t* __restrict__ vdig,
                  const int32_t* __restrict__ u_status, uint32_t* __restrict__ coefH) {
    if (u_status[k] != 0) return;
    // H = hash_g1_g2(U, V): m = (|V| > 64 ? sha3(V) : V) || compress(U)
    const uint64_t off = V_off[k], len = V_off[k + 1] - off;
    uint8_t dg[32];
    if (!vdig && len > 64) sha3_long(V + off, len, dg);
    uint8_t m[64 + 48];
    const uint32_t ml = hash_g1_g2_msg(V + off, len, vdig ? vdig + 32ull * k : dg, U48 + 48ull * k, m);
    uint8_t seed[32];
    sha3_bytes(m, ml, seed);
    const G2A h = hash_g2_from_seed(seed);
    g2_prepare(h.x, h.y, coefH + (uint64_t)k * 72 * kMillerSteps);
}
TDEC_WAVE1_KERNEL void tdec_ct_prepare(uint32_t n, const uint8_t* __restrict__ U48, const uint8_t* __restrict__ V,
                                       const uint64_t* __restrict__ V_off, const uint8_t* __restrict__ vdig,
                                       const int32_t* __restrict__ u_status, uint32_t* __restrict__ coefH) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) ct_h_body(k, U48, V, V_off, vdig, u_status, coefH);
}

// H (sponge inline) and W in ONE launch, for the batched schedule's few
// thousand ciphertexts (api.hip launch_lines): blocks [0, nb) build H's lines,
// [nb, 2 nb) W's.  Launched beside the share leaves; as two launches on two
// extra streams the second sat behind the first (the runtime put both streams
// on one hardware queue), so one grid keeps the two concurrent.
TDEC_WAVE1_KERNEL void tdec_ct_prepare_hw(uint32_t n, const uint8_t* __restrict__ U48, const uint8_t* __restrict__ V,
                                          const uint64_t* __restrict__ V_off, const uint8_t* __restrict__ W96,
                                          uint32_t* __restrict__ ct_u, const int32_t* __restrict__ u_status,
                                          int32_t* __restrict__ ct_status, uint32_t* __restrict__ coefH,
                                          uint32_t* __restrict__ coefW) {
    const uint32_t nb = (n + 63) / 64;
    if (blockIdx.x < nb) {
        const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
        if (k < n) ct_h_body(k, U48, V, V_off, nullptr, u_status, coefH);
    } else {
        const uint32_t k = (blockIdx.x - nb) * blockDim.x + threadIdx.x;
        if (k < n) ct_w_body(k, W96, ct_u, u_status, ct_status, coefW);
    }
}

// Affine record (kAffWords words: x[12] y[12] inf): pk tables and the
// verified-share table the combine reads.
BD void store_aff(uint32_t* d, const G1A& p) {
    store_fp(d, p.x);
    store_fp(d + 12, p.y);
    d[24] = p.inf ? 1u : 0u;
}

TDEC_KERNEL void tdec_pk_prepare(uint32_t n, const uint8_t* __restrict__ pk48,
                                                      uint32_t* __restrict__ pk_aff, int32_t* __restrict__ pk_status) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    G1A p;
    const bool ok = g1_decompress(pk48 + 48ull * k, p, true);
    store_aff(pk_aff + 32ull * k, p);
    pk_status[k] = ok ? 0 : HBG_E_INVALID_POINT;
}

TDEC_WAVE1_KERNEL void tdec_verify_shares(uint64_t cap, const uint32_t* __restrict__ n_dev,
                                                         const uint8_t* __restrict__ share48,
                                                         const uint32_t* __restrict__ share_ct,
                                                         const uint32_t* __restrict__ share_pk,
                                                         const uint32_t* __restrict__ ct_u,
                                                         const int32_t* __restrict__ ct_status,
                                                         const uint32_t* __restrict__ coefH,
                                                         const uint32_t* __restrict__ coefW,
                                                         const uint32_t* __restrict__ pk_aff,
                                                         const int32_t* __restrict__ pk_status,
                                                         uint8_t* __restrict__ ok, const uint32_t* __restrict__ sel,
                                                         uint32_t* __restrict__ share_aff) {
    const uint64_t i = grid_lane();
    if (i >= dev_count(n_dev, cap)) return;
    const uint64_t k = sel ? sel[i] : i;  // sel: share indices (batched path's failing leaves)
#ifdef HBG_DEBUG_CHECKS
    if (!HBG_DBG_RANGE(k, g_dbg[0], "verify_shares k")) return;
#endif
    const uint32_t ct = share_ct[k], pk = share_pk[k];  // sanitised: invalid pairs point at the sentinels
#ifdef HBG_DEBUG_CHECKS
    if (!HBG_DBG_RANGE(ct, g_dbg[2], "verify_shares ct") || !HBG_DBG_RANGE(pk, g_dbg[3], "verify_shares pk")) return;
#endif
    bool good = ct_status[ct] == 0 && pk_status[pk] == 0;
    G1A s;
    if (sel && share_aff) {  // a batched leaf: decoded and subgroup-checked by tdec_batch_leaves, its point stored
        const uint32_t* sa = share_aff + (uint64_t)kAffWords * k;
        s = {load_fp(sa), load_fp(sa + 12), sa[24] != 0};
    } else {
        if (good) good = g1_decompress(share48 + 48ull * k, s, true);
        if (good && share_aff) store_aff(share_aff + (uint64_t)kAffWords * k, s);
    }
    if (good) {
        const uint32_t* pa = pk_aff + 32ull * pk;
        const Fp pkx = load_fp(pa), pky = fp_neg(load_fp(pa + 12));
        const bool pk_inf = pa[24] != 0;
        const bool w_inf = ct_u[32ull * ct + 25] != 0;
        good = pairing_check2(coefH + (uint64_t)ct * 72 * kMillerSteps, s.x, s.y, !s.inf,
                              coefW + (uint64_t)ct * 72 * kMillerSteps, pkx, pky, !pk_inf && !w_inf);
    }
    ok[k] = good ? 1 : 0;
}

// Device-mode index check of (ciphertext/document, key) pairs: an out-of-range
// pair is redirected to the sentinel entries (a_bound, b_bound), whose status
// words are invalid, so its ok bit is 0 and nothing out of range is read; the
// call's sticky error becomes HBG_E_ARG.
__global__ __launch_bounds__(256) void tdec_index_sanitize(uint64_t n, const uint32_t* __restrict__ a,
                                                           uint32_t a_bound, const uint32_t* __restrict__ b,
                                                           uint32_t b_bound, uint32_t* __restrict__ a_out,
                                                           uint32_t* __restrict__ b_out, int32_t* __restrict__ err) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t x = a[k], y = b[k];
    const bool good = x < a_bound && y < b_bound;
    a_out[k] = good ? x : a_bound;
    b_out[k] = good ? y : b_bound;
    if (!good) flag_error(err, HBG_E_ARG);
}


// ---------------------------------------------------------------- batched share verification
// verify_decryption_share for many shares of ONE ciphertext c shares (H, W):
// e(S_i, H) == e(PK_i, W) for all i in a batch  <=  e(sum r_i S_i, H) ==
// e(sum r_i PK_i, W) with secret 127-bit weights r_i (Bellare-Garay-Rabin
// small-exponent batch test).  r_i = a + b|x| + c x^2 + d|x|^3 with a (odd),
// b, c, d the four 32-bit words of SHA3(K || D || i) (w4_weight; the coin
// shares' leaves use r_i = a + b x^2 with the two 64-bit halves instead,
// batch_weight): K is the context's secret batch key (32 bytes from getrandom
// at hbg_init, never exposed), D a digest of the whole batch.  Either way the
// 2^127 tuples are 2^127 distinct integers below the group order (every digit
// is below its base: a < 2^64 < x^2, resp. 32-bit quarters < |x|), so for any batch holding an invalid share
// and any fixed choice of the other weights at most one value of r_i makes the
// weighted product 1: a (sub)tree holding an invalid share passes with
// probability <= 2^-127, and no sender can grind shares against the weights
// offline (without K they are unpredictable).  A batch is up to 64
// shares of one ciphertext, tested as a BINARY tree with sibling derivation
// (round 5): round 0 checks every batch sum; a failing node's left child is
// checked and its right child's value is DERIVED — the checks are values in
// GT (e(sum r S, H) e(-sum r PK, W) after the final exponentiation), which
// multiply over disjoint leaf sets, so right = parent * left^-1 (the inverse
// in the cyclotomic subgroup is the conjugate).  Each failing node costs one
// pairing, and six rounds (32, 16, 8, 4, 2, 1 shares) reach the single
// shares.  A single's value is g^r for g = e(S, H) e(-PK, W) and its weight r
// (nonzero and below the group order), so it is 1 exactly when the
// reference's per-share equation holds: every reported 0 is that equation's
// verdict, every 1 a passing (sub)tree's.  Round 4's 4-ary
// tree (4 checks per failing node, three rounds) ran its rounds at 2-4 full
// generations of one wave per SIMD; here a round holds ~one check per bad
// share (<= 64 k items at 1 % of 6.4 M: one generation).
struct BatchDesc {
    uint32_t start, end, ct, pad;
};
struct CheckItem {
    uint32_t b, node;  // node 0..15: quad, 16..19: 16-share group, 20: whole batch
};
constexpr uint32_t kJacWords = 36;                    // Jacobian G1: x, y, z
constexpr uint32_t kSumWords = 2 * kJacWords;         // (sum r S, sum r PK)
// 4-ary group-testing tree of the coin-share batches (sig_*): nodes 0..15 =
// quads (4 shares), 16..19 = 16-share groups, 20 = the batch.
constexpr uint32_t kNodes = 21, kNodeBatch = 20, kNode16 = 16;
// Binary tree of the decryption-share batches: heap ids (root 1, children 2h
// and 2h + 1, single shares 64..127).  Stored per batch: the root (slot 0)
// and every LEFT node h (slot h / 2) — the right ones are derived.
constexpr uint32_t kBinSlots = 64;
constexpr uint32_t kBatchSumWords = kBinSlots * kSumWords;
static_assert(kBatchSumBytes == 4 * kBatchSumWords, "tdec_kernels.h");
constexpr uint32_t kGtWords = 144;  // a GT value: Fp12 after the final exponentiation
struct BinItem {
    uint32_t b;      // batch
    uint32_t h;      // the LEFT child to check (even heap id); its sibling h + 1 is derived
    uint32_t ppos;   // the parent's GT value: item ppos of the previous round (round 1: batch ppos)
    uint32_t pside;  // 0: that item's checked node, 1: its derived node
};
static_assert(sizeof(BinItem) == kBinItemBytes, "tdec_kernels.h");
BD uint32_t bin_depth(uint32_t h) { return 31u - __builtin_clz(h); }
BD uint32_t bin_size(uint32_t h) { return kBatchShares >> bin_depth(h); }
BD uint32_t bin_first(uint32_t h) { return (h - (1u << bin_depth(h))) * bin_size(h); }

__global__ void tdec_iota(uint32_t n, uint32_t* __restrict__ v) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

// gs[q] = q where the (sorted) ciphertext key changes, else 0 (max-scan -> group start)
__global__ void tdec_group_marks(uint32_t n, const uint32_t* __restrict__ key, uint32_t* __restrict__ gs) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) gs[q] = (q == 0 || key[q] != key[q - 1]) ? q : 0u;
}

__global__ void tdec_batch_heads(uint32_t n, const uint32_t* __restrict__ gs, uint32_t* __restrict__ head) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) head[q] = ((q - gs[q]) % kBatchShares == 0) ? 1u : 0u;
}

__global__ void tdec_batch_desc(uint32_t n, const uint32_t* __restrict__ key, const uint32_t* __restrict__ head,
                                const uint32_t* __restrict__ bid, BatchDesc* __restrict__ desc) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const uint32_t b = bid[q] - 1u;  // bid: inclusive count of batch heads in [0, q]
    if (head[q]) {
        desc[b].start = q;
        desc[b].ct = key[q];
    }
    if (q + 1 == n || head[q + 1]) desc[b].end = q + 1;
}

BD void store_jac(uint32_t* d, const G1& p) {
    store_fp(d, p.x);
    store_fp(d + 12, p.y);
    store_fp(d + 24, p.z);
}
BD G1 load_jac(const uint32_t* d) { return {load_fp(d), load_fp(d + 12), load_fp(d + 24)}; }

BD G1 g1_shfl_xor(const G1& p, int m) {
    G1 r;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        r.x[i] = __shfl_xor(p.x[i], m);
        r.y[i] = __shfl_xor(p.y[i], m);
        r.z[i] = __shfl_xor(p.z[i], m);
    }
    return r;
}

// Fixed-base tables of the public key shares for the batch weights:
// tbl[pk][w][v] (v in 1..255; v = 0 unused), affine.  Layout 0 (the coin
// shares' 64-bit halves a + b x^2): [v 2^(8w)] PK for w in 0..7, so [a] PK is
// 8 mixed additions, no doublings (the b half reads the same entries through
// (beta x, -y)).  Layout 1 (the decryption shares' four 32-bit quarters
// a + b|x| + c x^2 + d|x|^3, w4_weight): [v 2^(8w)] PK for w in 0..3 and
// [v 2^(8(w - 4))] ([|x|] PK) for w in 4..7 — 16 mixed additions either way.
constexpr uint32_t kPkTblWords = 8 * 256 * 24;
TDEC_KERNEL void tdec_pk_table(uint32_t n_pk, const uint32_t* __restrict__ pk_aff,
                                                    uint32_t* __restrict__ tbl, uint32_t layout) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // (pk, w, v)
    if (i >= n_pk * 2048u) return;
    const uint32_t pk = i >> 11, w = (i >> 8) & 7u, v = i & 255u;
    const uint32_t* pa = pk_aff + 32ull * pk;
    uint32_t* o = tbl + (uint64_t)pk * kPkTblWords + (uint64_t)(w * 256 + v) * 24;
    if (v == 0 || pa[24] != 0) return;
    const Fp px = load_fp(pa), py = load_fp(pa + 12);
    G1 e;
    if (layout == 1 && w >= 4) {
        // [|x|] PK != O for PK in G1 (pk_prepare checked the subgroup)
        e = g1_mul_u64_jac(g1_mul_u64(px, py, kBlsX), (uint64_t)v << (8 * (w - 4)));
    } else {
        e = g1_mul_u64(px, py, (uint64_t)v << (8 * w));
    }
    const G1A r = g1_to_affine(e);
    store_fp(o, r.x);
    store_fp(o + 12, r.y);
}

// One 64-lane block per batch: lane = share.  Decompress + subgroup check,
// weight, and the quad / 16-group / batch sums by cross-lane butterfly
// (ds_swizzle/bpermute shuffles: no LDS for the points, so occupancy is set
// by VGPRs alone).
// [a]P + [b]([x^2]P) for P in G1 (affine) and 64-bit a, b: on G1 [x^2]P =
// -phi(P) = (beta px, -py), so the batch weight r = a + b x^2 (mod r; the
// 2^128 pairs give 2^128 distinct weights) costs a 64-bit joint double-and-add
// (branch-free addend select, as g1_mul_fr) instead of a 128-bit one.
// The three addends P, [x^2]P and both = P + [x^2]P = (X, Y, Z) share one
// denominator on the isomorphic curve E_Z: y^2 = x^3 + 4 Z^6, reached by
// (x, y) -> (x Z^2, y Z^3): there both is the affine (X, Y) and P, [x^2]P are
// (px Z^2, py Z^3), (beta px Z^2, -py Z^3).  The a = 0 doubling and mixed
// addition formulas never read the curve constant, so the loop runs on E_Z
// with mixed additions (11 multiplications instead of 16) and the result
// (X', Y', Z') maps back to E as (X', Y', Z' Z).  Z != 0: (1 + x^2) P != O
// for P in G1.
BD G1 g1_mul_ab64(const Fp& px, const Fp& py, uint64_t a, uint64_t b) {
    const G1 both = g1_add_mixed({px, py, fp_one()}, fp_mul(px, fp_const(kBeta)), fp_neg(py));
    Fp z2 = fp_sqr(both.z), z3, tx, ty;
    z3 = fp_mul(z2, both.z);
    fp_mul2(tx, ty, px, z2, py, z3);
    const Fp ux = fp_mul(tx, fp_const(kBeta)), uy = fp_neg(ty);
    G1 r = {fp_one(), fp_one(), fp_zero()};
#pragma unroll 1
    for (int bit = 63; bit >= 0; --bit) {
        r = g1_dbl(r);
        const bool ea = (a >> bit) & 1u, eb = (b >> bit) & 1u;
        const G1 sum = g1_add_mixed(r, ea ? (eb ? both.x : tx) : ux, ea ? (eb ? both.y : ty) : uy);
        if (ea || eb) r = sum;
    }
    return {r.x, r.y, fp_mul(r.z, both.z)};
}

// The batch weight of lane i: (a, b) = the two 64-bit halves of
// SHA3(K || D || i) (K: the context's secret batch key, D: the batch digest),
// a forced odd so r = a + b x^2 is never 0.
BD void batch_weight(const BatchKey& key, const uint8_t* D, uint32_t lane, uint64_t& a, uint64_t& b) {
    uint8_t m[68], dg[32];
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 4; ++j) m[4 * i + j] = (uint8_t)(key.w[i] >> (8 * j));
    for (int i = 0; i < 32; ++i) m[32 + i] = D[i];
    for (int i = 0; i < 4; ++i) m[64 + i] = (uint8_t)(lane >> (8 * i));
    sha3_bytes(m, 68, dg);
    a = 0;
    b = 0;
    for (int i = 0; i < 8; ++i) {
        a |= (uint64_t)dg[i] << (8 * i);
        b |= (uint64_t)dg[8 + i] << (8 * i);
    }
    a |= 1u;
}

// ---- the decryption shares' weights: four 32-bit quarters -------------------
// r = a + b|x| + c x^2 + d|x|^3 (a odd), a, b, c, d the four LE 32-bit words of
// SHA3(K || D || lane) — the same key, digest and derivation as batch_weight.
// 2^127 distinct integers (the quarters are below |x| > 2^63, so the base-|x|
// representation is unique) below 2^224 < the group order, nonzero (a odd).
// On G1, [x^2]P = -phi(P) = (beta x, -y) and [|x|^3]P = -phi([|x|]P), and
// [|x|]P is the subgroup check's intermediate (g1_subgroup_t1): the four
// points cost nothing extra, and r P is two 32-step joint double-and-adds
// sharing their 32 doublings (g1_mul_w4) instead of one 64-step one.
struct W4 {
    uint32_t a, b, c, d;
};
BD W4 w4_weight(const BatchKey& key, const uint8_t* D, uint32_t lane) {
    uint8_t m[68], dg[32];
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 4; ++j) m[4 * i + j] = (uint8_t)(key.w[i] >> (8 * j));
    for (int i = 0; i < 32; ++i) m[32 + i] = D[i];
    for (int i = 0; i < 4; ++i) m[64 + i] = (uint8_t)(lane >> (8 * i));
    sha3_bytes(m, 68, dg);
    auto word = [&](int k) {
        return (uint32_t)dg[4 * k] | ((uint32_t)dg[4 * k + 1] << 8) | ((uint32_t)dg[4 * k + 2] << 16) |
               ((uint32_t)dg[4 * k + 3] << 24);
    };
    return {word(0) | 1u, word(1), word(2), word(3)};
}

// P in G1 (g1_in_subgroup's test, phi(P) == [-x^2]P), keeping T1 = [|x|]P
// (Jacobian, Z != 0 when the test passes) for g1_mul_w4.
BD bool g1_subgroup_t1(const Fp& px, const Fp& py, G1& t1) {
    t1 = g1_mul_u64(px, py, kBlsX);
    if (fp_is_zero(t1.z)) return false;
    const G1 u = g1_mul_u64_jac(t1, kBlsX);
    if (fp_is_zero(u.z)) return false;
    const Fp z2 = fp_sqr(u.z), z3 = fp_mul(z2, u.z);
    return fp_eq(fp_mul(fp_mul(px, fp_const(kBeta)), z2), u.x) && fp_eq(fp_mul(py, z3), fp_neg(u.y));
}

// [a + b|x| + c x^2 + d|x|^3] P for P in G1 (affine, not infinity) and
// T1 = [|x|]P (Jacobian): pair A = (P, -phi P, their sum) takes the (a, c)
// bits, pair B = (T1, -phi T1, their sum) the (b, d) bits; per step one
// doubling and two branch-free mixed additions.  All six addends are put on
// one isomorphic curve E_W: y^2 = x^3 + 4 W^6, W = Z_A Z_B Z_1 (a Jacobian
// (X, Y, Z) is the affine (X (W/Z)^2, Y (W/Z)^3) there; the a = 0 formulas
// never read the constant), and the result maps back as (X', Y', Z' W).
// Z_A, Z_B, Z_1 != 0 for P != O in G1 (phi has no eigenvalue -1 there).
BD G1 g1_mul_w4(const Fp& px, const Fp& py, const G1& t1, const W4& k) {
    const Fp bx = fp_mul(px, fp_const(kBeta));
    const G1 sa = g1_add_mixed({px, py, fp_one()}, bx, fp_neg(py));           // P - phi P
    const G1 tc = {fp_mul(t1.x, fp_const(kBeta)), fp_neg(t1.y), t1.z};        // -phi T1
    const G1 sb = g1_add(t1, tc);                                              // T1 - phi T1
    Fp zab, zb1, za1;
    fp_mul3(zab, zb1, za1, sa.z, sb.z, sb.z, t1.z, sa.z, t1.z);
    const Fp W = fp_mul(zab, t1.z);                                            // lambda of P, -phi P
    // lambda^2, lambda^3 of P (W), T1 (zab), A (zb1), B (za1)
    Fp w2, t2, a2, b2, w3, t3, a3, b3;
    fp_mul2(w2, t2, W, W, zab, zab);
    fp_mul2(a2, b2, zb1, zb1, za1, za1);
    fp_mul2(w3, t3, w2, W, t2, zab);
    fp_mul2(a3, b3, a2, zb1, b2, za1);
    Fp pxw, pyw, ax, ay, tx, ty, bxw, byw;
    fp_mul2(pxw, pyw, px, w2, py, w3);
    fp_mul2(ax, ay, sa.x, a2, sa.y, a3);
    fp_mul2(tx, ty, t1.x, t2, t1.y, t3);
    fp_mul2(bxw, byw, sb.x, b2, sb.y, b3);
    const Fp pcx = fp_mul(pxw, fp_const(kBeta));  // -phi P on E_W: (pcx, -pyw)
    const Fp tcx = fp_mul(tx, fp_const(kBeta));   // -phi T1 on E_W: (tcx, -ty)
    G1 r = {fp_one(), fp_one(), fp_zero()};
#pragma unroll 1
    for (int bit = 31; bit >= 0; --bit) {
        r = g1_dbl(r);
        // the y of -phi is the selected y negated per step (a select of a
        // bit-dependent value: not hoisted, two fewer 12-word values live)
        const bool ea = (k.a >> bit) & 1u, ec = (k.c >> bit) & 1u;
        const Fp ya = (ea && ec) ? ay : pyw;
        const G1 s1 = g1_add_mixed(r, ea ? (ec ? ax : pxw) : pcx, ea ? ya : fp_neg(ya));
        if (ea || ec) r = s1;
        const bool eb = (k.b >> bit) & 1u, ed = (k.d >> bit) & 1u;
        const Fp yb = (eb && ed) ? byw : ty;
        const G1 s2 = g1_add_mixed(r, eb ? (ed ? bxw : tx) : tcx, eb ? yb : fp_neg(yb));
        if (eb || ed) r = s2;
    }
    return {r.x, r.y, fp_mul(r.z, W)};
}

// r PK from the key's layout-1 table (tdec_pk_table): the a and c quarters
// from windows 0..3 (c through (beta x, -y) = [x^2]), b and d from windows
// 4..7 ([|x|] PK; d through (beta x, -y)): 16 mixed additions, no doublings.
BD G1 pk_tbl_mul_w4(const uint32_t* t, const W4& k) {
    G1 B = {fp_one(), fp_one(), fp_zero()};
    for (int w = 0; w < 4; ++w) {
        const uint32_t va = (k.a >> (8 * w)) & 255u, vc = (k.c >> (8 * w)) & 255u;
        const uint32_t vb = (k.b >> (8 * w)) & 255u, vd = (k.d >> (8 * w)) & 255u;
        if (va) {
            const uint32_t* e = t + (w * 256 + va) * 24;
            B = g1_add_mixed(B, load_fp(e), load_fp(e + 12));
        }
        if (vc) {
            const uint32_t* e = t + (w * 256 + vc) * 24;
            B = g1_add_mixed(B, fp_mul(load_fp(e), fp_const(kBeta)), fp_neg(load_fp(e + 12)));
        }
        if (vb) {
            const uint32_t* e = t + ((4 + w) * 256 + vb) * 24;
            B = g1_add_mixed(B, load_fp(e), load_fp(e + 12));
        }
        if (vd) {
            const uint32_t* e = t + ((4 + w) * 256 + vd) * 24;
            B = g1_add_mixed(B, fp_mul(load_fp(e), fp_const(kBeta)), fp_neg(load_fp(e + 12)));
        }
    }
    return B;
}

// [a + b x^2] PK from the key's fixed-base table (windows 0..7 of both halves;
// the b half through (beta x, -y)): 16 mixed additions, no doublings.
BD G1 pk_tbl_mul_ab64(const uint32_t* t, uint64_t a, uint64_t b) {
    G1 B = {fp_one(), fp_one(), fp_zero()};
    for (int w = 0; w < 8; ++w) {
        const uint32_t va = (uint32_t)(a >> (8 * w)) & 255u, vb = (uint32_t)(b >> (8 * w)) & 255u;
        if (va) {
            const uint32_t* e = t + (w * 256 + va) * 24;
            B = g1_add_mixed(B, load_fp(e), load_fp(e + 12));
        }
        if (vb) {
            const uint32_t* e = t + (w * 256 + vb) * 24;
            B = g1_add_mixed(B, fp_mul(load_fp(e), fp_const(kBeta)), fp_neg(load_fp(e + 12)));
        }
    }
    return B;
}

TDEC_KERNEL void tdec_batch_leaves(uint32_t cap, const uint32_t* __restrict__ nb_dev, uint32_t n_ct,
                                                        const BatchDesc* __restrict__ desc,
                                                        const uint32_t* __restrict__ perm,
                                                        const uint8_t* __restrict__ share48,
                                                        const uint32_t* __restrict__ share_pk,
                                                        const uint8_t* __restrict__ U48,
                                                        const int32_t* __restrict__ ct_status,
                                                        const uint32_t* __restrict__ pk_aff,
                                                        const int32_t* __restrict__ pk_status,
                                                        const uint32_t* __restrict__ pk_tbl,
                                                        uint32_t* __restrict__ sums, uint8_t* __restrict__ leaf_ok,
                                                        const BatchKey key, uint32_t* __restrict__ share_aff) {
    // ct_status: U's decode status (the ciphertext table's final status, W's
    // decode included, is applied by the root round)
    __shared__ uint8_t sDig[kBatchShares * 32], sBatch[32];
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    if (b >= dev_count(nb_dev, cap)) return;  // grid sized for the bound; the batch count is a device word
    const BatchDesc d = desc[b];
#ifdef HBG_DEBUG_CHECKS
    if (lane == 0 && (!HBG_DBG_RANGE(d.end, g_dbg[0] + 1, "leaves d.end") || !HBG_DBG_RANGE(d.start, d.end, "leaves d.start") ||
                      !HBG_DBG_RANGE(d.end - d.start, 65, "leaves size") || !HBG_DBG_RANGE(d.ct, g_dbg[2], "leaves d.ct")))
        printf("  batch %u of %u\n", b, *nb_dev);
#endif
    const uint32_t q = d.start + lane;
    const bool in = q < d.end;
    const uint32_t k = in ? perm[q] : 0u;
    const uint32_t pk = in ? share_pk[k] : 0u;
    const bool real_ct = d.ct < n_ct;  // the sentinel batch (out-of-range indices) reads no U
    bool valid = in && ct_status[d.ct] == 0 && pk_status[pk] == 0;
    G1A s;
    G1 t1;  // [|x|] S, the subgroup check's intermediate (the weight's b, d points)
    if (valid) valid = g1_decompress(share48 + 48ull * k, s, false);
    if (valid && !s.inf) valid = g1_subgroup_t1(s.x, s.y, t1);
    if (valid && share_aff) store_aff(share_aff + (uint64_t)kAffWords * k, s);  // for the combine
    // Weights: r_i from SHA3(K || D || i) with D = SHA3(d_0 || ...) over the
    // leaf digests d_i = SHA3(U || S_i || pk_i) — secret (K) and bound to the
    // whole batch (changing any share re-randomises every weight).
    if (in && real_ct) {
        uint8_t m[100];
        for (int i = 0; i < 48; ++i) m[i] = U48[48ull * d.ct + i];
        for (int i = 0; i < 48; ++i) m[48 + i] = share48[48ull * k + i];
        for (int i = 0; i < 4; ++i) m[96 + i] = (uint8_t)(pk >> (8 * i));
        sha3_bytes(m, 100, sDig + 32 * lane);
    }
    __syncthreads();
    if (lane == 0) sha3_bytes(sDig, 32u * (d.end - d.start), sBatch);
    __syncthreads();
    G1 A = {fp_one(), fp_one(), fp_zero()}, B = A;
    if (valid) {
        // weight r_i = a + b|x| + c x^2 + d|x|^3 (w4_weight; a odd: nonzero);
        // S_i and pk_i are in G1 (subgroup-checked)
        const W4 w = w4_weight(key, sBatch, lane);
        if (!s.inf) A = g1_mul_w4(s.x, s.y, t1, w);
        const uint32_t* pa = pk_aff + 32ull * pk;
        if (pa[24] == 0) {
            if (pk_tbl) {
                B = pk_tbl_mul_w4(pk_tbl + (uint64_t)pk * kPkTblWords, w);
            } else {
                const Fp px = load_fp(pa), py = load_fp(pa + 12);
                B = g1_mul_w4(px, py, g1_mul_u64(px, py, kBlsX), w);
            }
        }
    }
    leaf_ok[(uint64_t)b * kBatchShares + lane] = valid ? 1 : 0;
    // the binary tree's left nodes (slot h / 2) and the root (slot 0): the
    // weighted single of an even lane, then after each butterfly level the
    // sum of every even group of 2m lanes, held by the group's first lane
    uint32_t* out = sums + (uint64_t)b * kBatchSumWords;
    if ((lane & 1u) == 0) {
        store_jac(out + (32u + (lane >> 1)) * kSumWords, A);
        store_jac(out + (32u + (lane >> 1)) * kSumWords + kJacWords, B);
    }
#pragma unroll 1
    for (uint32_t m = 1; m < 64; m <<= 1) {
        A = g1_add(A, g1_shfl_xor(A, m));
        B = g1_add(B, g1_shfl_xor(B, m));
        const uint32_t gsz = 2u * m;  // group size; group j = lane / gsz is heap node 64 / gsz + j
        const uint32_t slot = gsz == 64 ? 0u : (64u / gsz + lane / gsz) / 2u;
        if ((lane & (2u * gsz - 1u)) == 0 || (gsz == 64 && lane == 0)) {
            store_jac(out + slot * kSumWords, A);
            store_jac(out + slot * kSumWords + kJacWords, B);
        }
    }
}

// Node geometry of a check item in its batch's 4-ary tree: leaf lanes [l0, l1).
BD uint32_t node_size(uint32_t node) { return node == kNodeBatch ? 64u : (node >= kNode16 ? 16u : 4u); }
BD uint32_t node_first(uint32_t node) {
    return node == kNodeBatch ? 0u : (node >= kNode16 ? 16u * (node - kNode16) : 4u * node);
}
BD bool node_any_valid(const uint8_t* lok, uint32_t l0, uint32_t l1) {
    bool any = false;
    for (uint32_t l = l0; l < l1; ++l) any |= lok[l] != 0;
    return any;
}

// One group-testing step for a checked node: a pass vouches for the node's
// valid leaves; a failing batch / 16-group pushes its (non-empty) four
// children; a failing quad appends its valid leaves to the per-share list.
// With `children_checked` (a speculative round that checked a batch together
// with its four 16-groups) a failing batch pushes nothing.
BD void batch_tree_step(bool pass, const CheckItem& it, const BatchDesc& d, const uint8_t* lok,
                        const uint32_t* __restrict__ perm, uint8_t* __restrict__ ok, CheckItem* __restrict__ next,
                        uint32_t* __restrict__ next_n, uint32_t* __restrict__ fail_list,
                        uint32_t* __restrict__ fail_n, bool children_checked = false) {
    const uint32_t size = node_size(it.node), l0 = node_first(it.node), l1 = l0 + size;
    if (pass) {
        for (uint32_t l = l0; l < l1; ++l)
            if (lok[l]) ok[perm[d.start + l]] = 1;
    } else if (children_checked) {
        return;
    } else if (size > 4u) {  // four children of a quarter the size
        const uint32_t cs = size / 4u;
        for (uint32_t c = 0; c < 4; ++c) {
            const uint32_t c0 = l0 + c * cs;
            const uint32_t node = size == 64u ? kNode16 + c : c0 / 4u;
            if (node_any_valid(lok, c0, c0 + cs)) next[atomicAdd(next_n, 1u)] = CheckItem{it.b, node};
        }
    } else {
        for (uint32_t l = l0; l < l1; ++l)
            if (lok[l]) fail_list[atomicAdd(fail_n, 1u)] = perm[d.start + l];
    }
}

// GT values of the binary rounds (kGtWords words, the Fp12's 12 Fp in order)
BD void store_gt(uint32_t* d, const Fp12& v) {
    const Fp x[12] = {v.c0.c0.c0, v.c0.c0.c1, v.c0.c1.c0, v.c0.c1.c1, v.c0.c2.c0, v.c0.c2.c1,
                      v.c1.c0.c0, v.c1.c0.c1, v.c1.c1.c0, v.c1.c1.c1, v.c1.c2.c0, v.c1.c2.c1};
#pragma unroll
    for (int i = 0; i < 12; ++i) store_fp(d + 12 * i, x[i]);
}
BD Fp12 load_gt(const uint32_t* d) {
    auto f2 = [&](int i) { return Fp2{load_fp(d + 12 * i), load_fp(d + 12 * i + 12)}; };
    return {{f2(0), f2(2), f2(4)}, {f2(6), f2(8), f2(10)}};
}

// GT value of one stored node (slot) of batch d: e(sum r S, H) e(-sum r PK, W)
BD Fp12 bin_node_value(const uint32_t* __restrict__ sums, uint32_t b, uint32_t slot, const BatchDesc& d,
                       const uint32_t* __restrict__ ct_u, const uint32_t* __restrict__ coefH,
                       const uint32_t* __restrict__ coefW) {
    const uint32_t* sm = sums + (uint64_t)b * kBatchSumWords + slot * kSumWords;
    const G1 a = load_jac(sm), bj = load_jac(sm + kJacWords);
    const bool w_inf = ct_u[32ull * d.ct + 25] != 0;
    return pairing_value2_jac(coefH + (uint64_t)d.ct * kLineWordsPerPoint, a, coefW + (uint64_t)d.ct * kLineWordsPerPoint,
                              {bj.x, fp_neg(bj.y), bj.z}, !w_inf);
}

// One tree node's verdict: a pass vouches for its valid leaves; a failing
// single is an invalid share (its ok byte stays 0); a failing larger node is
// pushed as the next round's item (its left child to check, its own value
// stored at this item's side slot for the derivation) — or, past the next
// round's capacity, its valid leaves go to the per-share round.
BD void bin_node_verdict(uint32_t h, bool pass, const Fp12& v, uint32_t b, const BatchDesc& d, const uint8_t* lok,
                         const uint32_t* __restrict__ perm, uint8_t* __restrict__ ok, uint32_t pos, uint32_t side,
                         uint32_t* __restrict__ gt_out, BinItem* __restrict__ next, uint32_t* __restrict__ next_n,
                         uint32_t next_cap, uint32_t* __restrict__ fail_list, uint32_t* __restrict__ fail_n) {
    const uint32_t l0 = bin_first(h), l1 = l0 + bin_size(h);
    if (pass) {
        for (uint32_t l = l0; l < l1; ++l)
            if (lok[l]) ok[perm[d.start + l]] = 1;
        return;
    }
    if (l1 - l0 == 1) return;
    const uint32_t q = atomicAdd(next_n, 1u);
    if (q < next_cap) {
        store_gt(gt_out + (uint64_t)(2 * pos + side) * kGtWords, v);
        next[q] = BinItem{b, 2 * h, pos, side};
    } else {
        for (uint32_t l = l0; l < l1; ++l)
            if (lok[l]) fail_list[atomicAdd(fail_n, 1u)] = perm[d.start + l];
    }
}

// Round 0, one lane per batch: the batch sum (slot 0).  A failing batch's
// value goes to gt_out[2 b] and its left half to the round-1 list.
TDEC_WAVE1_KERNEL void tdec_bin_root(uint32_t cap, const uint32_t* __restrict__ nb_dev,
                                     const BatchDesc* __restrict__ desc, const uint32_t* __restrict__ perm,
                                     const uint32_t* __restrict__ sums, const uint8_t* __restrict__ leaf_ok,
                                     const int32_t* __restrict__ ct_status,
                                     const uint32_t* __restrict__ ct_u, const uint32_t* __restrict__ coefH,
                                     const uint32_t* __restrict__ coefW, uint8_t* __restrict__ ok,
                                     uint32_t* __restrict__ gt_out, BinItem* __restrict__ next,
                                     uint32_t* __restrict__ next_n, uint32_t next_cap,
                                     uint32_t* __restrict__ fail_list, uint32_t* __restrict__ fail_n) {
    const uint64_t i = grid_lane();
    if (i >= dev_count(nb_dev, cap)) return;
    const uint32_t b = (uint32_t)i;
    const BatchDesc d = desc[b];
#ifdef HBG_DEBUG_CHECKS
    if (!HBG_DBG_RANGE(d.end, g_dbg[0] + 1, "root d.end") || !HBG_DBG_RANGE(d.ct, g_dbg[2], "root d.ct")) return;
#endif
    // the leaves saw U's status only: a ciphertext whose W failed to decode has
    // no lines and every share of it stays 0
    if (ct_status[d.ct] != 0) return;
    const uint8_t* lok = leaf_ok + (uint64_t)b * kBatchShares;
    if (!node_any_valid(lok, 0, kBatchShares)) return;  // nothing valid to vouch for: those shares stay 0
    const Fp12 v = bin_node_value(sums, b, 0, d, ct_u, coefH, coefW);
    bin_node_verdict(1, fp12_is_one(v), v, b, d, lok, perm, ok, b, 0, gt_out, next, next_n, next_cap, fail_list,
                     fail_n);
}

// Rounds 1..6, one lane per item (a failing parent): check its left child,
// derive the right one (parent * conj(left): the GT values multiply over the
// disjoint halves; a side without valid leaves is the identity, so the other
// side equals the parent and needs no check either), verdict for both.
TDEC_WAVE1_KERNEL void tdec_bin_step(uint32_t cap, const uint32_t* __restrict__ n_dev,
                                     const BinItem* __restrict__ items, const BatchDesc* __restrict__ desc,
                                     const uint32_t* __restrict__ perm, const uint32_t* __restrict__ sums,
                                     const uint8_t* __restrict__ leaf_ok, const uint32_t* __restrict__ ct_u,
                                     const uint32_t* __restrict__ coefH, const uint32_t* __restrict__ coefW,
                                     uint8_t* __restrict__ ok, const uint32_t* __restrict__ gt_in,
                                     uint32_t* __restrict__ gt_out, BinItem* __restrict__ next,
                                     uint32_t* __restrict__ next_n, uint32_t next_cap,
                                     uint32_t* __restrict__ fail_list, uint32_t* __restrict__ fail_n) {
    const uint64_t i = grid_lane();
    if (i >= dev_count(n_dev, cap)) return;
    const BinItem it = items[i];
#ifdef HBG_DEBUG_CHECKS
    if (!HBG_DBG_RANGE(it.b, g_dbg[1], "step it.b") || !HBG_DBG_RANGE(it.h, 128, "step h")) return;
#endif
    const BatchDesc d = desc[it.b];
    const uint8_t* lok = leaf_ok + (uint64_t)it.b * kBatchShares;
    const uint32_t hl = it.h, s = bin_size(hl), l0 = bin_first(hl);
    const bool lany = node_any_valid(lok, l0, l0 + s), rany = node_any_valid(lok, l0 + s, l0 + 2 * s);
    Fp12 lv = fp12_one();
    bool lpass = true;
    if (lany && rany) {
        lv = bin_node_value(sums, it.b, hl / 2, d, ct_u, coefH, coefW);
        lpass = fp12_is_one(lv);
    }
    const Fp12 pv = load_gt(gt_in + (uint64_t)(2 * it.ppos + it.pside) * kGtWords);  // != 1: the parent failed
    Fp12 rv = pv;
    bool rpass = !rany;
    if (lany && !rany) {
        lv = pv;
        lpass = false;
    } else if (lany && !lpass) {
        const Fp12 cl = fp12_conj(lv);
        fp12_mul_n(&rv, &pv, &cl);
        rpass = fp12_is_one(rv);
    }
    if (lany)
        bin_node_verdict(hl, lpass, lv, it.b, d, lok, perm, ok, (uint32_t)i, 0, gt_out, next, next_n, next_cap,
                         fail_list, fail_n);
    if (rany)
        bin_node_verdict(hl + 1, rpass, rv, it.b, d, lok, perm, ok, (uint32_t)i, 1, gt_out, next, next_n, next_cap,
                         fail_list, fail_n);
}

TDEC_WAVE1_KERNEL void tdec_ct_verify(uint32_t n, const uint32_t* __restrict__ ct_u,
                                                     const int32_t* __restrict__ ct_status,
                                                     const uint32_t* __restrict__ coefH,
                                                     const uint32_t* __restrict__ coefW, uint8_t* __restrict__ ok) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    bool good = ct_status[k] == 0;
    if (good) {
        const uint32_t* cu = ct_u + 32ull * k;
        const bool u_inf = cu[24] != 0, w_inf = cu[25] != 0;
        const Fp ux = load_fp(cu), nuy = fp_neg(load_fp(cu + 12));
        // e(G1, W) * e(-U, H) == 1
        good = pairing_check2(coefW + (uint64_t)k * 72 * kMillerSteps, fp_const(kG1x), fp_const(kG1y), !w_inf,
                              coefH + (uint64_t)k * 72 * kMillerSteps, ux, nuy, !u_inf);
    }
    ok[k] = good ? 1 : 0;
}

// ---------------------------------------------------------------- ThresholdDecrypt glue (a18)
// hbbft ThresholdDecrypt [EXT, src/threshold_decrypt.rs, recalled from
// upstream] for one ciphertext of the epoch, given every sender's share
// verdict (PublicKeyShare::verify_decryption_share, computed for all shares
// by the batched verifier).  The arrival list (arrival_len entries, ended by
// the first entry >= N other than HBG_ARRIVAL_CIPHERTEXT) is replayed:
//  * before the ciphertext marker (HoneyBadger has not output the proposal
//    yet): handle_message holds the share unverified; a sender already held
//    is replaced (same bytes) and faulted (MultipleDecryptionShares:
//    HBG_SHARE_REPEAT flag);
//  * at the marker (no marker: before the first arrival): set_ciphertext —
//    an invalid ciphertext (Ciphertext::verify false) ends the instance;
//    start_decryption drops the held shares that fail verification
//    (UnverifiedDecryptionShareSender: HBG_SHARE_FAULTY), keeps the rest
//    (HBG_SHARE_ACCEPTED), at a validator's marker (HBG_ARRIVAL_OWN | i)
//    inserts node i's own share (trusted, never verified) and try_output
//    fires if more than t are held;
//  * after it, until terminated: an invalid share is a fault, a valid one is
//    held, a valid one from a held sender is a repeat fault; try_output fires
//    at t+1 held;
//  * try_output terminates and decrypts with the first t+1 held shares in
//    node-id order (the sender BTreeMap); later arrivals are ignored
//    (HBG_SHARE_IGNORED, never checked).
// One thread per ciphertext (the outcome bytes double as its per-sender
// state; kPending marks a share held before the ciphertext).  Outputs: the
// t+1 selected (index, share) pairs sorted by node index for hbg_tdec_combine's
// kernel, a per-(ct, sender) outcome byte and the selection status.
__global__ __launch_bounds__(256) void tdec_select(uint32_t n_ct, uint32_t N, uint32_t t,
                                                   const uint8_t* __restrict__ ct_ok, const uint8_t* __restrict__ ok,
                                                   const uint32_t* __restrict__ arrival, uint32_t arrival_len,
                                                   const uint8_t* __restrict__ share48, uint32_t* __restrict__ sel_idx,
                                                   uint8_t* __restrict__ sel48, uint8_t* __restrict__ outcome,
                                                   int32_t* __restrict__ sel_status) {
    constexpr uint8_t kPending = 0x80, kBase = 3;
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_ct) return;
    const uint32_t m = t + 1;
    uint8_t* oc = outcome + k * N;
    uint32_t* idx = sel_idx + k * m;
    const uint32_t* arr = arrival ? arrival + k * (uint64_t)arrival_len : nullptr;
    const uint32_t len = arrival ? arrival_len : N;
    for (uint32_t i = 0; i < N; ++i) oc[i] = HBG_SHARE_NONE;
    // the list's end and whether it carries the ciphertext marker
    uint32_t end = len;
    bool marker = false;
    auto is_marker = [&](uint32_t s) {
        return s == HBG_ARRIVAL_CIPHERTEXT || ((s & HBG_ARRIVAL_OWN) && (s & ~HBG_ARRIVAL_OWN) < N);
    };
    for (uint32_t j = 0; j < len; ++j) {
        const uint32_t s = arr ? arr[j] : j;
        if (is_marker(s)) {
            marker = true;
        } else if (s >= N) {
            end = j;
            break;
        }
    }
    uint32_t held = 0;
    bool ct_set = !marker, term = false;
    int32_t st = HBG_E_NOT_ENOUGH_SHARES;
    const bool good_ct = ct_ok[k] != 0;
    if (ct_set && !good_ct) st = HBG_E_INVALID_CIPHERTEXT;
    for (uint32_t j = 0; j < end && st != HBG_E_INVALID_CIPHERTEXT; ++j) {
        const uint32_t s = arr ? arr[j] : j;
        if (is_marker(s)) {
            if (ct_set) continue;
            ct_set = true;
            if (!good_ct) {
                st = HBG_E_INVALID_CIPHERTEXT;
                break;
            }
            // start_decryption, node-id order: drop the invalid held shares, then (a
            // validator, HBG_ARRIVAL_OWN | i) insert its own share — trusted, never
            // verified — so the first t+1 held by node id are the selection
            const uint32_t own = s == HBG_ARRIVAL_CIPHERTEXT ? N : (s & ~HBG_ARRIVAL_OWN);
            for (uint32_t i = 0; i < N; ++i) {
                bool add = false;
                if (oc[i] & kPending) {
                    add = ok[k * N + i] != 0;
                    oc[i] = (uint8_t)((oc[i] & HBG_SHARE_REPEAT) | (add ? HBG_SHARE_ACCEPTED : HBG_SHARE_FAULTY));
                }
                if (i == own) {
                    add = true;
                    oc[i] = (uint8_t)((oc[i] & HBG_SHARE_REPEAT) | HBG_SHARE_ACCEPTED);
                }
                if (add) {
                    if (held < m) idx[held] = i;
                    ++held;
                }
            }
            term = held >= m;
            continue;
        }
        if (!ct_set) {
            if (oc[s] & kPending) oc[s] |= HBG_SHARE_REPEAT;
            oc[s] |= kPending;
            continue;
        }
        const uint32_t base = oc[s] & kBase;
        if (term) {
            if (base == HBG_SHARE_NONE) oc[s] |= HBG_SHARE_IGNORED;
            continue;
        }
        if (!ok[k * N + s]) {
            oc[s] = (uint8_t)((oc[s] & HBG_SHARE_REPEAT) | HBG_SHARE_FAULTY);
        } else if (base == HBG_SHARE_ACCEPTED) {
            oc[s] |= HBG_SHARE_REPEAT;
        } else {
            oc[s] = (uint8_t)((oc[s] & HBG_SHARE_REPEAT) | HBG_SHARE_ACCEPTED);
            idx[held++] = s;
            term = held == m;
        }
    }
    for (uint32_t i = 0; i < N; ++i) oc[i] &= (uint8_t)~kPending;  // left by an invalid ciphertext
    if (term && st != HBG_E_INVALID_CIPHERTEXT) st = 0;
    uint32_t* dst = reinterpret_cast<uint32_t*>(sel48 + k * m * 48ull);
    if (st != 0) {  // no output: a deterministic (invalid) selection
        for (uint32_t q = 0; q < m; ++q) idx[q] = q;
        for (uint32_t w = 0; w < 12 * m; ++w) dst[w] = 0;
    } else {
        for (uint32_t a = 1; a < m; ++a) {  // node-id order (the BTreeMap the crate iterates)
            const uint32_t v = idx[a];
            uint32_t b = a;
            for (; b > 0 && idx[b - 1] > v; --b) idx[b] = idx[b - 1];
            idx[b] = v;
        }
        for (uint32_t q = 0; q < m; ++q) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(share48 + (k * N + idx[q]) * 48ull);
            for (int w = 0; w < 12; ++w) dst[12 * q + w] = src[w];
        }
    }
    sel_status[k] = st;
}

// per-(ct, sender) verify work items of the epoch: share (k, i) -> ct k, key i
__global__ __launch_bounds__(256) void tdec_pair_index(uint64_t n, uint32_t N, uint32_t* __restrict__ sct,
                                                       uint32_t* __restrict__ spk) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    sct[q] = (uint32_t)(q / N);
    spk[q] = (uint32_t)(q % N);
}

// status = selection status where it is not 0 (no output), else combine's
__global__ __launch_bounds__(256) void tdec_status_merge(uint32_t n, const int32_t* __restrict__ sel_status,
                                                         int32_t* __restrict__ status) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n && sel_status[k] != 0) status[k] = sel_status[k];
}

// ---------------------------------------------------------------- Fr (scalar field) for Lagrange
// r < 2^255, 8 x u32 limbs, Montgomery with R = 2^256 (plain C: low volume).
struct Fr {
    uint32_t v[8];
};
constexpr uint32_t kR_N0 = 0xFFFFFFFFu;  // -r^-1 mod 2^32 (r = 1 mod 2^32)

BD Fr fr_mul(const Fr& a, const Fr& b) {
    uint32_t t[10] = {0};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            c += (uint64_t)a.v[j] * b.v[i] + t[j];
            t[j] = (uint32_t)c;
            c >>= 32;
        }
        c += t[8];
        t[8] = (uint32_t)c;
        t[9] = (uint32_t)(c >> 32);
        const uint32_t m = t[0] * kR_N0;
        c = (uint64_t)m * kR[0] + t[0];
        c >>= 32;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            c += (uint64_t)m * kR[j] + t[j];
            t[j - 1] = (uint32_t)c;
            c >>= 32;
        }
        c += t[8];
        t[7] = (uint32_t)c;
        t[8] = t[9] + (uint32_t)(c >> 32);
    }
    Fr r, u;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) u.v[i] = __builtin_subc(t[i], kR[i], br, &br);
    const bool ge = t[8] || !br;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = ge ? u.v[i] : t[i];
    return r;
}

BD Fr fr_from_u32(uint32_t x) {  // Montgomery form of a small integer: x * R mod r = mul(x, R^2)
    Fr a = {{x, 0, 0, 0, 0, 0, 0, 0}};
    Fr r2;
#pragma unroll
    for (int i = 0; i < 8; ++i) r2.v[i] = kFrR2[i];
    return fr_mul(a, r2);
}

BD Fr fr_sub(const Fr& a, const Fr& b) {
    Fr r, u;
    uint32_t br = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
#pragma unroll
    for (int i = 0; i < 8; ++i) u.v[i] = __builtin_addc(r.v[i], kR[i], c, &c);
    return br ? u : r;
}

BD Fr fr_inv(const Fr& a) {  // a^(r-2)
    Fr r = a;
    for (int i = 253; i >= 0; --i) {
        r = fr_mul(r, r);
        if ((kRm2[i >> 5] >> (i & 31)) & 1u) r = fr_mul(r, a);
    }
    return r;
}

BD bool fr_is_zero(const Fr& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.v[i];
    return o == 0;
}

BD Fr fr_canonical(const Fr& a) {
    Fr one = {{1, 0, 0, 0, 0, 0, 0, 0}};
    return fr_mul(a, one);
}

// PublicKeySet::decrypt for one ciphertext per work-item.
// shares: [n][t+1][48] compressed (already verified: no subgroup re-check, as
// in the crate where decrypt consumes parsed shares); idx: [n][t+1] node indices.
TDEC_KERNEL void tdec_combine(uint32_t n, uint32_t t, const uint8_t* __restrict__ share48,
                                                   const uint32_t* __restrict__ idx, uint8_t* __restrict__ seeds,
                                                   int32_t* __restrict__ status, uint32_t* __restrict__ scratch) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t m = t + 1;
    const uint32_t* ix = idx + (uint64_t)k * m;
    // per-lane scratch: lambda[m][8] then points[m][24]
    uint32_t* lam = scratch + (uint64_t)k * m * 32;
    uint32_t* pts = lam + m * 8;
    int32_t st = 0;
    // duplicate indices -> DuplicateEntry (non-invertible denominator)
    for (uint32_t i = 0; i < m && st == 0; ++i)
        for (uint32_t j = i + 1; j < m; ++j)
            if (ix[i] == ix[j]) st = HBG_E_DUPLICATE_ENTRY;
    // decompress
    for (uint32_t i = 0; i < m && st == 0; ++i) {
        G1A p;
        if (!g1_decompress(share48 + ((uint64_t)k * m + i) * 48, p, false)) {
            st = HBG_E_INVALID_POINT;
            break;
        }
        store_fp(pts + 24 * i, p.x);
        store_fp(pts + 24 * i + 12, p.y);
        // an identity share contributes nothing; mark it with a top y limb no
        // field element can have (p's top limb is 0x1a0111ea)
        if (p.inf) pts[24 * i + 23] = 0xFFFFFFFFu;
    }
    status[k] = st;
    if (st != 0) return;
    // lambda_i = prod_{j != i} x_j / prod_{j != i} (x_j - x_i),  x = index + 1  (mod r)
    for (uint32_t i = 0; i < m; ++i) {
        Fr num = fr_from_u32(1), den = fr_from_u32(1);
        const Fr xi = fr_from_u32(ix[i] + 1);
        for (uint32_t j = 0; j < m; ++j) {
            if (j == i) continue;
            const Fr xj = fr_from_u32(ix[j] + 1);
            num = fr_mul(num, xj);
            den = fr_mul(den, fr_sub(xj, xi));
        }
        const Fr l = fr_canonical(fr_mul(num, fr_inv(den)));
#pragma unroll
        for (int w = 0; w < 8; ++w) lam[8 * i + w] = l.v[w];
    }
    // sum lambda_i * S_i  (Straus, 1-bit window, shared doublings)
    G1 acc = {fp_one(), fp_one(), fp_zero()};
    for (int bit = 254; bit >= 0; --bit) {
        acc = g1_dbl(acc);
        for (uint32_t i = 0; i < m; ++i) {
            if (pts[24 * i + 23] == 0xFFFFFFFFu) continue;
            if ((lam[8 * i + (bit >> 5)] >> (bit & 31)) & 1u)
                acc = g1_add_mixed(acc, load_fp(pts + 24 * i), load_fp(pts + 24 * i + 12));
        }
    }
    const G1A g = g1_to_affine(acc);
    uint8_t cg[48];
    g1_compress(cg, g);
    sha3_bytes(cg, 48, seeds + 32ull * k);  // xor_with_hash's key: the keystream runs in tdec_keystream_xor
}

// GLV split on G1 (Gallant–Lambert–Vanstone): phi(x, y) = (beta x, y) acts as
// [-x^2] on G1 (the subgroup check above), so for l = q x^2 + rem
// [l]P = [rem]P + [q]([x^2]P) with [x^2]P = (beta px, -py); rem < x^2 < 2^128
// and q < 2^129 for any 256-bit l.  x^2 = 0xac45a4010001a402_00000001_00000000.
inline constexpr uint32_t kX2[4] = {0x00000000u, 0x00000001u, 0x0001a402u, 0xac45a401u};

BD void split_x2(const uint32_t (&l)[8], uint32_t (&q)[5], uint32_t (&rm)[5]) {
#pragma unroll
    for (int w = 0; w < 5; ++w) q[w] = rm[w] = 0u;
#pragma unroll
    for (int w = 7; w >= 0; --w) {  // schoolbook binary long division, static word indices
        const uint32_t lw = l[w];
        uint32_t qw = 0;
#pragma unroll 1
        for (int b = 31; b >= 0; --b) {
#pragma unroll
            for (int i = 4; i > 0; --i) rm[i] = (rm[i] << 1) | (rm[i - 1] >> 31);
            rm[0] = (rm[0] << 1) | ((lw >> b) & 1u);
            bool ge = rm[4] != 0, decided = ge;
#pragma unroll
            for (int i = 3; i >= 0; --i)
                if (!decided && rm[i] != kX2[i]) {
                    ge = rm[i] > kX2[i];
                    decided = true;
                }
            if (!decided) ge = true;  // equal
            if (ge) {
                uint32_t borrow = 0;
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const uint64_t d = (uint64_t)rm[i] - (i < 4 ? kX2[i] : 0u) - borrow;
                    rm[i] = (uint32_t)d;
                    borrow = (uint32_t)(d >> 63);
                }
                qw |= 1u << b;
            }
        }
        if (w < 5) q[w] = qw;  // q < 2^129: words 5..7 of the quotient are zero
    }
}

// [l]P for a 256-bit scalar (8 LE words, any value: [l]P = [l mod r]P), P
// affine and in G1: joint double-and-add (Straus–Shamir) over the 129-bit GLV
// halves with the three points P, [x^2]P and their sum.  Branch-free per step
// (one Jacobian add whose operand is selected per lane) so lanes with
// different scalars stay converged: 129 doublings + 129 adds instead of 256
// doublings + 256 (divergent) mixed adds.
BD G1 g1_mul_fr(const Fp& px, const Fp& py, const uint32_t (&l)[8]) {
    uint32_t q[5], rm[5];
    split_x2(l, q, rm);
    // P + [x^2]P (never infinity) and the addends on its isomorphic curve E_Z
    // (g1_mul_ab64): mixed additions only, the result mapped back by Z
    const G1 both = g1_add_mixed({px, py, fp_one()}, fp_mul(px, fp_const(kBeta)), fp_neg(py));
    Fp z2 = fp_sqr(both.z), z3, tx, ty;
    z3 = fp_mul(z2, both.z);
    fp_mul2(tx, ty, px, z2, py, z3);
    const Fp ux = fp_mul(tx, fp_const(kBeta)), uy = fp_neg(ty);
    G1 r = {fp_one(), fp_one(), fp_zero()};  // doubling / adding to infinity stays exact
#pragma unroll
    for (int w = 4; w >= 0; --w) {
        const uint32_t qw = q[w], rw = rm[w];
#pragma unroll 1
        for (int bit = (w == 4 ? 0 : 31); bit >= 0; --bit) {
            r = g1_dbl(r);
            const bool a = (rw >> bit) & 1u, b = (qw >> bit) & 1u;
            const G1 sum = g1_add_mixed(r, a ? (b ? both.x : tx) : ux, a ? (b ? both.y : ty) : uy);
            if (a || b) r = sum;
        }
    }
    return {r.x, r.y, fp_mul(r.z, both.z)};
}

// PublicKeySet::decrypt as a bucket multi-scalar multiplication per G-lane
// group (G = 16: four ciphertexts per wave, t + 1 <= 24, lane i owning shares
// i and i + 16; G = 32: two, t + 1 <= 32 or, two shares a lane, <= 64); same
// sum, same error precedence (DuplicateEntry before an undecodable share) as
// the one-lane-per-ciphertext tdec_combine (kept for t + 1 > 64):
//  1. per owned share: DuplicateEntry / decode checks (or, inside
//     ThresholdDecrypt, the verification's decoded point: share_aff),
//     lambda_i and its GLV halves (lambda_i = q x^2 + rm: [lambda_i]S_i =
//     [rm]S_i + [q]([x^2]S_i), both < 2^129) — S_i (x, y, beta x) and the two
//     scalars go to LDS;
//  2. every lane owns kPer = 64 / G 2-bit windows of the 129-bit scalars (the
//     last lane also window 64, whose digits are single bits): per window
//     three buckets take one mixed addition per point whose digit is nonzero,
//     W = b1 + 2 b2 + 3 b3, and the lane folds its windows by Horner;
//  3. a log2(G)-level butterfly joins neighbouring lane ranges (the upper range
//     shifted by its first window: 2 kPer (G - 1) doublings on the critical path).
// Fewer lanes per ciphertext cost more windows per lane but fewer butterfly
// doublings per ciphertext: G = 16 issues ~30 % less per ciphertext than
// G = 32 at t = 21 (round 4; round 3's G = 32 replaced a per-lane joint
// double-and-add: 317 -> 231 ms per 100 k ciphertexts, profiles/r03z).
template <int G, int MMAX>
TDEC_KERNEL void tdec_combine_msm(uint32_t n, uint32_t t, const uint8_t* __restrict__ share48,
                                  const uint32_t* __restrict__ idx, uint32_t* __restrict__ sums,
                                  int32_t* __restrict__ status, const uint32_t* __restrict__ share_aff,
                                  uint32_t n_nodes, const int32_t* __restrict__ pre_status,
                                  const uint8_t* __restrict__ share_ok) {
    static_assert(G == 16 || G == 32 || G == 64, "a quarter, half or whole wave per ciphertext");
    static_assert(MMAX <= 2 * G, "at most two shares per lane");
    constexpr uint32_t GPB = 64 / G;                 // groups per 64-lane block
    constexpr uint32_t kPer = 64 / G;                // 2-bit windows per lane (the last lane: one more)
    constexpr uint32_t SPL = (MMAX + G - 1) / G;     // shares per lane
    // beta x kept in LDS, except where it would cost occupancy (more than
    // 20 KB a block leaves fewer than 8 blocks a CU — <32, 64>: 23 KB; beta x
    // is then recomputed per use)
    constexpr bool kBetaLds = GPB * MMAX * (36 * 4 + 2 * 5 * 4) <= 20480;
    constexpr uint32_t kPtWords = kBetaLds ? 36 : 24;
    __shared__ uint32_t sPt[GPB][MMAX][kPtWords];    // S_i: x, y, beta x ([x^2]S_i = (beta x, -y))
    __shared__ uint32_t sSc[GPB][2 * MMAX][5];       // point 2i: rm_i (S_i); 2i + 1: q_i ([x^2]S_i)
    const uint32_t gl = threadIdx.x / G, i = threadIdx.x % G, gshift = gl * G;
    const uint32_t g = blockIdx.x * GPB + gl;
    const uint32_t m = t + 1;
    const bool live = g < n;  // no early return: the barrier and the group shuffles need every lane
    const uint32_t* ix = idx + (uint64_t)(live ? g : 0) * m;
    // a failed selection (share_aff path): nothing to combine, the status is the selection's
    const int32_t pre = (share_aff && pre_status && live) ? pre_status[g] : 0;
    G1A p[SPL];
    uint32_t me[SPL];
    bool dup = false, bad = false;
#pragma unroll
    for (uint32_t r = 0; r < SPL; ++r) {
        const uint32_t sI = i + G * r;
        const bool act = live && sI < m;
        me[r] = act ? ix[sI] : 0u;
        p[r] = {fp_zero(), fp_zero(), true};
        if (act)
            for (uint32_t j = sI + 1; j < m; ++j) dup |= ix[j] == me[r];
        if (act && pre == 0) {
            const uint64_t slot = (uint64_t)g * n_nodes + (me[r] < n_nodes ? me[r] : 0u);
            // the verification's decoded point for a selected share that verified;
            // a selected share that did not (a validator's own share: trusted, never
            // verified — it may not even decode) is decompressed here
            if (share_aff && (!share_ok || share_ok[slot])) {
                const uint32_t* a = share_aff + slot * kAffWords;
                p[r].x = load_fp(a);
                p[r].y = load_fp(a + 12);
                p[r].inf = a[24] != 0;
            } else {
                bad |= !g1_decompress(share48 + ((uint64_t)g * m + sI) * 48, p[r], false);
            }
        }
    }
    const uint64_t gmask = G == 64 ? ~0ull : ((1ull << G) - 1ull);
    const bool any_dup = (__ballot(dup) >> gshift) & gmask;
    const bool any_bad = (__ballot(bad) >> gshift) & gmask;
    const int32_t st = pre != 0 ? pre : (any_dup ? HBG_E_DUPLICATE_ENTRY : (any_bad ? HBG_E_INVALID_POINT : 0));
#pragma unroll
    for (uint32_t r = 0; r < SPL; ++r) {
        const uint32_t sI = i + G * r;
        const bool act = live && sI < m;
        uint32_t q[5] = {0, 0, 0, 0, 0}, rm[5] = {0, 0, 0, 0, 0};
        if (act && st == 0 && !p[r].inf) {
            // lambda_i = prod_{j != i} x_j / prod_{j != i} (x_j - x_i),  x = index + 1  (mod r)
            Fr num = fr_from_u32(1), den = fr_from_u32(1);
            const Fr xi = fr_from_u32(me[r] + 1);
            for (uint32_t j = 0; j < m; ++j) {
                if (j == sI) continue;
                const Fr xj = fr_from_u32(ix[j] + 1);
                num = fr_mul(num, xj);
                den = fr_mul(den, fr_sub(xj, xi));
            }
            const Fr l = fr_canonical(fr_mul(num, fr_inv(den)));
            uint32_t lw[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) lw[w] = l.v[w];
            split_x2(lw, q, rm);
        }
        // shares past t + 1 keep zero scalars (no contribution)
        if (sI < MMAX) {
            uint32_t* a = sPt[gl][sI];
            store_fp(a, p[r].x);
            store_fp(a + 12, p[r].y);
            if (kBetaLds) store_fp(a + 24, fp_mul(p[r].x, fp_const(kBeta)));
#pragma unroll
            for (int w = 0; w < 5; ++w) {
                sSc[gl][2 * sI][w] = rm[w];
                sSc[gl][2 * sI + 1][w] = q[w];
            }
        }
    }
    __syncthreads();
    // this lane's windows [w0, w1], folded from the top one down
    const uint32_t w0 = i * kPer, w1 = i * kPer + kPer - 1 + (i == G - 1 ? 1u : 0u);
    const uint32_t np = 2 * m;
    G1 L = {fp_one(), fp_one(), fp_zero()};
#pragma unroll 1
    for (int w = (int)w1; w >= (int)w0; --w) {
        G1 b1 = {fp_one(), fp_one(), fp_zero()}, b2 = b1, b3 = b1;
        const uint32_t word = (uint32_t)w >> 4, sh = (2u * (uint32_t)w) & 31u;
#pragma unroll 1
        for (uint32_t j = 0; j < np; ++j) {
            const uint32_t d = (sSc[gl][j][word] >> sh) & 3u;
            if (!__any(d != 0)) continue;  // wave-uniform skip (no lane has this digit)
            const uint32_t* pt = sPt[gl][j >> 1];
            Fp px;
            if (kBetaLds) px = load_fp(pt + ((j & 1u) ? 24 : 0));
            else px = (j & 1u) ? fp_mul(load_fp(pt), fp_const(kBeta)) : load_fp(pt);
            Fp py = load_fp(pt + 12);
            if (j & 1u) py = fp_neg(py);
            const G1 sel = d == 1u ? b1 : (d == 2u ? b2 : b3);
            const G1 sum = g1_add_mixed(sel, px, py);
            if (d == 1u) b1 = sum;
            if (d == 2u) b2 = sum;
            if (d == 3u) b3 = sum;
        }
        // W = b1 + 2 b2 + 3 b3 = b3 + (b3 + b2) + (b3 + b2 + b1)
        G1 run = b3, win = b3;
        run = g1_add(run, b2);
        win = g1_add(win, run);
        run = g1_add(run, b1);
        win = g1_add(win, run);
        L = g1_add(g1_dbl(g1_dbl(L)), win);
    }
    // butterfly: the lower range absorbs the upper one shifted by 2 kPer 2^k bits
#pragma unroll 1
    for (uint32_t k = 0; (1u << k) < (uint32_t)G; ++k) {
        const G1 other = g1_shfl_xor(L, 1 << k);
        const bool lower = (i & (1u << k)) == 0;
        G1 x = lower ? other : L;
        const uint32_t dbls = 2u * kPer * (1u << k);
#pragma unroll 1
        for (uint32_t d = 0; d < dbls; ++d) x = g1_dbl(x);
        if (lower) L = g1_add(L, x);
    }
    if (!live || i != 0) return;
    status[g] = st;
    if (st == 0) store_jac(sums + 36ull * g, L);  // affine + compress + SHA3: tdec_combine_seed
}

// The combination's epilogue, one lane per ciphertext: the Jacobian sum to
// affine (one field inversion), compressed, SHA3 -> xor_with_hash's key (the
// keystream runs in tdec_keystream_xor).  In the MSM kernel only each group's
// first lane did this, 4 of 64 lanes busy through the inversion.
TDEC_KERNEL void tdec_combine_seed(uint32_t n, const uint32_t* __restrict__ sums,
                                   const int32_t* __restrict__ status, uint8_t* __restrict__ seeds) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n || status[k] != 0) return;
    const G1A sum = g1_to_affine(load_jac(sums + 36ull * k));
    uint8_t cg[48];
    g1_compress(cg, sum);
    sha3_bytes(cg, 48, seeds + 32ull * k);
}

// ------------------------------------------------------------------ SURVEY.md §8(f1)/(f2)
// Wire-message signatures (threshold_crypto SecretKey::sign / PublicKey::verify,
// reached from hydrabadger lib.rs:405-416 / :434) and the proposer / node side
// of ThresholdDecrypt (PublicKey::encrypt_with_rng with r explicit,
// SecretKeyShare::decrypt_share_no_verify).  One work-item per message.

BD void g2_compress(uint8_t* b, const G2A& p) {
    if (p.inf) {
        b[0] = 0xC0;
        for (int i = 1; i < 96; ++i) b[i] = 0;
        return;
    }
    fp_to_be(b, fp_from_mont(p.x.c1));
    fp_to_be(b + 48, fp_from_mont(p.x.c0));
    b[0] |= 0x80;
    if (fp2_gt(p.y, fp2_neg(p.y))) b[0] |= 0x20;
}

// 32-byte little-endian scalar (an Fr value; [k]P == [k mod r]P for P of order r)
BD void load_scalar(const uint8_t* p, uint32_t (&k)[8]) {
#pragma unroll
    for (int w = 0; w < 8; ++w)
        k[w] = (uint32_t)p[4 * w] | (uint32_t)p[4 * w + 1] << 8 | (uint32_t)p[4 * w + 2] << 16 |
               (uint32_t)p[4 * w + 3] << 24;
}

// [k]P for P in G2 (affine) and a 256-bit scalar: psi acts as [x] on G2, so
// psi^2 = [x^2] and the G1 split applies unchanged — k = q x^2 + rem,
// [k]P = [rem]P + [q]psi^2(P) (psi^2 of an affine point is affine) — with the
// same branch-free joint double-and-add: 129 doublings + 129 additions instead
// of 256 + 256 divergent mixed additions.  Callers pass subgroup points only
// (hash_g2 outputs; shares the crate deserialised, i.e. subgroup-checked).
BD G2 g2_mul_scalar(const Fp2& px, const Fp2& py, const uint32_t (&k)[8]) {
    uint32_t q[5], rm[5];
    split_x2(k, q, rm);
    const G2 B = g2_psi(g2_psi({px, py, fp2_one()}));  // [x^2]P, Z = 1
    const G2 both = g2_add_mixed({px, py, fp2_one()}, B.x, B.y);
    // the addends on the isomorphic curve of both's Z (g1_mul_ab64): mixed additions
    const Fp2 z2 = fp2_sqr(both.z), z3 = fp2_mul(z2, both.z);
    const Fp2 tx = fp2_mul(px, z2), ty = fp2_mul(py, z3), ux = fp2_mul(B.x, z2), uy = fp2_mul(B.y, z3);
    G2 r = {fp2_one(), fp2_one(), fp2_zero()};
#pragma unroll
    for (int w = 4; w >= 0; --w) {
        const uint32_t qw = q[w], rw = rm[w];
#pragma unroll 1
        for (int bit = (w == 4 ? 0 : 31); bit >= 0; --bit) {
            r = g2_dbl(r);
            const bool a = (rw >> bit) & 1u, b = (qw >> bit) & 1u;
            const G2 sum = g2_add_mixed(r, a ? (b ? both.x : tx) : ux, a ? (b ? both.y : ty) : uy);
            if (a || b) r = sum;
        }
    }
    return {r.x, r.y, fp2_mul(r.z, both.z)};
}

// hash_g2(msg): ChaChaRng seeded with SHA3-256(msg)
BD G2A hash_g2_msg(const uint8_t* msg, uint32_t len) {
    uint8_t seed[32];
    sha3_bytes(msg, len, seed);
    return hash_g2_from_seed(seed);
}

// SecretKey::sign(msg) = hash_g2(msg) * sk
TDEC_WAVE1_KERNEL void bls_sign(uint64_t n, uint32_t n_sk, const uint8_t* __restrict__ sk32,
                          const uint32_t* __restrict__ msg_sk, const uint8_t* __restrict__ msg,
                          const uint64_t* __restrict__ off, uint8_t* __restrict__ sig96, int32_t* __restrict__ err) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    if (msg_sk[k] >= n_sk) {  // device-mode index check: all-zero bytes (no valid encoding), HBG_E_ARG
        for (int i = 0; i < 96; ++i) sig96[96ull * k + i] = 0;
        flag_error(err, HBG_E_ARG);
        return;
    }
    const G2A h = hash_g2_msg(msg + off[k], (uint32_t)(off[k + 1] - off[k]));
    uint32_t sk[8];
    load_scalar(sk32 + 32ull * msg_sk[k], sk);
    G2A s = {fp2_zero(), fp2_zero(), true};
    if (!h.inf) s = g2_to_affine(g2_mul_scalar(h.x, h.y, sk));
    g2_compress(sig96 + 96ull * k, s);
}

// PublicKey::verify(sig, msg): e(pk, hash_g2(msg)) == e(G1, sig); the signature
// decodes with the crate's subgroup check (SignedWireMessage deserialisation).
TDEC_WAVE1_KERNEL void bls_verify(uint64_t n, uint32_t n_pk, const uint32_t* __restrict__ pk_aff,
                            const int32_t* __restrict__ pk_status, const uint32_t* __restrict__ msg_pk,
                            const uint8_t* __restrict__ msg, const uint64_t* __restrict__ off,
                            const uint8_t* __restrict__ sig96, uint32_t* __restrict__ lines, uint8_t* __restrict__ ok,
                            int32_t* __restrict__ err) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t p = msg_pk[k];
    if (p >= n_pk) {  // device-mode index check
        ok[k] = 0;
        flag_error(err, HBG_E_ARG);
        return;
    }
    G2A sig;
    bool good = pk_status[p] == 0 && g2_decompress(sig96 + 96ull * k, sig, true);
    if (good) {
        const G2A h = hash_g2_msg(msg + off[k], (uint32_t)(off[k + 1] - off[k]));
        uint32_t* lh = lines + k * 2ull * kLineWordsPerPoint;
        uint32_t* ls = lh + kLineWordsPerPoint;
        g2_prepare(h.x, h.y, lh);
        if (!sig.inf) g2_prepare(sig.x, sig.y, ls);
        const uint32_t* pa = pk_aff + 32ull * p;
        good = pairing_check2(lh, load_fp(pa), load_fp(pa + 12), pa[24] == 0, ls, fp_const(kG1x),
                              fp_neg(fp_const(kG1y)), !sig.inf);
    }
    ok[k] = good ? 1 : 0;
}

// WireMessages::poll (src/lib.rs:397-420) for one length-delimited frame:
// LengthDelimitedCodec's BE u32 length == frame body, bincode SignedWireMessage
// { message: Vec<u8> (u64 LE len), sig: Signature (96-B compressed G2 tuple) }
// with the crate's point check, then the WireMessage kind (bincode u32 variant
// of WireMessageKind, src/lib.rs:250-270) and, for Message (7) / KeyGen (9)
// only, PublicKey::verify(sig, message) with the peer's key.
__device__ __forceinline__ uint64_t wire_le(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int b = 0; b < nb; ++b) v |= (uint64_t)p[b] << (8 * b);
    return v;
}

// poll's bincode::deserialize::<WireMessage> for the two verified kinds, as far
// as the reference tree defines their fields (oracle/wire.py body_status):
// Message(Uid, DhbMessage): Uid = u64 length (16) + 16 bytes, then the hbbft
// message's u32 index; KeyGen(InstanceId {BuiltIn, User(Uid)},
// key_gen::Message {kind: Part | Ack}) + the first 4 bytes of Part / Ack.
BD int32_t wire_uid(const uint8_t* m, uint64_t len, uint64_t& p) {
    if (len < p + 8) return HBG_E_WIRE_EOF;
    const uint64_t n = wire_le(m + p, 8);
    p += 8;
    if (n > len - p) return HBG_E_WIRE_EOF;
    if (n != 16) return HBG_E_WIRE_VALUE;
    p += 16;
    return HBG_OK;
}
BD int32_t wire_body_status(const uint8_t* m, uint64_t len) {
    const uint32_t kind = (uint32_t)wire_le(m, 4);
    uint64_t p = 4;
    if (kind == HBG_WIRE_KIND_MESSAGE) {
        const int32_t st = wire_uid(m, len, p);
        if (st) return st;
        return len >= p + 4 ? HBG_OK : HBG_E_WIRE_EOF;
    }
    if (kind == HBG_WIRE_KIND_KEYGEN) {
        if (len < p + 4) return HBG_E_WIRE_EOF;
        const uint32_t inst = (uint32_t)wire_le(m + p, 4);
        p += 4;
        if (inst > 1) return HBG_E_WIRE_TAG;
        if (inst == 1) {
            const int32_t st = wire_uid(m, len, p);
            if (st) return st;
        }
        if (len < p + 4) return HBG_E_WIRE_EOF;
        if ((uint32_t)wire_le(m + p, 4) > 1) return HBG_E_WIRE_TAG;
        return len >= p + 8 ? HBG_OK : HBG_E_WIRE_EOF;
    }
    return HBG_OK;
}

TDEC_WAVE1_KERNEL void wire_verify_frames(uint64_t n, const uint32_t* __restrict__ pk_aff,
                                    const int32_t* __restrict__ pk_status, uint32_t n_pk,
                                    const uint32_t* __restrict__ frame_pk, const uint8_t* __restrict__ frames,
                                    const uint64_t* __restrict__ off, uint32_t* __restrict__ lines,
                                    int32_t* __restrict__ status) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint8_t* f = frames + off[k];
    const uint64_t flen = off[k + 1] - off[k];
    int32_t st = HBG_OK;
    uint64_t mlen = 0;
    G2A sig;
    const uint64_t head = flen < 4 ? 0 : ((uint64_t)f[0] << 24 | (uint64_t)f[1] << 16 | (uint64_t)f[2] << 8 | f[3]);
    if (flen < 4) st = HBG_E_WIRE_EOF;
    else if (head > HBG_WIRE_MAX_FRAME || head != flen - 4) st = HBG_E_WIRE_FRAME;  // codec: too big / bad framing
    else if (flen - 4 < 8) st = HBG_E_WIRE_EOF;
    else {
        mlen = wire_le(f + 4, 8);
        if (mlen > flen - 12 || flen - 12 - mlen < 96) st = HBG_E_WIRE_EOF;
        else if (!g2_decompress(f + 12 + mlen, sig, true)) st = HBG_E_INVALID_POINT;
        else if (mlen < 4) st = HBG_E_WIRE_EOF;
        else {
            const uint32_t kind = (uint32_t)wire_le(f + 12, 4);
            if (kind > HBG_WIRE_KIND_MAX) st = HBG_E_WIRE_TAG;
            else if ((st = wire_body_status(f + 12, mlen)) != HBG_OK) {
                // Error::Serde: the WireMessage does not deserialise (before any verification)
            } else if (kind == HBG_WIRE_KIND_MESSAGE || kind == HBG_WIRE_KIND_KEYGEN) {
                const uint32_t p = frame_pk[k];
                if (p >= n_pk || pk_status[p] != 0) st = HBG_E_UNKNOWN_PEER;
            }
        }
    }
    const bool check = st == HBG_OK && (wire_le(f + 12, 4) == HBG_WIRE_KIND_MESSAGE ||
                                        wire_le(f + 12, 4) == HBG_WIRE_KIND_KEYGEN);
    if (check) {
        const G2A h = hash_g2_msg(f + 12, (uint32_t)mlen);
        uint32_t* lh = lines + k * 2ull * kLineWordsPerPoint;
        uint32_t* ls = lh + kLineWordsPerPoint;
        g2_prepare(h.x, h.y, lh);
        if (!sig.inf) g2_prepare(sig.x, sig.y, ls);
        const uint32_t* pa = pk_aff + 32ull * frame_pk[k];
        if (!pairing_check2(lh, load_fp(pa), load_fp(pa + 12), pa[24] == 0, ls, fp_const(kG1x),
                            fp_neg(fp_const(kG1y)), !sig.inf))
            st = HBG_E_INVALID_SIGNATURE;
    }
    status[k] = st;
}

// PublicKey::encrypt_with_rng with r explicit: U = r G1, V = xor_with_hash(r PK, msg),
// W = r hash_g1_g2(U, V), in three launches: tdec_encrypt_u (U and the
// keystream key SHA3(compress(r PK))), tdec_keystream_xor (V at the message's
// offsets; SHA3(V) by tdec_v_digest when |V| > 64), tdec_encrypt_w (W).
// est[k] != 0 (an undecodable public key): all-zero U and W, V untouched.
TDEC_KERNEL void tdec_encrypt_u(uint64_t n, const uint32_t* __restrict__ pk_aff, const int32_t* __restrict__ pk_status,
                                const uint8_t* __restrict__ r32, uint8_t* __restrict__ U48,
                                uint8_t* __restrict__ W96, uint8_t* __restrict__ seeds, int32_t* __restrict__ est,
                                int32_t* __restrict__ err) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    if (pk_status[0] != 0) {  // the public key does not decode: HBG_E_INVALID_POINT, all-zero U and W
        for (int i = 0; i < 48; ++i) U48[48ull * k + i] = 0;
        for (int i = 0; i < 96; ++i) W96[96ull * k + i] = 0;
        est[k] = HBG_E_INVALID_POINT;
        if (k == 0) flag_error(err, HBG_E_INVALID_POINT);
        return;
    }
    est[k] = 0;
    uint32_t r[8];
    load_scalar(r32 + 32ull * k, r);
    const G1A u = g1_to_affine(g1_mul_fr(fp_const(kG1x), fp_const(kG1y), r));
    g1_compress(U48 + 48ull * k, u);
    G1A g = {fp_zero(), fp_zero(), true};
    if (pk_aff[24] == 0) g = g1_to_affine(g1_mul_fr(load_fp(pk_aff), load_fp(pk_aff + 12), r));
    uint8_t cg[48];
    g1_compress(cg, g);
    sha3_bytes(cg, 48, seeds + 32ull * k);
}

TDEC_WAVE1_KERNEL void tdec_encrypt_w(uint64_t n, const uint8_t* __restrict__ r32, const uint8_t* __restrict__ U48,
                                const uint8_t* __restrict__ V, const uint64_t* __restrict__ off,
                                const uint8_t* __restrict__ vdig, const int32_t* __restrict__ est,
                                uint8_t* __restrict__ W96) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n || est[k] != 0) return;
    uint32_t r[8];
    load_scalar(r32 + 32ull * k, r);
    // H = hash_g1_g2(U, V): m = (|V| > 64 ? sha3(V) : V) || compress(U)
    const uint64_t o = off[k], len = off[k + 1] - o;
    uint8_t m[64 + 48], seed[32];
    const uint32_t ml = hash_g1_g2_msg(V + o, len, vdig + 32ull * k, U48 + 48ull * k, m);
    sha3_bytes(m, ml, seed);
    const G2A h = hash_g2_from_seed(seed);
    G2A w = {fp2_zero(), fp2_zero(), true};
    if (!h.inf) w = g2_to_affine(g2_mul_scalar(h.x, h.y, r));
    g2_compress(W96 + 96ull * k, w);
}

// SecretKeyShare::decrypt_share_no_verify: share = U * sk_i (U already decoded:
// u_aff records from tdec_pk_prepare over the U48 table).
TDEC_KERNEL void tdec_decrypt_share(uint64_t n, uint32_t n_ct, uint32_t n_sk, const uint32_t* __restrict__ u_aff,
                                    const int32_t* __restrict__ u_status, const uint8_t* __restrict__ sk32,
                                    const uint32_t* __restrict__ share_ct, const uint32_t* __restrict__ share_sk,
                                    uint8_t* __restrict__ share48, int32_t* __restrict__ status,
                                    int32_t* __restrict__ err) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t c = share_ct[k];
    if (c >= n_ct || share_sk[k] >= n_sk) {  // device-mode index check: identity encoding, HBG_E_ARG
        g1_compress(share48 + 48ull * k, {fp_zero(), fp_zero(), true});
        status[k] = HBG_E_ARG;
        flag_error(err, HBG_E_ARG);
        return;
    }
    const uint32_t* ua = u_aff + 32ull * c;
    G1A s = {fp_zero(), fp_zero(), true};
    const int32_t st = u_status[c];
    if (st == 0 && ua[24] == 0) {
        uint32_t sk[8];
        load_scalar(sk32 + 32ull * share_sk[k], sk);
        s = g1_to_affine(g1_mul_fr(load_fp(ua), load_fp(ua + 12), sk));
    }
    g1_compress(share48 + 48ull * k, s);
    status[k] = st;
}

// ------------------------------------------------------------------ SURVEY.md §8(f3)
// threshold_sign common coin: PublicKeySet::combine_signatures (interpolation
// at 0 over the first t+1 G2 signature shares) + Signature::parity.  One
// 32-lane group per coin, lane = share (per-lane joint double-and-add over
// the GLV halves, then a G2 butterfly).
BD G2 g2_shfl_xor(const G2& p, int m) {
    G2 r;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        r.x.c0[i] = __shfl_xor(p.x.c0[i], m);
        r.x.c1[i] = __shfl_xor(p.x.c1[i], m);
        r.y.c0[i] = __shfl_xor(p.y.c0[i], m);
        r.y.c1[i] = __shfl_xor(p.y.c1[i], m);
        r.z.c0[i] = __shfl_xor(p.z.c0[i], m);
        r.z.c1[i] = __shfl_xor(p.z.c1[i], m);
    }
    return r;
}

template <int G>
TDEC_WAVE1_KERNEL void coin_combine_grp(uint32_t n, uint32_t t, const uint8_t* __restrict__ share96,
                                  const uint32_t* __restrict__ idx, uint8_t* __restrict__ sig96,
                                  uint8_t* __restrict__ parity, int32_t* __restrict__ status) {
    static_assert(G == 32 || G == 64, "group = half or whole wave");
    const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) / G;
    const uint32_t i = threadIdx.x & (G - 1), half = threadIdx.x & 32u & (uint32_t)(64 - G);
    const uint32_t m = t + 1;
    const bool live = g < n;  // no early return: the group shuffles below need every lane
    const bool act = live && i < m;
    const uint32_t* ix = idx + (uint64_t)(live ? g : 0) * m;
    const uint32_t me = act ? ix[i] : 0u;
    bool dup = false;
    if (act)
        for (uint32_t j = i + 1; j < m; ++j) dup |= ix[j] == me;
    G2A p = {fp2_zero(), fp2_zero(), true};
    bool bad = false;
    if (act) bad = !g2_decompress(share96 + ((uint64_t)g * m + i) * 96, p, false);
    const uint64_t gmask = G == 64 ? ~0ull : 0xFFFFFFFFull;
    const bool any_dup = (__ballot(dup) >> half) & gmask;
    const bool any_bad = (__ballot(bad) >> half) & gmask;
    const int32_t st = any_dup ? HBG_E_DUPLICATE_ENTRY : (any_bad ? HBG_E_INVALID_POINT : 0);
    G2 acc = {fp2_one(), fp2_one(), fp2_zero()};
    if (act && st == 0 && !p.inf) {
        Fr num = fr_from_u32(1), den = fr_from_u32(1);
        const Fr xi = fr_from_u32(me + 1);
        for (uint32_t j = 0; j < m; ++j) {
            if (j == i) continue;
            const Fr xj = fr_from_u32(ix[j] + 1);
            num = fr_mul(num, xj);
            den = fr_mul(den, fr_sub(xj, xi));
        }
        const Fr l = fr_canonical(fr_mul(num, fr_inv(den)));
        uint32_t lw[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) lw[w] = l.v[w];
        acc = g2_mul_scalar(p.x, p.y, lw);
    }
#pragma unroll 1
    for (int s = 1; s < G; s <<= 1) acc = g2_add(acc, g2_shfl_xor(acc, s));
    if (!live || i != 0) return;
    status[g] = st;
    if (st != 0) return;
    const G2A sig = g2_to_affine(acc);
    g2_compress(sig96 + 96ull * g, sig);
    // parity of the ones in the XOR of the 192 uncompressed bytes == parity of
    // all ones of the encoding (flag byte 0x40 for the identity)
    uint32_t x = 0;
    if (sig.inf) {
        x = 0x40u;
    } else {
        const Fp c[4] = {fp_from_mont(sig.x.c0), fp_from_mont(sig.x.c1), fp_from_mont(sig.y.c0),
                         fp_from_mont(sig.y.c1)};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int w = 0; w < 12; ++w) x ^= c[k][w];
    }
    parity[g] = (uint8_t)(__builtin_popcount(x) & 1u);
}

// ---------------------------------------------------------------- batched signature-share verification
// PublicKeyShare::verify(sig_i, doc) (threshold_sign / common coin, SURVEY.md
// §8(f3)) for the shares of ONE document: e(pk_i, H) == e(G1, sig_i) for all
// i  <=  e(sum r_i pk_i, H) == e(G1, sum r_i sig_i), H = hash_g2(doc) hashed
// and prepared ONCE per document (the per-share bls_verify hashes to G2 and
// prepares H once per share).  Same secret 127-bit weights (batch_weight), a
// 4-ary group-testing tree and per-share fallback as the decryption shares
// above, so every 0 bit is the reference's per-share equation and a 1 from a
// passing (sub)batch is wrong with probability <= 2^-127.
constexpr uint32_t kG2JacWords = 72;
constexpr uint32_t kSigSumWords = kJacWords + kG2JacWords;  // (sum r pk: G1, sum r sig: G2)
constexpr uint32_t kSigBatchSumWords = kNodes * kSigSumWords;

BD void store_g2jac(uint32_t* d, const G2& p) {
    store_fp(d, p.x.c0);
    store_fp(d + 12, p.x.c1);
    store_fp(d + 24, p.y.c0);
    store_fp(d + 36, p.y.c1);
    store_fp(d + 48, p.z.c0);
    store_fp(d + 60, p.z.c1);
}
BD G2 load_g2jac(const uint32_t* d) {
    return {{load_fp(d), load_fp(d + 12)}, {load_fp(d + 24), load_fp(d + 36)}, {load_fp(d + 48), load_fp(d + 60)}};
}

// per document: seed = SHA3-256(doc) (the ChaCha seed of hash_g2), G2Prepared lines of H
TDEC_WAVE1_KERNEL void sig_doc_prepare(uint32_t n, const uint8_t* __restrict__ doc, const uint64_t* __restrict__ off,
                                 uint32_t* __restrict__ coefH, uint8_t* __restrict__ seeds) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint8_t seed[32];
    sha3_bytes(doc + off[k], (uint32_t)(off[k + 1] - off[k]), seed);
    for (int i = 0; i < 32; ++i) seeds[32ull * k + i] = seed[i];
    const G2A h = hash_g2_from_seed(seed);
    g2_prepare(h.x, h.y, coefH + (uint64_t)k * kLineWordsPerPoint);
}

// One 64-lane block per batch (shares of one document), lane = share: decode
// the G2 share with the crate's subgroup check, weight r_i from SHA3(K || D || i)
// (batch_weight; D = SHA3 of the leaf digests SHA3(doc seed || share || key index)), then
// [r_i] sig_i (G2) and [r_i] pk_i (G1, fixed-base tables when given) and the
// quad / 16-group / batch sums by cross-lane butterflies.
// [a]P + [b]psi^2(P) = [a + b x^2]P for P in G2 (affine), 64-bit a, b (psi = [x]
// on G2; psi^2 of an affine point is affine) — the G2 half of the coin
// shares' batch weights, same joint double-and-add (and the same mixed
// additions on the isomorphic curve y^2 = x^3 + b' Z^6 of the common
// denominator Z of both = P + psi^2(P)) as g1_mul_ab64.
BD G2 g2_mul_ab64(const Fp2& px, const Fp2& py, uint64_t a, uint64_t b) {
    const G2 B = g2_psi(g2_psi({px, py, fp2_one()}));  // affine: conj(conj(1)) = 1
    const G2 both = g2_add_mixed({px, py, fp2_one()}, B.x, B.y);
    const Fp2 z2 = fp2_sqr(both.z), z3 = fp2_mul(z2, both.z);
    const Fp2 tx = fp2_mul(px, z2), ty = fp2_mul(py, z3), ux = fp2_mul(B.x, z2), uy = fp2_mul(B.y, z3);
    G2 r = {fp2_one(), fp2_one(), fp2_zero()};
#pragma unroll 1
    for (int bit = 63; bit >= 0; --bit) {
        r = g2_dbl(r);
        const bool ea = (a >> bit) & 1u, eb = (b >> bit) & 1u;
        const G2 sum = g2_add_mixed(r, ea ? (eb ? both.x : tx) : ux, ea ? (eb ? both.y : ty) : uy);
        if (ea || eb) r = sum;
    }
    return {r.x, r.y, fp2_mul(r.z, both.z)};
}

TDEC_WAVE1_KERNEL void sig_batch_leaves(uint32_t cap, const uint32_t* __restrict__ nb_dev, uint32_t n_doc,
                                  const BatchDesc* __restrict__ desc, const uint32_t* __restrict__ perm,
                                  const uint8_t* __restrict__ share96, const uint32_t* __restrict__ share_pk,
                                  const uint8_t* __restrict__ seeds, const uint32_t* __restrict__ pk_aff,
                                  const int32_t* __restrict__ pk_status, const uint32_t* __restrict__ pk_tbl,
                                  uint32_t* __restrict__ sums, uint8_t* __restrict__ leaf_ok, const BatchKey key) {
    __shared__ uint8_t sDig[kBatchShares * 32], sBatch[32];
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    if (b >= dev_count(nb_dev, cap)) return;  // grid sized for the bound; the batch count is a device word
    const BatchDesc d = desc[b];
    const uint32_t q = d.start + lane;
    const bool in = q < d.end;
    const uint32_t k = in ? perm[q] : 0u;
    const uint32_t pk = in ? share_pk[k] : 0u;
    bool valid = in && pk_status[pk] == 0;  // the sentinel key (out-of-range indices) is invalid
    G2A s;
    if (valid) valid = g2_decompress(share96 + 96ull * k, s, true);
    if (in && d.ct < n_doc) {
        uint8_t m[32 + 96 + 4];
        for (int i = 0; i < 32; ++i) m[i] = seeds[32ull * d.ct + i];
        for (int i = 0; i < 96; ++i) m[32 + i] = share96[96ull * k + i];
        for (int i = 0; i < 4; ++i) m[128 + i] = (uint8_t)(pk >> (8 * i));
        sha3_bytes(m, sizeof(m), sDig + 32 * lane);
    }
    __syncthreads();
    if (lane == 0) sha3_bytes(sDig, 32u * (d.end - d.start), sBatch);
    __syncthreads();
    uint64_t ra = 0, rb = 0;  // weight r_i = a + b x^2 (a odd: nonzero); pk_i in G1, sig_i in G2
    if (valid) batch_weight(key, sBatch, lane, ra, rb);
    leaf_ok[(uint64_t)b * kBatchShares + lane] = valid ? 1 : 0;
    uint32_t* out = sums + (uint64_t)b * kSigBatchSumWords;
    // G1 side: sum r_i pk_i
    {
        G1 B = {fp_one(), fp_one(), fp_zero()};
        const uint32_t* pa = pk_aff + 32ull * pk;
        if (valid && pa[24] == 0)
            B = pk_tbl ? pk_tbl_mul_ab64(pk_tbl + (uint64_t)pk * kPkTblWords, ra, rb)
                       : g1_mul_ab64(load_fp(pa), load_fp(pa + 12), ra, rb);
#pragma unroll 1
        for (int m = 1; m < 64; m <<= 1) {
            B = g1_add(B, g1_shfl_xor(B, m));
            if (m == 2 && (lane & 3u) == 0) store_jac(out + (lane >> 2) * kSigSumWords, B);
            if (m == 8 && (lane & 15u) == 0) store_jac(out + (kNode16 + (lane >> 4)) * kSigSumWords, B);
        }
        if (lane == 0) store_jac(out + kNodeBatch * kSigSumWords, B);
    }
    // G2 side: sum r_i sig_i
    {
        G2 A = {fp2_one(), fp2_one(), fp2_zero()};
        if (valid && !s.inf) A = g2_mul_ab64(s.x, s.y, ra, rb);
#pragma unroll 1
        for (int m = 1; m < 64; m <<= 1) {
            A = g2_add(A, g2_shfl_xor(A, m));
            if (m == 2 && (lane & 3u) == 0) store_g2jac(out + (lane >> 2) * kSigSumWords + kJacWords, A);
            if (m == 8 && (lane & 15u) == 0)
                store_g2jac(out + (kNode16 + (lane >> 4)) * kSigSumWords + kJacWords, A);
        }
        if (lane == 0) store_g2jac(out + kNodeBatch * kSigSumWords + kJacWords, A);
    }
}

// e(pk, H) * e(-G1, sig) == 1 with H's lines prepared; sig's lines go to `ls`.
BD bool sig_pair_check(const uint32_t* coefH, const Fp& pkx, const Fp& pky, bool pk_inf, const G2A& sig,
                       uint32_t* ls) {
    if (!sig.inf) g2_prepare(sig.x, sig.y, ls);
    return pairing_check2(coefH, pkx, pky, !pk_inf, ls, fp_const(kG1x), fp_neg(fp_const(kG1y)), !sig.inf);
}

// One lane per check item (item base + i; items == null: round 0 over every
// batch, or with `spec` over every batch AND its four 16-groups, item
// 5b + j, so a small batch count does not pay a separate latency-bound round
// for the 16-groups); lines: one G2Prepared slot per lane of this launch.
TDEC_WAVE1_KERNEL void sig_batch_check(uint64_t base, uint32_t cap, const uint32_t* __restrict__ n_dev, uint32_t spec,
                                 const CheckItem* __restrict__ items,
                                 const BatchDesc* __restrict__ desc, const uint32_t* __restrict__ perm,
                                 const uint32_t* __restrict__ sums, const uint8_t* __restrict__ leaf_ok,
                                 const uint32_t* __restrict__ coefH, uint32_t* __restrict__ lines,
                                 uint8_t* __restrict__ ok, CheckItem* __restrict__ next,
                                 uint32_t* __restrict__ next_n, uint32_t* __restrict__ fail_list,
                                 uint32_t* __restrict__ fail_n) {
    // items == null: every batch (count *n_dev), or with `spec` every batch and its 16-groups (5 items each)
    const uint64_t n_items = items ? dev_count(n_dev, cap) : (spec ? 5ull : 1ull) * dev_count(n_dev, cap);
    const uint64_t i = base + grid_lane();
    if (i >= n_items) return;
    uint32_t* my_lines = lines + grid_lane() * kLineWordsPerPoint;  // one G2Prepared slot per lane of a chunk
    const uint32_t j = (uint32_t)i;
    const CheckItem it = items ? items[j]
                               : (spec ? CheckItem{j / 5u, j % 5u == 0 ? kNodeBatch : kNode16 + j % 5u - 1u}
                                       : CheckItem{j, kNodeBatch});
    const BatchDesc d = desc[it.b];
    const uint8_t* lok = leaf_ok + (uint64_t)it.b * kBatchShares;
    const uint32_t l0 = node_first(it.node);
    if (!node_any_valid(lok, l0, l0 + node_size(it.node))) return;
    const uint32_t* sm = sums + (uint64_t)it.b * kSigBatchSumWords + it.node * kSigSumWords;
    const G1A a = g1_to_affine(load_jac(sm));
    const G2A sg = g2_to_affine(load_g2jac(sm + kJacWords));
    const bool pass = sig_pair_check(coefH + (uint64_t)d.ct * kLineWordsPerPoint, a.x, a.y, a.inf, sg, my_lines);
    batch_tree_step(pass, it, d, lok, perm, ok, next, next_n, fail_list, fail_n,
                    spec && !items && it.node == kNodeBatch);
}

// Per-share PublicKeyShare::verify with H prepared per document: share
// sel[base + i] (or base + i), lines: one G2Prepared slot per lane.
TDEC_WAVE1_KERNEL void sig_verify_shares(uint64_t base, uint64_t cap, const uint32_t* __restrict__ n_dev, const uint32_t* __restrict__ sel,
                                   const uint8_t* __restrict__ share96, const uint32_t* __restrict__ share_doc,
                                   const uint32_t* __restrict__ share_pk, const uint32_t* __restrict__ pk_aff,
                                   const int32_t* __restrict__ pk_status, const uint32_t* __restrict__ coefH,
                                   uint32_t* __restrict__ lines, uint8_t* __restrict__ ok) {
    const uint64_t i = base + grid_lane();
    if (i >= dev_count(n_dev, cap)) return;
    uint32_t* my_lines = lines + grid_lane() * kLineWordsPerPoint;  // one G2Prepared slot per lane of a chunk
    const uint64_t k = sel ? sel[i] : i;
    const uint32_t p = share_pk[k];  // sanitised: an out-of-range pair points at the invalid sentinel key
    G2A sig;
    bool good = pk_status[p] == 0 && g2_decompress(share96 + 96ull * k, sig, true);
    if (good) {
        const uint32_t* pa = pk_aff + 32ull * p;
        good = sig_pair_check(coefH + (uint64_t)share_doc[k] * kLineWordsPerPoint, load_fp(pa), load_fp(pa + 12),
                              pa[24] != 0, sig, my_lines);
    }
    ok[k] = good ? 1 : 0;
}

// ------------------------------------------------------------------ unit-test hook
// op: 0 fp_mul(a,b)  1 fp_inv(a)  2 fp2_sqrt(a)  3 g1_decompress  4 g2_decompress
//     5 pairing(P,Q) = final_exp(miller)  6 hash_g2(seed)  7 miller_loop(P,Q) 8 final_exp(f)
//     9 [k]P (64-bit k)  10 P + Q (Jacobian add)  11 Legendre(a), is_square(a + b u)
// Field values cross the boundary as canonical raw limbs (12 u32 LE).
TDEC_WAVE1_KERNEL void tdec_test(int op, uint32_t n, const uint32_t* __restrict__ in,
                                                uint32_t* __restrict__ out, uint32_t in_words,
                                                uint32_t out_words, uint32_t* __restrict__ lines) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t* a = in + (uint64_t)k * in_words;
    uint32_t* o = out + (uint64_t)k * out_words;
    auto ld = [&](int w) { return fp_to_mont(load_fp(a + w)); };
    auto st = [&](int w, const Fp& x) { store_fp(o + w, fp_from_mont(x)); };
    auto st12 = [&](const Fp12& f) {
        const Fp* c[12] = {&f.c0.c0.c0, &f.c0.c0.c1, &f.c0.c1.c0, &f.c0.c1.c1, &f.c0.c2.c0, &f.c0.c2.c1,
                           &f.c1.c0.c0, &f.c1.c0.c1, &f.c1.c1.c0, &f.c1.c1.c1, &f.c1.c2.c0, &f.c1.c2.c1};
        for (int i = 0; i < 12; ++i) st(12 * i, *c[i]);
    };
    if (op == 0) {
        st(0, fp_mul(ld(0), ld(12)));
    } else if (op == 1) {
        st(0, fp_inv(ld(0)));
    } else if (op == 2) {
        bool ok;
        const Fp2 r = fp2_sqrt({ld(0), ld(12)}, ok);
        st(0, r.c0);
        st(12, r.c1);
        o[24] = ok;
    } else if (op == 3) {
        G1A p;
        const bool ok = g1_decompress(reinterpret_cast<const uint8_t*>(a), p, true);
        st(0, p.x);
        st(12, p.y);
        o[24] = ok;
        o[25] = p.inf;
    } else if (op == 4) {
        G2A p;
        const bool ok = g2_decompress(reinterpret_cast<const uint8_t*>(a), p, true);
        st(0, p.x.c0);
        st(12, p.x.c1);
        st(24, p.y.c0);
        st(36, p.y.c1);
        o[48] = ok;
        o[49] = p.inf;
    } else if (op == 5 || op == 7) {
        // in: P.x P.y Q.x0 Q.x1 Q.y0 Q.y1 (canonical affine)
        uint32_t* ln = lines + (uint64_t)k * 72 * kMillerSteps;
        g2_prepare({ld(24), ld(36)}, {ld(48), ld(60)}, ln);
        Fp12 f = miller_loop2<false>(ln, ld(0), ld(12), ld(12), true, ln, ld(0), ld(12), ld(12), false);
        if (op == 5) final_exponentiation(&f);
        st12(f);
    } else if (op == 6) {
        const G2A h = hash_g2_from_seed(reinterpret_cast<const uint8_t*>(a));
        st(0, h.x.c0);
        st(12, h.x.c1);
        st(24, h.y.c0);
        st(36, h.y.c1);
    } else if (op == 9) {
        // in: P.x P.y k_lo k_hi -> affine [k]P (x, y, inf)
        const uint64_t kk = (uint64_t)a[24] | ((uint64_t)a[25] << 32);
        const G1A r = g1_to_affine(g1_mul_u64(ld(0), ld(12), kk));
        st(0, r.x);
        st(12, r.y);
        o[24] = r.inf;
    } else if (op == 10) {
        // in: P.x P.y Q.x Q.y (affine, Z = 1) -> affine P + Q via the Jacobian g1_add
        const G1 p = {ld(0), ld(12), fp_one()}, q = {ld(24), ld(36), fp_one()};
        const G1A r = g1_to_affine(g1_add(p, q));
        st(0, r.x);
        st(12, r.y);
        o[24] = r.inf;
    } else if (op == 11) {
        // in: a (canonical) -> Legendre symbol of a, and fp2_is_square((a, b))
        o[0] = (uint32_t)fp_legendre(ld(0));
        o[1] = fp2_is_square({ld(0), ld(12)}) ? 1u : 0u;
    } else if (op == 8) {
        Fp12 f;
        Fp* c[12] = {&f.c0.c0.c0, &f.c0.c0.c1, &f.c0.c1.c0, &f.c0.c1.c1, &f.c0.c2.c0, &f.c0.c2.c1,
                     &f.c1.c0.c0, &f.c1.c0.c1, &f.c1.c1.c0, &f.c1.c1.c1, &f.c1.c2.c0, &f.c1.c2.c1};
        for (int i = 0; i < 12; ++i) *c[i] = ld(12 * i);
        final_exponentiation(&f);
        st12(f);
    }
}

// ------------------------------------------------------------------ launchers
// Latency build: tdec_kernels_lat.hip compiles this file a second time into
// namespace bls_lat with a one-wave-per-SIMD register budget for every
// kernel.  Launches of at most g_lat_lanes lanes (one wave per SIMD: the
// epoch's 128 ciphertexts, up to ~65 k messages) take those kernels — a lone
// wave has the whole register file and its Fp2 products run as three
// interleaved chains (hbg_fpmul3) — and larger ones the G1 kernels at two
// waves per SIMD.
#if HBG_TDEC_LAT_TU || defined(HBG_FP_COUNT) || defined(HBG_DEBUG_CHECKS)
// (the latency build itself, and the instrumented / diagnostic tool builds:
// every launch stays in this build so counts and checks see all of it)
#define HBG_LAT_DISPATCH(lanes, call) ((void)0)
#else
}  // namespace bls
namespace bls_lat {
hipError_t launch_tdec_ct_decode(uint32_t n, const uint8_t* U48, uint32_t* ct_u, int32_t* u_status, hipStream_t st);
hipError_t launch_tdec_ct_prepare(uint32_t n, const uint8_t* U48, const uint8_t* V, const uint64_t* V_off,
                                  const int32_t* ct_status, uint32_t* coefH, uint8_t* vdig, hipStream_t st);
hipError_t launch_tdec_ct_prepare_w(uint32_t n, const uint8_t* W96, uint32_t* ct_u, const int32_t* u_status,
                                    int32_t* ct_status, uint32_t* coefW, hipStream_t st);
hipError_t launch_tdec_ct_prepare_hw(uint32_t n, const uint8_t* U48, const uint8_t* V, const uint64_t* V_off,
                                     const uint8_t* W96, uint32_t* ct_u, const int32_t* u_status, int32_t* ct_status,
                                     uint32_t* coefH, uint32_t* coefW, hipStream_t st);
hipError_t launch_tdec_pk_prepare(uint32_t n, const uint8_t* pk48, uint32_t* pk_aff, int32_t* pk_status,
                                  hipStream_t st);
hipError_t launch_tdec_verify_shares(uint64_t cap, const uint32_t* n_dev, const uint8_t* share48,
                                     const uint32_t* share_ct, const uint32_t* share_pk, const uint32_t* ct_u,
                                     const int32_t* ct_status, const uint32_t* coefH, const uint32_t* coefW,
                                     const uint32_t* pk_aff, const int32_t* pk_status, uint8_t* ok, hipStream_t st,
                                     const uint32_t* sel, uint32_t* share_aff);
hipError_t launch_tdec_ct_verify(uint32_t n, const uint32_t* ct_u, const int32_t* ct_status, const uint32_t* coefH,
                                 const uint32_t* coefW, uint8_t* ok, hipStream_t st);
hipError_t launch_tdec_combine(uint32_t n, uint32_t t, const uint8_t* share48, const uint32_t* idx,
                               const uint8_t* V, const uint64_t* V_off, uint8_t* out, int32_t* status,
                               uint32_t* scratch, uint8_t* seeds, hipStream_t st, const uint32_t* share_aff,
                               uint32_t n_nodes, const int32_t* pre_status, const uint8_t* share_ok);
hipError_t launch_bls_sign(uint64_t n, uint32_t n_sk, const uint8_t* sk32, const uint32_t* msg_sk,
                           const uint8_t* msg, const uint64_t* off, uint8_t* sig96, int32_t* err, hipStream_t st);
hipError_t launch_bls_verify(uint64_t n, uint32_t n_pk, const uint32_t* pk_aff, const int32_t* pk_status,
                             const uint32_t* msg_pk, const uint8_t* msg, const uint64_t* off, const uint8_t* sig96,
                             uint32_t* lines, uint8_t* ok, int32_t* err, hipStream_t st);
hipError_t launch_wire_verify_frames(uint64_t n, const uint32_t* pk_aff, const int32_t* pk_status, uint32_t n_pk,
                                     const uint32_t* frame_pk, const uint8_t* frames, const uint64_t* off,
                                     uint32_t* lines, int32_t* status, hipStream_t st);
hipError_t launch_tdec_encrypt(uint64_t n, const uint32_t* pk_aff, const int32_t* pk_status, const uint8_t* r32,
                               const uint8_t* msg, const uint64_t* off, uint8_t* U48, uint8_t* V, uint8_t* W96,
                               uint8_t* seeds, uint8_t* vdig, int32_t* est, int32_t* err, hipStream_t st);
hipError_t launch_tdec_decrypt_share(uint64_t n, uint32_t n_ct, uint32_t n_sk, const uint32_t* u_aff,
                                     const int32_t* u_status, const uint8_t* sk32, const uint32_t* share_ct,
                                     const uint32_t* share_sk, uint8_t* share48, int32_t* status, int32_t* err,
                                     hipStream_t st);
hipError_t launch_sig_doc_prepare(uint32_t n, const uint8_t* doc, const uint64_t* off, uint32_t* coefH,
                                  uint8_t* seeds, hipStream_t st);
}  // namespace bls_lat
namespace bls {
// 1,024 waves of 64 lanes: one per SIMD, the latency build's occupancy
// (hbg_test_set_latency_lanes overrides it: the parity tests run both builds)
std::atomic<uint64_t> g_lat_lanes{64ull * 1024};
#define HBG_LAT_DISPATCH(lanes, call)                                                           \
    do {                                                                                        \
        if ((uint64_t)(lanes) <= g_lat_lanes.load(std::memory_order_relaxed)) return ::hbg::bls_lat::call; \
    } while (0)
#endif
#ifdef HBG_FP_COUNT
// Instrumented builds (tools/fpcount.py): every launcher first closes the
// previous launch's count (stream sync + read/clear of g_fp_count) and
// attributes it to that launch's kernel; hbg_fp_count_report() closes the
// last one and returns {"kernel": [fp_mul, fp_sqr, launches], ...} as JSON.
}  // namespace bls
}  // namespace hbg
#include <map>
#include <string>
namespace hbg {
namespace bls {
static std::map<std::string, uint64_t[3]> g_count_by_kernel;
static std::string g_count_cur;
static hipStream_t g_count_stream = nullptr;
static void count_mark(const char* name, hipStream_t st) {
    if (g_count_stream) (void)hipStreamSynchronize(g_count_stream);
    unsigned long long v[2] = {0, 0};
    (void)hipMemcpyFromSymbol(v, HIP_SYMBOL(g_fp_count), sizeof(v));
    const unsigned long long z[2] = {0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fp_count), z, sizeof(z));
    if (!g_count_cur.empty()) {
        g_count_by_kernel[g_count_cur][0] += v[0];
        g_count_by_kernel[g_count_cur][1] += v[1];
    }
    g_count_cur = name ? name : "";
    g_count_stream = st;
    if (name) g_count_by_kernel[g_count_cur][2] += 1;
}
#define HBG_COUNT_MARK(name, st) count_mark(name, st)
#else
#define HBG_COUNT_MARK(name, st) ((void)0)
#endif
// Up to this many items per call SHA3(V) runs one wave per item (latency);
// beyond it one lane per item (throughput: configs[3]'s 100 k short V).
constexpr uint64_t kVDigestWaveMax = 8192;
hipError_t launch_tdec_v_digest(uint64_t n, const uint8_t* V, const uint64_t* V_off, uint8_t* dig, hipStream_t st) {
    HBG_COUNT_MARK("tdec_v_digest", st);
    if (n == 0) return hipSuccess;
    HBG_GRID_CHECK((n + 63) / 64, 64);
#ifdef HBG_TOOL_AB
    // tool builds only (tools/build_variant.py ... -DHBG_TOOL_AB; tools/sha3v_probe.py): A/B switches of
    // the sponge schedule and of the wave / lane cut, read once per process
    static const bool wave64 = std::getenv("HBG_SHA3_WAVE64") != nullptr;  // the (lo, hi)-per-lane sponge
    static const bool three_stage = std::getenv("HBG_SHA3_3STAGE") != nullptr;  // theta in two stages
    static const uint64_t wave_max = [] {
        const char* v = std::getenv("HBG_VDIGEST_WAVE_MAX");
        char* end = nullptr;
        const unsigned long long x = v ? std::strtoull(v, &end, 10) : 0;
        return (v && end != v && *end == 0) ? (uint64_t)x : kVDigestWaveMax;  // malformed: the default
    }();
#else
    constexpr bool wave64 = false, three_stage = false;
    constexpr uint64_t wave_max = kVDigestWaveMax;
#endif
    if (n <= wave_max && wave64)
        tdec_v_digest_wave64<<<dim3((uint32_t)n), dim3(64), 0, st>>>(n, V, V_off, dig);
    else if (n <= wave_max && three_stage)
        tdec_v_digest_wave<false><<<dim3((uint32_t)n), dim3(64), 0, st>>>(n, V, V_off, dig);
    else if (n <= wave_max)  // few items (the epoch's contributions): one wave per sponge
        tdec_v_digest_wave<true><<<dim3((uint32_t)n), dim3(64), 0, st>>>(n, V, V_off, dig);
    else
        tdec_v_digest<<<dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, st>>>(n, V, V_off, dig);
    return hipGetLastError();
}
hipError_t launch_tdec_keystream_xor(uint64_t n, const uint8_t* seeds, const uint8_t* in, const uint64_t* off,
                                     uint8_t* out, const int32_t* status, hipStream_t st) {
    HBG_COUNT_MARK("tdec_keystream_xor", st);
    if (n == 0) return hipSuccess;
    constexpr uint64_t kMaxBlocks = 1ull << 16;  // items stride over the grid beyond this
    tdec_keystream_xor<<<dim3((uint32_t)(n < kMaxBlocks ? n : kMaxBlocks)), dim3(256), 0, st>>>(n, seeds, in, off,
                                                                                             out, status);
    return hipGetLastError();
}
hipError_t launch_tdec_ct_decode(uint32_t n, const uint8_t* U48, uint32_t* ct_u, int32_t* u_status, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_tdec_ct_decode(n, U48, ct_u, u_status, st));
    HBG_COUNT_MARK("tdec_ct_decode", st);
    if (n == 0) return hipSuccess;
    tdec_ct_decode<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(n, U48, ct_u, u_status);
    return hipGetLastError();
}
hipError_t launch_tdec_ct_prepare(uint32_t n, const uint8_t* U48, const uint8_t* V, const uint64_t* V_off,
                                  const int32_t* ct_status, uint32_t* coefH, uint8_t* vdig, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_tdec_ct_prepare(n, U48, V, V_off, ct_status, coefH, vdig, st));
    if (vdig) {  // else the sponge runs inline, one lane per ciphertext
        hipError_t e = launch_tdec_v_digest(n, V, V_off, vdig, st);
        if (e != hipSuccess) return e;
    }
    HBG_COUNT_MARK("tdec_ct_prepare", st);
    tdec_ct_prepare<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(n, U48, V, V_off, vdig, ct_status, coefH);
    return hipGetLastError();
}
hipError_t launch_tdec_ct_prepare_w(uint32_t n, const uint8_t* W96, uint32_t* ct_u, const int32_t* u_status,
                                    int32_t* ct_status, uint32_t* coefW, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_tdec_ct_prepare_w(n, W96, ct_u, u_status, ct_status, coefW, st));
    HBG_COUNT_MARK("tdec_ct_prepare_w", st);
    if (n == 0) return hipSuccess;
    tdec_ct_prepare_w<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(n, W96, ct_u, u_status, ct_status, coefW);
    return hipGetLastError();
}
hipError_t launch_tdec_ct_prepare_hw(uint32_t n, const uint8_t* U48, const uint8_t* V, const uint64_t* V_off,
                                     const uint8_t* W96, uint32_t* ct_u, const int32_t* u_status, int32_t* ct_status,
                                     uint32_t* coefH, uint32_t* coefW, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_tdec_ct_prepare_hw(n, U48, V, V_off, W96, ct_u, u_status, ct_status, coefH, coefW, st));
    HBG_COUNT_MARK("tdec_ct_prepare_hw", st);
    if (n == 0) return hipSuccess;
    tdec_ct_prepare_hw<<<dim3(2 * ((n + 63) / 64)), dim3(64), 0, st>>>(n, U48, V, V_off, W96, ct_u, u_status,
                                                                       ct_status, coefH, coefW);
    return hipGetLastError();
}
hipError_t launch_tdec_pk_prepare(uint32_t n, const uint8_t* pk48, uint32_t* pk_aff, int32_t* pk_status,
                                  hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_tdec_pk_prepare(n, pk48, pk_aff, pk_status, st));
    HBG_COUNT_MARK("tdec_pk_prepare", st);
    tdec_pk_prepare<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(n, pk48, pk_aff, pk_status);
    return hipGetLastError();
}
// Grid of a round over at most `cap` items, one item per lane: lanes past the
// device-side count return at once.  The TDec kernels handle ONE item per lane
// (round 1's launch shape, run at 6.4M shares); a grid-stride variant over a
// resident grid faulted at >= 4M shares, root cause open.
static dim3 item_grid(uint64_t cap) { return dim3((uint32_t)((cap + 63) / 64)); }
// Chunks for kernels with a per-lane G2Prepared slot (sig_*): launches of at
// most kChunkLanes items, the slot indexed by the lane within the chunk.
constexpr uint64_t kChunkLanes = 64ull * kResidentBlocks;

hipError_t launch_tdec_verify_shares(uint64_t cap, const uint32_t* n_dev, const uint8_t* share48,
                                     const uint32_t* share_ct, const uint32_t* share_pk, const uint32_t* ct_u,
                                     const int32_t* ct_status, const uint32_t* coefH, const uint32_t* coefW,
                                     const uint32_t* pk_aff, const int32_t* pk_status, uint8_t* ok, hipStream_t st,
                                     const uint32_t* sel, uint32_t* share_aff) {
    HBG_LAT_DISPATCH(cap, launch_tdec_verify_shares(cap, n_dev, share48, share_ct, share_pk, ct_u, ct_status, coefH, coefW, pk_aff, pk_status, ok, st, sel, share_aff));
    HBG_COUNT_MARK("tdec_verify_shares", st);
    if (cap == 0) return hipSuccess;
    tdec_verify_shares<<<item_grid(cap), dim3(64), 0, st>>>(cap, n_dev, share48, share_ct, share_pk, ct_u,
                                                                ct_status, coefH, coefW, pk_aff, pk_status, ok, sel,
                                                                share_aff);
    return hipGetLastError();
}

hipError_t launch_tdec_index_sanitize(uint64_t n, const uint32_t* a, uint32_t a_bound, const uint32_t* b,
                                      uint32_t b_bound, uint32_t* a_out, uint32_t* b_out, int32_t* err,
                                      hipStream_t st) {
    HBG_COUNT_MARK("tdec_index_sanitize", st);
    if (n == 0) return hipSuccess;
    HBG_GRID_CHECK((n + 255) / 256, 256);
    tdec_index_sanitize<<<dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st>>>(n, a, a_bound, b, b_bound, a_out,
                                                                               b_out, err);
    return hipGetLastError();
}

// ---- batched verification host driver pieces
size_t tdec_batch_temp_bytes(uint32_t n) {
    size_t a = 0, b = 0, c = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    (void)hipcub::DeviceScan::InclusiveScan(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, hipcub::Max(),
                                            (int)n);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    return (a > b ? (a > c ? a : c) : (b > c ? b : c)) + 256;
}

// Sort shares by ciphertext (stable), cut batches; *nb_dev <- number of batches
// (a device word: no host round trip).  Keys are < n_keys.
hipError_t launch_tdec_batch_plan(uint32_t n, uint32_t n_keys, const uint32_t* share_ct, uint32_t* keys,
                                  uint32_t* perm, uint32_t* tmp_a, uint32_t* tmp_b, BatchDesc* desc, void* temp,
                                  size_t temp_bytes, uint32_t* nb_dev, hipStream_t st) {
    HBG_COUNT_MARK("tdec_batch_plan", st);
    const dim3 g((n + 255) / 256), blk(256);
    int bits = 1;
    while (bits < 32 && (1ull << bits) < n_keys) ++bits;
    tdec_iota<<<g, blk, 0, st>>>(n, tmp_a);
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, share_ct, keys, tmp_a, perm, (int)n, 0, bits,
                                                      st);
    if (e != hipSuccess) return e;
    tdec_group_marks<<<g, blk, 0, st>>>(n, keys, tmp_a);
    e = hipcub::DeviceScan::InclusiveScan(temp, temp_bytes, tmp_a, tmp_b, hipcub::Max(), (int)n, st);
    if (e != hipSuccess) return e;
    tdec_batch_heads<<<g, blk, 0, st>>>(n, tmp_b, tmp_a);            // tmp_a = head flags
    e = hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, tmp_a, tmp_b, (int)n, st);  // tmp_b = batch id + 1
    if (e != hipSuccess) return e;
    tdec_batch_desc<<<g, blk, 0, st>>>(n, keys, tmp_a, tmp_b, desc);
    // number of batches = heads in [0, n)
    return hipMemcpyAsync(nb_dev, tmp_b + (n - 1), 4, hipMemcpyDeviceToDevice, st);
}

void tdec_debug_bounds(uint64_t n, uint64_t nb_max, uint64_t n_ct1, uint64_t n_pk1) {
#ifdef HBG_DEBUG_CHECKS
    const uint64_t v[4] = {n, nb_max, n_ct1, n_pk1};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), v, sizeof(v));
#else
    (void)n, (void)nb_max, (void)n_ct1, (void)n_pk1;
#endif
}

uint32_t tdec_batch_bound(uint32_t n, uint32_t n_keys) {
    // sum over keys of ceil(count / 64) <= n / 64 + (number of distinct keys)
    const uint64_t distinct = n < n_keys ? n : n_keys;
    const uint64_t b = (uint64_t)n / kBatchShares + distinct;
    return (uint32_t)(b < n ? b : n);
}

hipError_t launch_tdec_batch_leaves(uint32_t nb_max, const uint32_t* nb_dev, uint32_t n_ct, const BatchDesc* desc,
                                    const uint32_t* perm, const uint8_t* share48, const uint32_t* share_pk,
                                    const uint8_t* U48, const int32_t* ct_status, const uint32_t* pk_aff,
                                    const int32_t* pk_status, const uint32_t* pk_tbl, uint32_t* sums,
                                    uint8_t* leaf_ok, const BatchKey& key, hipStream_t st, uint32_t* share_aff) {
    HBG_COUNT_MARK("tdec_batch_leaves", st);
    if (nb_max == 0) return hipSuccess;
    tdec_batch_leaves<<<dim3(nb_max), dim3(64), 0, st>>>(nb_max, nb_dev, n_ct, desc, perm, share48, share_pk, U48, ct_status,
                                                         pk_aff, pk_status, pk_tbl, sums, leaf_ok, key, share_aff);
    return hipGetLastError();
}

size_t tdec_pk_table_bytes(uint32_t n_pk) { return 4ull * kPkTblWords * n_pk; }

hipError_t launch_tdec_pk_table(uint32_t n_pk, const uint32_t* pk_aff, uint32_t* tbl, hipStream_t st,
                                uint32_t layout) {
    HBG_COUNT_MARK("tdec_pk_table", st);
    if (n_pk == 0) return hipSuccess;
    tdec_pk_table<<<dim3((n_pk * 2048u + 63) / 64), dim3(64), 0, st>>>(n_pk, pk_aff, tbl, layout);
    return hipGetLastError();
}

hipError_t launch_tdec_bin_root(uint32_t cap, const uint32_t* nb_dev, const BatchDesc* desc, const uint32_t* perm,
                                const uint32_t* sums, const uint8_t* leaf_ok, const int32_t* ct_status,
                                const uint32_t* ct_u, const uint32_t* coefH, const uint32_t* coefW, uint8_t* ok,
                                uint32_t* gt_out, BinItem* next, uint32_t* next_n, uint32_t next_cap,
                                uint32_t* fail_list, uint32_t* fail_n, hipStream_t st) {
    HBG_COUNT_MARK("tdec_bin_root", st);
    if (cap == 0) return hipSuccess;
    tdec_bin_root<<<item_grid(cap), dim3(64), 0, st>>>(cap, nb_dev, desc, perm, sums, leaf_ok, ct_status, ct_u, coefH,
                                                       coefW, ok, gt_out, next, next_n, next_cap, fail_list, fail_n);
    return hipGetLastError();
}
hipError_t launch_tdec_bin_step(uint32_t cap, const uint32_t* n_dev, const BinItem* items, const BatchDesc* desc,
                                const uint32_t* perm, const uint32_t* sums, const uint8_t* leaf_ok,
                                const uint32_t* ct_u, const uint32_t* coefH, const uint32_t* coefW, uint8_t* ok,
                                const uint32_t* gt_in, uint32_t* gt_out, BinItem* next, uint32_t* next_n,
                                uint32_t next_cap, uint32_t* fail_list, uint32_t* fail_n, hipStream_t st) {
    HBG_COUNT_MARK("tdec_bin_step", st);
    if (cap == 0) return hipSuccess;
    tdec_bin_step<<<item_grid(cap), dim3(64), 0, st>>>(cap, n_dev, items, desc, perm, sums, leaf_ok, ct_u, coefH,
                                                       coefW, ok, gt_in, gt_out, next, next_n, next_cap, fail_list,
                                                       fail_n);
    return hipGetLastError();
}
hipError_t launch_tdec_select(uint32_t n_ct, uint32_t N, uint32_t t, const uint8_t* ct_ok, const uint8_t* ok,
                              const uint32_t* arrival, uint32_t arrival_len, const uint8_t* share48,
                              uint32_t* sel_idx, uint8_t* sel48, uint8_t* outcome, int32_t* sel_status,
                              hipStream_t st) {
    HBG_COUNT_MARK("tdec_select", st);
    if (n_ct == 0) return hipSuccess;
    tdec_select<<<dim3((n_ct + 255) / 256), dim3(256), 0, st>>>(n_ct, N, t, ct_ok, ok, arrival, arrival_len, share48,
                                                                 sel_idx, sel48, outcome, sel_status);
    return hipGetLastError();
}
hipError_t launch_tdec_pair_index(uint64_t n, uint32_t N, uint32_t* sct, uint32_t* spk, hipStream_t st) {
    HBG_COUNT_MARK("tdec_pair_index", st);
    if (n == 0) return hipSuccess;
    HBG_GRID_CHECK((n + 255) / 256, 256);
    tdec_pair_index<<<dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st>>>(n, N, sct, spk);
    return hipGetLastError();
}
hipError_t launch_tdec_status_merge(uint32_t n, const int32_t* sel_status, int32_t* status, hipStream_t st) {
    HBG_COUNT_MARK("tdec_status_merge", st);
    if (n == 0) return hipSuccess;
    tdec_status_merge<<<dim3((n + 255) / 256), dim3(256), 0, st>>>(n, sel_status, status);
    return hipGetLastError();
}
hipError_t launch_tdec_ct_verify(uint32_t n, const uint32_t* ct_u, const int32_t* ct_status, const uint32_t* coefH,
                                 const uint32_t* coefW, uint8_t* ok, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_tdec_ct_verify(n, ct_u, ct_status, coefH, coefW, ok, st));
    HBG_COUNT_MARK("tdec_ct_verify", st);
    tdec_ct_verify<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(n, ct_u, ct_status, coefH, coefW, ok);
    return hipGetLastError();
}
hipError_t launch_tdec_combine(uint32_t n, uint32_t t, const uint8_t* share48, const uint32_t* idx,
                               const uint8_t* V, const uint64_t* V_off, uint8_t* out, int32_t* status,
                               uint32_t* scratch, uint8_t* seeds, hipStream_t st, const uint32_t* share_aff,
                               uint32_t n_nodes, const int32_t* pre_status, const uint8_t* share_ok) {
    HBG_LAT_DISPATCH((uint64_t)n * (t + 1 <= 24 ? 16u : 32u),
                     launch_tdec_combine(n, t, share48, idx, V, V_off, out, status, scratch, seeds, st, share_aff,
                                         n_nodes, pre_status, share_ok));
    HBG_COUNT_MARK("tdec_combine", st);
    if (n == 0) return hipSuccess;
    HBG_GRID_CHECK(n, 64);  // every grid of this call, before the first launch
    // scratch: >= 36 words per ciphertext (the MSM kernels' Jacobian sums)
    if (t + 1 <= 24)
        tdec_combine_msm<16, 24><<<dim3((n + 3) / 4), dim3(64), 0, st>>>(n, t, share48, idx, scratch, status,
                                                                         share_aff, n_nodes, pre_status, share_ok);
    else if (t + 1 <= 32)
        tdec_combine_msm<32, 32><<<dim3((n + 1) / 2), dim3(64), 0, st>>>(n, t, share48, idx, scratch, status,
                                                                         share_aff, n_nodes, pre_status, share_ok);
    else if (t + 1 <= 64)  // two shares a lane: ~28 % fewer Fp products per ciphertext than <64, 64> at t = 42
        tdec_combine_msm<32, 64><<<dim3((n + 1) / 2), dim3(64), 0, st>>>(n, t, share48, idx, scratch, status,
                                                                         share_aff, n_nodes, pre_status, share_ok);
    else
        tdec_combine<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(n, t, share48, idx, seeds, status, scratch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (t + 1 <= 64) {
        tdec_combine_seed<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(n, scratch, status, seeds);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    // xor_with_hash(g, V) of every ciphertext whose combination succeeded
    return launch_tdec_keystream_xor(n, seeds, V, V_off, out, status, st);
}
static dim3 grid64(uint64_t n) { return dim3((uint32_t)((n + 63) / 64)); }
hipError_t launch_bls_sign(uint64_t n, uint32_t n_sk, const uint8_t* sk32, const uint32_t* msg_sk,
                           const uint8_t* msg, const uint64_t* off, uint8_t* sig96, int32_t* err, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_bls_sign(n, n_sk, sk32, msg_sk, msg, off, sig96, err, st));
    HBG_COUNT_MARK("bls_sign", st);
    if (n == 0) return hipSuccess;
    bls_sign<<<grid64(n), dim3(64), 0, st>>>(n, n_sk, sk32, msg_sk, msg, off, sig96, err);
    return hipGetLastError();
}
hipError_t launch_bls_verify(uint64_t n, uint32_t n_pk, const uint32_t* pk_aff, const int32_t* pk_status,
                             const uint32_t* msg_pk, const uint8_t* msg, const uint64_t* off, const uint8_t* sig96,
                             uint32_t* lines, uint8_t* ok, int32_t* err, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_bls_verify(n, n_pk, pk_aff, pk_status, msg_pk, msg, off, sig96, lines, ok, err, st));
    HBG_COUNT_MARK("bls_verify", st);
    if (n == 0) return hipSuccess;
    bls_verify<<<grid64(n), dim3(64), 0, st>>>(n, n_pk, pk_aff, pk_status, msg_pk, msg, off, sig96, lines, ok, err);
    return hipGetLastError();
}
hipError_t launch_wire_verify_frames(uint64_t n, const uint32_t* pk_aff, const int32_t* pk_status, uint32_t n_pk,
                                     const uint32_t* frame_pk, const uint8_t* frames, const uint64_t* off,
                                     uint32_t* lines, int32_t* status, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_wire_verify_frames(n, pk_aff, pk_status, n_pk, frame_pk, frames, off, lines, status, st));
    HBG_COUNT_MARK("wire_verify_frames", st);
    if (n == 0) return hipSuccess;
    wire_verify_frames<<<grid64(n), dim3(64), 0, st>>>(n, pk_aff, pk_status, n_pk, frame_pk, frames, off, lines,
                                                       status);
    return hipGetLastError();
}
hipError_t launch_tdec_encrypt(uint64_t n, const uint32_t* pk_aff, const int32_t* pk_status, const uint8_t* r32,
                               const uint8_t* msg, const uint64_t* off, uint8_t* U48, uint8_t* V, uint8_t* W96,
                               uint8_t* seeds, uint8_t* vdig, int32_t* est, int32_t* err, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_tdec_encrypt(n, pk_aff, pk_status, r32, msg, off, U48, V, W96, seeds, vdig, est, err, st));
    HBG_COUNT_MARK("tdec_encrypt", st);
    if (n == 0) return hipSuccess;
    HBG_GRID_CHECK((n + 63) / 64, 64);  // every grid of this call (v_digest's too), before the first launch
    tdec_encrypt_u<<<grid64(n), dim3(64), 0, st>>>(n, pk_aff, pk_status, r32, U48, W96, seeds, est, err);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = launch_tdec_keystream_xor(n, seeds, msg, off, V, est, st);
    if (e == hipSuccess) e = launch_tdec_v_digest(n, V, off, vdig, st);
    if (e != hipSuccess) return e;
    HBG_COUNT_MARK("tdec_encrypt", st);
    tdec_encrypt_w<<<grid64(n), dim3(64), 0, st>>>(n, r32, U48, V, off, vdig, est, W96);
    return hipGetLastError();
}
hipError_t launch_tdec_decrypt_share(uint64_t n, uint32_t n_ct, uint32_t n_sk, const uint32_t* u_aff,
                                     const int32_t* u_status, const uint8_t* sk32, const uint32_t* share_ct,
                                     const uint32_t* share_sk, uint8_t* share48, int32_t* status, int32_t* err,
                                     hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_tdec_decrypt_share(n, n_ct, n_sk, u_aff, u_status, sk32, share_ct, share_sk, share48, status, err, st));
    HBG_COUNT_MARK("tdec_decrypt_share", st);
    if (n == 0) return hipSuccess;
    tdec_decrypt_share<<<grid64(n), dim3(64), 0, st>>>(n, n_ct, n_sk, u_aff, u_status, sk32, share_ct, share_sk,
                                                       share48, status, err);
    return hipGetLastError();
}
hipError_t launch_coin_combine(uint32_t n, uint32_t t, const uint8_t* share96, const uint32_t* idx, uint8_t* sig96,
                               uint8_t* parity, int32_t* status, hipStream_t st) {
    HBG_COUNT_MARK("coin_combine", st);
    if (n == 0) return hipSuccess;
    if (t + 1 > 64) return hipErrorInvalidValue;
    if (t + 1 <= 32)
        coin_combine_grp<32><<<dim3((n + 1) / 2), dim3(64), 0, st>>>(n, t, share96, idx, sig96, parity, status);
    else
        coin_combine_grp<64><<<dim3(n), dim3(64), 0, st>>>(n, t, share96, idx, sig96, parity, status);
    return hipGetLastError();
}
hipError_t launch_tdec_test(int op, uint32_t n, const uint32_t* in, uint32_t* out, uint32_t in_words,
                            uint32_t out_words, uint32_t* lines, hipStream_t st) {
    HBG_COUNT_MARK("tdec_test", st);
    tdec_test<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(op, n, in, out, in_words, out_words, lines);
    return hipGetLastError();
}

#undef BD

hipError_t launch_sig_doc_prepare(uint32_t n, const uint8_t* doc, const uint64_t* off, uint32_t* coefH,
                                  uint8_t* seeds, hipStream_t st) {
    HBG_LAT_DISPATCH(n, launch_sig_doc_prepare(n, doc, off, coefH, seeds, st));
    HBG_COUNT_MARK("sig_doc_prepare", st);
    if (n == 0) return hipSuccess;
    sig_doc_prepare<<<dim3((n + 63) / 64), dim3(64), 0, st>>>(n, doc, off, coefH, seeds);
    return hipGetLastError();
}
hipError_t launch_sig_batch_leaves(uint32_t nb_max, const uint32_t* nb_dev, uint32_t n_doc, const BatchDesc* desc,
                                   const uint32_t* perm, const uint8_t* share96, const uint32_t* share_pk,
                                   const uint8_t* seeds, const uint32_t* pk_aff, const int32_t* pk_status,
                                   const uint32_t* pk_tbl, uint32_t* sums, uint8_t* leaf_ok, const BatchKey& key,
                                   hipStream_t st) {
    HBG_COUNT_MARK("sig_batch_leaves", st);
    if (nb_max == 0) return hipSuccess;
    sig_batch_leaves<<<dim3(nb_max), dim3(64), 0, st>>>(nb_max, nb_dev, n_doc, desc, perm, share96, share_pk, seeds, pk_aff,
                                                        pk_status, pk_tbl, sums, leaf_ok, key);
    return hipGetLastError();
}
// lines: kResidentBlocks * 64 G2Prepared slots (one per lane of a launch chunk)
hipError_t launch_sig_batch_check(uint32_t cap, const uint32_t* n_dev, uint32_t spec, const CheckItem* items,
                                  const BatchDesc* desc, const uint32_t* perm, const uint32_t* sums,
                                  const uint8_t* leaf_ok, const uint32_t* coefH, uint32_t* lines, uint8_t* ok,
                                  CheckItem* next, uint32_t* next_n, uint32_t* fail_list, uint32_t* fail_n,
                                  hipStream_t st) {
    HBG_COUNT_MARK("sig_batch_check", st);
    if (cap == 0) return hipSuccess;
    const uint64_t items_cap = items ? cap : (spec ? 5ull : 1ull) * cap;
    for (uint64_t base = 0; base < items_cap; base += kChunkLanes) {
        const uint64_t m = items_cap - base < kChunkLanes ? items_cap - base : kChunkLanes;
        sig_batch_check<<<item_grid(m), dim3(64), 0, st>>>(base, cap, n_dev, spec, items, desc, perm, sums, leaf_ok,
                                                           coefH, lines, ok, next, next_n, fail_list, fail_n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t launch_sig_verify_shares(uint64_t cap, const uint32_t* n_dev, const uint32_t* sel, const uint8_t* share96,
                                    const uint32_t* share_doc, const uint32_t* share_pk, const uint32_t* pk_aff,
                                    const int32_t* pk_status, const uint32_t* coefH, uint32_t* lines, uint8_t* ok,
                                    hipStream_t st) {
    HBG_COUNT_MARK("sig_verify_shares", st);
    if (cap == 0) return hipSuccess;
    for (uint64_t base = 0; base < cap; base += kChunkLanes) {
        const uint64_t m = cap - base < kChunkLanes ? cap - base : kChunkLanes;
        sig_verify_shares<<<item_grid(m), dim3(64), 0, st>>>(base, cap, n_dev, sel, share96, share_doc, share_pk,
                                                             pk_aff, pk_status, coefH, lines, ok);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace bls
}  // namespace hbg

#ifdef HBG_FP_COUNT
#if !HBG_TDEC_LAT_TU  // one definition: the throughput build reports its own launches
extern "C" int hbg_fp_count_report(char* buf, uint64_t cap) {
    using namespace hbg::bls;
    count_mark(nullptr, nullptr);
    std::string js = "{";
    bool first = true;
    for (auto& kv : g_count_by_kernel) {
        js += (first ? "\"" : ", \"") + kv.first + "\": [" + std::to_string(kv.second[0]) + ", " +
              std::to_string(kv.second[1]) + ", " + std::to_string(kv.second[2]) + "]";
        first = false;
    }
    js += "}";
    g_count_by_kernel.clear();
    if (js.size() + 1 > cap) return -1;
    memcpy(buf, js.c_str(), js.size() + 1);
    return 0;
}
#endif
#endif

#if !HBG_TDEC_LAT_TU
// hbgpu_testing.h: launches of at most `lanes` lanes take the latency build
// (0: none, UINT64_MAX: all); returns the previous value.
extern "C" uint64_t hbg_test_set_latency_lanes(uint64_t lanes) {
#if defined(HBG_FP_COUNT) || defined(HBG_DEBUG_CHECKS)
    (void)lanes;
    return 0;
#else
    return hbg::bls::g_lat_lanes.exchange(lanes);
#endif
}
#endif
