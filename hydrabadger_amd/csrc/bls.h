// bls.h — BLS12-381 arithmetic for gfx950: one field element per work-item.
//
// Restates the zkcrypto `pairing` crate's bls12_381 module [EXT] as
// threshold_crypto uses it.  Values are bit-identical
// to the crate's (same Montgomery domain R = 2^384, same tower, same
// G2Prepared line coefficients, same final-exponentiation chain), so every
// intermediate can be unit-tested against oracle/bls12_381.py.
//
// gfx950 mapping
//  * Fp = 12 x u32 limbs as an ext_vector so it travels in VGPRs.  The
//    Montgomery multiplications are the only out-of-line code: fixed-register
//    leaf subroutines (bls_fp_sub.h, tools/gen_bls_fp_sub.py: 288
//    v_mad_u64_u32 + 288 carry counts per product, 1, 2 or 3 independent
//    products interleaved per call) entered by an inline-asm s_swappc whose
//    clobber list names exactly the registers they write — so everything
//    above them inlines and stays in registers across the calls (the standard
//    call ABI would clobber ~150 VGPRs per multiplication).
//  * Fp2 / Fp6 / Fp12 are plain structs of Fp; exponentiations run rolled
//    loops over constant exponent words (scalar loads, wave-uniform branches).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls_consts.h"
#ifdef HBG_FP_SUB_HEADER  // tool builds only (tools/build_variant.py): another generated body
#include HBG_FP_SUB_HEADER
#else
#include "bls_fp_sub.h"
#endif

namespace hbg {
namespace bls {

#define BD __device__ __forceinline__

template <int N>
BD Fp fp_const(const uint32_t (&c)[N]) {
    Fp r;
#pragma unroll
    for (int i = 0; i < 12; ++i) r[i] = c[i];
    return r;
}

BD Fp fp_zero() {
    Fp r;
#pragma unroll
    for (int i = 0; i < 12; ++i) r[i] = 0u;
    return r;
}

BD Fp fp_one() { return fp_const(kOne); }

// Instrumented builds only (tools/fpcount.py compiles with -DHBG_FP_COUNT):
// count the Fp multiplications / squarings every kernel executes, attributed
// per launch on the host (tdec_kernels.hip HBG_COUNT_MARK).  The product
// library has no counter.  The counter is one atomic add of 1 per active lane
// per product, with the compiler's wave-aggregating atomic optimizer off
// (tools/build_variant.py passes -amdgpu-atomic-optimizer-strategy=None): NO
// divergent branch next to the products.  Round 4's counter (mode 0: one
// wave-aggregated add by the first active lane, `if (lane == first)`) made
// the G2 kernels compute wrong points and then fault ("The
// HBG_FP_COUNT fault"); modes 0 and 4 stay for tools/ctw_probe.py.
#ifdef HBG_FP_COUNT
__device__ unsigned long long g_fp_count[2];  // [0] fp_mul, [1] fp_sqr
#ifndef HBG_FP_COUNT_MODE
#define HBG_FP_COUNT_MODE 1
#endif
__device__ __forceinline__ void fp_count(int which) {
#if HBG_FP_COUNT_MODE == 1  // every active lane adds 1 (no divergent branch)
    atomicAdd(&g_fp_count[which], 1ull);
#else
    const uint64_t m = __builtin_amdgcn_read_exec();
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
#if HBG_FP_COUNT_MODE == 0  // round 4: one wave-aggregated atomic by the first active lane
    if (lane == (uint32_t)__builtin_ctzll(m)) atomicAdd(&g_fp_count[which], (unsigned long long)__builtin_popcountll(m));
#else  // mode 4 (diagnostic): the same branch around an empty statement, no memory operation
    if (lane == (uint32_t)__builtin_ctzll(m)) asm volatile("s_nop 0" ::: "memory");
#endif
#endif
}
#define HBG_FP_COUNT_CALL(which) fp_count(which)
#else
#define HBG_FP_COUNT_CALL(which) ((void)0)
#endif

// Diagnostic tool builds only (tools/ctw_probe.py, -DHBG_FP_VERIFY): every
// product is recomputed by a portable CIOS multiplication (compiler code, no
// asm) and the first mismatch is recorded with its call site.
// (-DHBG_FP_PORTABLE, tool builds of tools/ctw_probe.py only: every product
// is this portable compiler-generated CIOS — no inline asm anywhere.)
#if defined(HBG_FP_VERIFY) || defined(HBG_FP_PORTABLE)
__device__ __forceinline__ Fp fp_mul_ref(const Fp& a, const Fp& b) {
    uint32_t t[14];
#pragma unroll
    for (int j = 0; j < 14; ++j) t[j] = 0;
#pragma unroll 1
    for (int i = 0; i < 12; ++i) {
        uint64_t C = 0, s;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            s = (uint64_t)t[j] + (uint64_t)a[j] * b[i] + C;
            t[j] = (uint32_t)s;
            C = s >> 32;
        }
        s = (uint64_t)t[12] + C;
        t[12] = (uint32_t)s;
        t[13] = (uint32_t)(s >> 32);
        const uint32_t m = t[0] * 0xFFFCFFFDu;
        s = (uint64_t)t[0] + (uint64_t)m * kP[0];
        C = s >> 32;
#pragma unroll
        for (int j = 1; j < 12; ++j) {
            s = (uint64_t)t[j] + (uint64_t)m * kP[j] + C;
            t[j - 1] = (uint32_t)s;
            C = s >> 32;
        }
        s = (uint64_t)t[12] + C;
        t[11] = (uint32_t)s;
        t[12] = t[13] + (uint32_t)(s >> 32);
    }
    Fp r, u;
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < 12; ++j) r[j] = t[j];
#pragma unroll
    for (int j = 0; j < 12; ++j) u[j] = __builtin_subc(r[j], kP[j], br, &br);
    const bool sub = t[12] != 0 || br == 0;
#pragma unroll
    for (int j = 0; j < 12; ++j) r[j] = sub ? u[j] : r[j];
    return r;
}
#endif
#ifdef HBG_FP_VERIFY
__device__ unsigned long long g_fp_verify[2];  // [0] mismatches, [1] checks
__device__ uint32_t g_fp_verify_rec[64];       // site, lane, a[12], b[12], asm r[12], ref r[12]
__device__ __noinline__ void fp_verify(Fp a, Fp b, Fp r, int site) {
    const Fp ref = fp_mul_ref(a, b);
    uint32_t d = 0;
#pragma unroll
    for (int j = 0; j < 12; ++j) d |= ref[j] ^ r[j];
    atomicAdd(&g_fp_verify[1], 1ull);
    if (d && atomicAdd(&g_fp_verify[0], 1ull) == 0) {
        g_fp_verify_rec[0] = (uint32_t)site;
        g_fp_verify_rec[1] = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) +
                             64u * (blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u);
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            g_fp_verify_rec[2 + j] = a[j];
            g_fp_verify_rec[14 + j] = b[j];
            g_fp_verify_rec[26 + j] = r[j];
            g_fp_verify_rec[38 + j] = ref[j];
        }
    }
}
#define HBG_FP_VERIFY_INPUT(name, v) const Fp name = (v)
#define HBG_FP_VERIFY_CALL(a, b, r) fp_verify((a), (b), (r), __LINE__)
#else
#define HBG_FP_VERIFY_INPUT(name, v) ((void)0)
#define HBG_FP_VERIFY_CALL(a, b, r) ((void)0)
#endif

// Montgomery products through the fixed-register subroutines: the operands
// are bound to the subroutine's input VGPRs, results come back over the
// first operands, the temporaries are clobbers (the asm is not volatile, so
// identical products may be merged by the compiler).
BD Fp fp_mul(Fp a, Fp b) {
    HBG_FP_COUNT_CALL(0);
#ifdef HBG_FP_PORTABLE
    return fp_mul_ref(a, b);
#endif
    HBG_FP_VERIFY_INPUT(a_in, a);
    asm(HBG_FP_SUB_CALL("hbg_fpmul1") : "+{v[0:11]}"(a) : "{v[12:23]}"(b) : HBG_FP_SUB1_CLOBBERS);
    HBG_FP_VERIFY_CALL(a_in, b, a);
    return a;
}

BD Fp fp_sqr(Fp a) {
    HBG_FP_COUNT_CALL(1);
#ifdef HBG_FP_PORTABLE
    return fp_mul_ref(a, a);
#endif
    HBG_FP_VERIFY_INPUT(a_in, a);
    asm(HBG_FP_SUB_CALL("hbg_fpmul1") : "+{v[0:11]}"(a) : "{v[12:23]}"(a) : HBG_FP_SUB1_CLOBBERS);
    HBG_FP_VERIFY_CALL(a_in, a_in, a);
    return a;
}

// (a0 b0, a1 b1): two independent products in one interleaved call
BD void fp_mul2(Fp& r0, Fp& r1, Fp a0, Fp b0, Fp a1, Fp b1) {
    HBG_FP_COUNT_CALL(0);
    HBG_FP_COUNT_CALL(0);
#ifdef HBG_FP_PORTABLE
    r0 = fp_mul_ref(a0, b0);
    r1 = fp_mul_ref(a1, b1);
    return;
#endif
    HBG_FP_VERIFY_INPUT(x0, a0);
    HBG_FP_VERIFY_INPUT(x1, a1);
    asm(HBG_FP_SUB_CALL("hbg_fpmul2")
        : "+{v[0:11]}"(a0), "+{v[24:35]}"(a1)
        : "{v[12:23]}"(b0), "{v[36:47]}"(b1)
        : HBG_FP_SUB2_CLOBBERS);
    HBG_FP_VERIFY_CALL(x0, b0, a0);
    HBG_FP_VERIFY_CALL(x1, b1, a1);
    r0 = a0;
    r1 = a1;
}

// (a0 b0, a1 b1, a2 b2): three independent products, no wait states
BD void fp_mul3(Fp& r0, Fp& r1, Fp& r2, Fp a0, Fp b0, Fp a1, Fp b1, Fp a2, Fp b2) {
    HBG_FP_COUNT_CALL(0);
    HBG_FP_COUNT_CALL(0);
    HBG_FP_COUNT_CALL(0);
#ifdef HBG_FP_PORTABLE
    r0 = fp_mul_ref(a0, b0);
    r1 = fp_mul_ref(a1, b1);
    r2 = fp_mul_ref(a2, b2);
    return;
#endif
    HBG_FP_VERIFY_INPUT(x0, a0);
    HBG_FP_VERIFY_INPUT(x1, a1);
    HBG_FP_VERIFY_INPUT(x2, a2);
    asm(HBG_FP_SUB_CALL("hbg_fpmul3")
        : "+{v[0:11]}"(a0), "+{v[24:35]}"(a1), "+{v[48:59]}"(a2)
        : "{v[12:23]}"(b0), "{v[36:47]}"(b1), "{v[60:71]}"(b2)
        : HBG_FP_SUB3_CLOBBERS);
    HBG_FP_VERIFY_CALL(x0, b0, a0);
    HBG_FP_VERIFY_CALL(x1, b1, a1);
    HBG_FP_VERIFY_CALL(x2, b2, a2);
    r0 = a0;
    r1 = a1;
    r2 = a2;
}

BD Fp fp_add(const Fp& a, const Fp& b) {
    Fp r, u;
    uint32_t c = 0, br = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) r[i] = __builtin_addc(a[i], b[i], c, &c);
#pragma unroll
    for (int i = 0; i < 12; ++i) u[i] = __builtin_subc(r[i], kP[i], br, &br);
    // a + b < 2p < 2^382: no carry out of limb 11; r >= p <=> no borrow
#pragma unroll
    for (int i = 0; i < 12; ++i) r[i] = br ? r[i] : u[i];
    return r;
}

BD Fp fp_sub(const Fp& a, const Fp& b) {
    Fp r, u;
    uint32_t br = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) r[i] = __builtin_subc(a[i], b[i], br, &br);
#pragma unroll
    for (int i = 0; i < 12; ++i) u[i] = __builtin_addc(r[i], kP[i], c, &c);
#pragma unroll
    for (int i = 0; i < 12; ++i) r[i] = br ? u[i] : r[i];
    return r;
}

BD bool fp_is_zero(const Fp& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) o |= a[i];
    return o == 0;
}

BD bool fp_eq(const Fp& a, const Fp& b) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) o |= a[i] ^ b[i];
    return o == 0;
}

BD Fp fp_neg(const Fp& a) { return fp_sub(fp_zero(), a); }
BD Fp fp_dbl(const Fp& a) { return fp_add(a, a); }

BD Fp fp_select(bool c, const Fp& a, const Fp& b) {
    Fp r;
#pragma unroll
    for (int i = 0; i < 12; ++i) r[i] = c ? a[i] : b[i];
    return r;
}

// Montgomery <-> canonical
BD Fp fp_to_mont(const Fp& raw) { return fp_mul(raw, fp_const(kR2)); }
BD Fp fp_from_mont(const Fp& a) {
    Fp one = fp_zero();
    one[0] = 1u;
    return fp_mul(a, one);
}

// canonical a > canonical b (both Montgomery)
BD bool fp_gt(const Fp& a, const Fp& b) {
    const Fp x = fp_from_mont(a), y = fp_from_mont(b);
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) (void)__builtin_subc(y[i], x[i], br, &br);
    return br != 0;  // y - x borrows <=> x > y
}

// raw (canonical) limbs < p ?
BD bool fp_raw_lt_p(const Fp& a) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) (void)__builtin_subc(a[i], kP[i], br, &br);
    return br != 0;
}

// a^e for an exponent held in constant memory (nbits significant bits, top
// bit set).  Sliding window of 4 bits over the odd powers a, a^3, .., a^15:
// the exponent is wave-uniform, so every branch below is uniform; 8 table
// multiplications + ~nbits/5 window multiplications instead of ~nbits/2
// (Fermat inverse: 380 squarings + 83 multiplications instead of + 190).
BD Fp fp_pow(Fp a, const uint32_t* __restrict__ e, int nbits) {
    Fp tbl[8];
    tbl[0] = a;
    const Fp a2 = fp_sqr(a);
#pragma unroll 1
    for (int k = 1; k < 8; ++k) tbl[k] = fp_mul(tbl[k - 1], a2);
    auto bit = [&](int i) -> uint32_t { return (e[i >> 5] >> (i & 31)) & 1u; };
    Fp r = fp_one();  // squarings of one before the first window (a leading zero bit) stay one
    bool first = true;
    int i = nbits - 1;
#pragma unroll 1
    while (i >= 0) {
        if (!bit(i)) {
            r = fp_sqr(r);
            --i;
            continue;
        }
        int j = i - 3 > 0 ? i - 3 : 0;  // window [j, i] ending in a set bit
        while (!bit(j)) ++j;
        uint32_t v = 0;
        for (int k = i; k >= j; --k) v = (v << 1) | bit(k);
        if (first) {
            r = tbl[v >> 1];
            first = false;
        } else {
#pragma unroll 1
            for (int k = i; k >= j; --k) r = fp_sqr(r);
            r = fp_mul(r, tbl[v >> 1]);
        }
        i = j - 1;
    }
    return r;
}

__device__ __constant__ static const uint32_t gExpPm2[12] = {
    kExpPm2[0], kExpPm2[1], kExpPm2[2], kExpPm2[3], kExpPm2[4],  kExpPm2[5],
    kExpPm2[6], kExpPm2[7], kExpPm2[8], kExpPm2[9], kExpPm2[10], kExpPm2[11]};
__device__ __constant__ static const uint32_t gExpSqrt[12] = {
    kExpSqrt[0], kExpSqrt[1], kExpSqrt[2], kExpSqrt[3], kExpSqrt[4],  kExpSqrt[5],
    kExpSqrt[6], kExpSqrt[7], kExpSqrt[8], kExpSqrt[9], kExpSqrt[10], kExpSqrt[11]};
__device__ __constant__ static const uint32_t gExpPm3d4[12] = {
    kExpPm3d4[0], kExpPm3d4[1], kExpPm3d4[2], kExpPm3d4[3], kExpPm3d4[4],  kExpPm3d4[5],
    kExpPm3d4[6], kExpPm3d4[7], kExpPm3d4[8], kExpPm3d4[9], kExpPm3d4[10], kExpPm3d4[11]};
__device__ __constant__ static const uint32_t gExpPm1d2[12] = {
    kExpPm1d2[0], kExpPm1d2[1], kExpPm1d2[2], kExpPm1d2[3], kExpPm1d2[4],  kExpPm1d2[5],
    kExpPm1d2[6], kExpPm1d2[7], kExpPm1d2[8], kExpPm1d2[9], kExpPm1d2[10], kExpPm1d2[11]};

constexpr int kPBits = 381;

BD Fp fp_inv(const Fp& a) { return fp_pow(a, gExpPm2, kPBits); }

// sqrt for p = 3 mod 4; ok = a is a square
BD Fp fp_sqrt(const Fp& a, bool& ok) {
    const Fp s = fp_pow(a, gExpSqrt, 379);  // (p+1)/4 has 379 bits
    ok = fp_eq(fp_sqr(s), a);
    return s;
}

// big-endian bytes <-> raw limbs
BD Fp fp_from_be(const uint8_t* p) {
    Fp r;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const uint8_t* q = p + 44 - 4 * i;
        r[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
    return r;
}

BD void fp_to_be(uint8_t* p, const Fp& raw) {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        uint8_t* q = p + 44 - 4 * i;
        q[0] = (uint8_t)(raw[i] >> 24);
        q[1] = (uint8_t)(raw[i] >> 16);
        q[2] = (uint8_t)(raw[i] >> 8);
        q[3] = (uint8_t)raw[i];
    }
}

// ============================================================== Fp2 = Fp[u]/(u^2+1)
struct Fp2 {
    Fp c0, c1;
};

BD Fp2 fp2_zero() { return {fp_zero(), fp_zero()}; }
BD Fp2 fp2_one() { return {fp_one(), fp_zero()}; }
BD Fp2 fp2_add(const Fp2& a, const Fp2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
BD Fp2 fp2_sub(const Fp2& a, const Fp2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
BD Fp2 fp2_neg(const Fp2& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
BD Fp2 fp2_dbl(const Fp2& a) { return {fp_dbl(a.c0), fp_dbl(a.c1)}; }
BD Fp2 fp2_conj(const Fp2& a) { return {a.c0, fp_neg(a.c1)}; }
BD bool fp2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
BD bool fp2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
BD Fp2 fp2_select(bool c, const Fp2& a, const Fp2& b) { return {fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)}; }

// Karatsuba: the three products are independent -> one hbg_fpmul3 call
BD Fp2 fp2_mul(const Fp2& a, const Fp2& b) {
    Fp t0, t1, t2;
    fp_mul3(t0, t1, t2, a.c0, b.c0, a.c1, b.c1, fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
    return {fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

BD Fp2 fp2_sqr(const Fp2& a) {
    Fp t, u;
    fp_mul2(t, u, a.c0, a.c1, fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
    return {u, fp_dbl(t)};
}

BD Fp2 fp2_mul_fp(const Fp2& a, const Fp& s) {
    Fp r0, r1;
    fp_mul2(r0, r1, a.c0, s, a.c1, s);
    return {r0, r1};
}

// * (1 + u)
BD Fp2 fp2_mul_xi(const Fp2& a) { return {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

BD Fp2 fp2_mul_small(const Fp2& a, int k) {
    Fp2 r = a;
    for (int i = 1; i < k; ++i) r = fp2_add(r, a);
    return r;
}

BD Fp2 fp2_inv(const Fp2& a) {
    const Fp t = fp_inv(fp_add(fp_sqr(a.c0), fp_sqr(a.c1)));
    return {fp_mul(a.c0, t), fp_neg(fp_mul(a.c1, t))};
}

// canonical lexicographic a > b (the crate's Fq2 Ord: c1 first, then c0)
BD bool fp2_gt(const Fp2& a, const Fp2& b) {
    if (!fp_eq(a.c1, b.c1)) return fp_gt(a.c1, b.c1);
    return fp_gt(a.c0, b.c0);
}

BD void fp2_pow_inplace(Fp2* x, const uint32_t* __restrict__ e, int nbits) {
    const Fp2 a = *x;
    Fp2 r = a;
    for (int i = nbits - 2; i >= 0; --i) {
        r = fp2_sqr(r);
        if ((e[i >> 5] >> (i & 31)) & 1u) r = fp2_mul(r, a);
    }
    *x = r;
}

// Algorithm 9 of eprint 2012/685 (the crate's Fq2::sqrt); ok = square.
BD Fp2 fp2_sqrt(const Fp2& a, bool& ok) {
    ok = true;
    if (fp2_is_zero(a)) return a;
    Fp2 a1 = a;
    fp2_pow_inplace(&a1, gExpPm3d4, 379);
    const Fp2 alpha = fp2_mul(fp2_sqr(a1), a);
    const Fp2 a0 = fp2_mul(fp2_conj(alpha), alpha);
    const Fp2 mone = fp2_neg(fp2_one());
    if (fp2_eq(a0, mone)) {
        ok = false;
        return a;
    }
    a1 = fp2_mul(a1, a);
    if (fp2_eq(alpha, mone)) return {fp_neg(a1.c1), a1.c0};  // a1 * u
    Fp2 b = {fp_add(alpha.c0, fp_one()), alpha.c1};
    fp2_pow_inplace(&b, gExpPm1d2, 380);
    return fp2_mul(a1, b);
}

template <int N>
BD Fp2 fp2_const(const uint32_t (&c)[N]) {
    Fp2 r;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        r.c0[i] = c[i];
        r.c1[i] = c[12 + i];
    }
    return r;
}

// ============================================================== Fp6 = Fp2[v]/(v^3 - xi)
struct Fp6 {
    Fp2 c0, c1, c2;
};

BD Fp6 fp6_zero() { return {fp2_zero(), fp2_zero(), fp2_zero()}; }
BD Fp6 fp6_one() { return {fp2_one(), fp2_zero(), fp2_zero()}; }
BD Fp6 fp6_add(const Fp6& a, const Fp6& b) { return {fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
BD Fp6 fp6_sub(const Fp6& a, const Fp6& b) { return {fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
BD Fp6 fp6_neg(const Fp6& a) { return {fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
BD Fp6 fp6_mul_by_v(const Fp6& a) { return {fp2_mul_xi(a.c2), a.c0, a.c1}; }
BD bool fp6_eq(const Fp6& a, const Fp6& b) { return fp2_eq(a.c0, b.c0) && fp2_eq(a.c1, b.c1) && fp2_eq(a.c2, b.c2); }

BD Fp6 fp6_mul(const Fp6& a, const Fp6& b) {
    const Fp2 t0 = fp2_mul(a.c0, b.c0), t1 = fp2_mul(a.c1, b.c1), t2 = fp2_mul(a.c2, b.c2);
    Fp6 r;
    r.c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), fp2_add(t1, t2))));
    r.c1 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
    r.c2 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), fp2_add(t0, t2)), t1);
    return r;
}

// a * (b0 + b1 v)   (the crate's Fq6::mul_by_01)
BD Fp6 fp6_mul_by_01(const Fp6& a, const Fp2& b0, const Fp2& b1) {
    const Fp2 t0 = fp2_mul(a.c0, b0), t1 = fp2_mul(a.c1, b1);
    Fp6 r;
    r.c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), b1), t1)), t0);
    r.c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b0, b1)), t0), t1);
    r.c2 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), b0), t0), t1);
    return r;
}

// a * (b1 v)   (the crate's Fq6::mul_by_1)
BD Fp6 fp6_mul_by_1(const Fp6& a, const Fp2& b1) {
    return {fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

BD Fp6 fp6_inv(const Fp6& a) {
    const Fp2 c0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
    const Fp2 c1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
    const Fp2 c2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
    const Fp2 t = fp2_inv(fp2_add(fp2_mul(a.c0, c0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, c1), fp2_mul(a.c1, c2)))));
    return {fp2_mul(c0, t), fp2_mul(c1, t), fp2_mul(c2, t)};
}

template <int K>
BD Fp6 fp6_frob(const Fp6& a) {
    const Fp2 x0 = (K & 1) ? fp2_conj(a.c0) : a.c0;
    const Fp2 x1 = (K & 1) ? fp2_conj(a.c1) : a.c1;
    const Fp2 x2 = (K & 1) ? fp2_conj(a.c2) : a.c2;
    if constexpr (K == 1) return {x0, fp2_mul(x1, fp2_const(kFrob6c1_1)), fp2_mul(x2, fp2_const(kFrob6c2_1))};
    if constexpr (K == 2) return {x0, fp2_mul(x1, fp2_const(kFrob6c1_2)), fp2_mul(x2, fp2_const(kFrob6c2_2))};
    if constexpr (K == 3) return {x0, fp2_mul(x1, fp2_const(kFrob6c1_3)), fp2_mul(x2, fp2_const(kFrob6c2_3))};
    return a;
}

// ============================================================== Fp12 = Fp6[w]/(w^2 - v)
// Register-resident: every Fp12 operation below is inlined down to the
// fp_mul / fp_sqr calls, so its operands and temporaries live in registers
// (the pairing kernels run one wave per SIMD: 256 VGPRs + 256 AGPRs, and
// fp_mul clobbers only v0-v39).  Round 3's pointer-passing Fp6 / Fp12 call
// frames round-tripped 288-576 B operands through scratch on every call
// (295 KB of HBM traffic per verified share, profiles/r03al).  Pointers remain
// only at the final exponentiation's Fp12 level (final_exponentiation), where
// five values are live at once and one load / store per Fp12 operation is
// noise next to its 18-54 multiplications.
struct Fp12 {
    Fp6 c0, c1;
};

BD Fp12 fp12_one() { return {fp6_one(), fp6_zero()}; }
BD Fp12 fp12_conj(const Fp12& a) { return {a.c0, fp6_neg(a.c1)}; }
BD bool fp12_eq(const Fp12& a, const Fp12& b) { return fp6_eq(a.c0, b.c0) && fp6_eq(a.c1, b.c1); }
BD bool fp12_is_one(const Fp12& a) { return fp12_eq(a, fp12_one()); }
BD Fp12 fp12_select(bool c, const Fp12& a, const Fp12& b) {
    return {{fp2_select(c, a.c0.c0, b.c0.c0), fp2_select(c, a.c0.c1, b.c0.c1), fp2_select(c, a.c0.c2, b.c0.c2)},
            {fp2_select(c, a.c1.c0, b.c1.c0), fp2_select(c, a.c1.c1, b.c1.c1), fp2_select(c, a.c1.c2, b.c1.c2)}};
}

BD Fp12 fp12_mul_v(const Fp12& a, const Fp12& b) {
    const Fp6 t0 = fp6_mul(a.c0, b.c0);
    const Fp6 t1 = fp6_mul(a.c1, b.c1);
    const Fp6 t2 = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1));
    return {fp6_add(t0, fp6_mul_by_v(t1)), fp6_sub(t2, fp6_add(t0, t1))};
}

// the crate's Fq12::square (complex squaring, 2 Fq6 mults)
BD Fp12 fp12_sqr_v(const Fp12& a) {
    const Fp6 ab = fp6_mul(a.c0, a.c1);
    const Fp6 c0 = fp6_sub(fp6_mul(fp6_add(fp6_mul_by_v(a.c1), a.c0), fp6_add(a.c0, a.c1)), ab);
    return {fp6_sub(c0, fp6_mul_by_v(ab)), fp6_add(ab, ab)};
}

// f * (c0 + c1 v + c4 v w)   (the crate's Fq12::mul_by_014), in place
BD void fp12_mul_by_014_v(Fp12& f, const Fp2& c0, const Fp2& c1, const Fp2& c4) {
    const Fp6 t = fp6_mul_by_01(fp6_add(f.c1, f.c0), c0, fp2_add(c1, c4));
    const Fp6 aa = fp6_mul_by_01(f.c0, c0, c1);
    const Fp6 bb = fp6_mul_by_1(f.c1, c4);
    f.c1 = fp6_sub(fp6_sub(t, aa), bb);
    f.c0 = fp6_add(fp6_mul_by_v(bb), aa);
}

BD Fp12 fp12_inv_v(const Fp12& a) {
    const Fp6 t = fp6_inv(fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_by_v(fp6_mul(a.c1, a.c1))));
    return {fp6_mul(a.c0, t), fp6_neg(fp6_mul(a.c1, t))};
}

template <int K>
BD Fp12 fp12_frob_v(const Fp12& a) {
    const Fp6 c0 = fp6_frob<K>(a.c0), c1 = fp6_frob<K>(a.c1);
    Fp2 g;
    if constexpr (K == 1) g = fp2_const(kFrob12c1_1);
    if constexpr (K == 2) g = fp2_const(kFrob12c1_2);
    if constexpr (K == 3) g = fp2_const(kFrob12c1_3);
    return {c0, {fp2_mul(c1.c0, g), fp2_mul(c1.c1, g), fp2_mul(c1.c2, g)}};
}

// Granger-Scott cyclotomic squaring (valid after the easy part of the final
// exponentiation: same values as plain squaring there).
BD void fp4_sqr(Fp2& r0, Fp2& r1, const Fp2& a, const Fp2& b) {
    const Fp2 t0 = fp2_sqr(a), t1 = fp2_sqr(b);
    r0 = fp2_add(fp2_mul_xi(t1), t0);
    r1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(a, b)), t0), t1);
}

BD Fp12 fp12_cyclotomic_sqr_v(const Fp12& f) {
    // z0..z5 = c0.c0, c1.c1, c1.c0, c0.c2, c0.c1, c1.c2
    Fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
    Fp2 t0, t1, t2, t3;
    fp4_sqr(t0, t1, z0, z1);
    z0 = fp2_add(fp2_dbl(fp2_sub(t0, z0)), t0);
    z1 = fp2_add(fp2_dbl(fp2_add(t1, z1)), t1);
    fp4_sqr(t0, t1, z2, z3);
    fp4_sqr(t2, t3, z4, z5);
    z4 = fp2_add(fp2_dbl(fp2_sub(t0, z4)), t0);
    z5 = fp2_add(fp2_dbl(fp2_add(t1, z5)), t1);
    t0 = fp2_mul_xi(t3);
    z2 = fp2_add(fp2_dbl(fp2_add(t0, z2)), t0);
    z3 = fp2_add(fp2_dbl(fp2_sub(t2, z3)), t2);
    return {{z0, z4, z3}, {z2, z1, z5}};
}

// Final-exponentiation steps: one Fp12 load / store at the call boundary, the
// body register-resident.
__device__ __noinline__ void fp12_mul_n(Fp12* r, const Fp12* a, const Fp12* b) { *r = fp12_mul_v(*a, *b); }
__device__ __noinline__ void fp12_inv_n(Fp12* r, const Fp12* a) { *r = fp12_inv_v(*a); }
template <int K>
__device__ __noinline__ void fp12_frob_n(Fp12* r, const Fp12* a) { *r = fp12_frob_v<K>(*a); }
__device__ __noinline__ void fp12_cyc_sqr_n(Fp12* r, const Fp12* a) { *r = fp12_cyclotomic_sqr_v(*a); }

// *f = conj(f^e) for a 64-bit e with top set bit `top` (cyclotomic squarings);
// with e = |x| this is the crate's exp_by_x (x < 0).  Square-and-multiply
// split into runs: the inner loop squares down to the next set bit with only
// the accumulator live (|x| has 5 set bits below its top, so the base is
// touched 5 times in 63 steps and waits outside the loop).
__device__ __noinline__ void fp12_cyc_pow_conj(Fp12* f, uint64_t e, int top) {
    const Fp12 a = *f;
    Fp12 r = a;
    uint64_t rem = e & ((1ull << top) - 1ull);
    int i = top - 1;
#pragma unroll 1
    for (;;) {
        const int nb = rem ? 63 - __builtin_clzll(rem) : -1;  // next set bit (wave-uniform)
#pragma unroll 1
        for (; i >= (nb < 0 ? 0 : nb); --i) r = fp12_cyclotomic_sqr_v(r);
        if (nb < 0) break;
        r = fp12_mul_v(r, a);
        rem &= ~(1ull << nb);
    }
    *f = fp12_conj(r);
}

BD void fp12_exp_by_x_inplace(Fp12* f) { fp12_cyc_pow_conj(f, kBlsX, 63); }

// ============================================================== curves
struct G1 {  // Jacobian; infinity <=> Z == 0
    Fp x, y, z;
};
struct G1A {
    Fp x, y;
    bool inf;
};
struct G2 {
    Fp2 x, y, z;
};
struct G2A {
    Fp2 x, y;
    bool inf;
};

// ---- G1 (y^2 = x^3 + 4), dbl-2009-l / add-2007-bl (a = 0)
// Independent products go through one fp_mul2 / fp_mul3 call (interleaved
// chains: a lone wave stalls less than on single products, bls_fp_sub.h).
BD G1 g1_dbl(const G1& p) {
    Fp A, B, C, T, F, YZ;
    fp_mul2(A, B, p.x, p.x, p.y, p.y);
    const Fp xb = fp_add(p.x, B);
    fp_mul2(C, T, B, B, xb, xb);
    const Fp D = fp_dbl(fp_sub(fp_sub(T, A), C));
    const Fp E = fp_add(fp_dbl(A), A);
    fp_mul2(F, YZ, E, E, p.y, p.z);
    G1 r;
    r.x = fp_sub(F, fp_dbl(D));
    r.y = fp_sub(fp_mul(E, fp_sub(D, r.x)), fp_dbl(fp_dbl(fp_dbl(C))));
    r.z = fp_dbl(YZ);
    return r;
}

// p + q with q affine (not infinity)
BD G1 g1_add_mixed(const G1& p, const Fp& qx, const Fp& qy) {
    if (fp_is_zero(p.z)) return {qx, qy, fp_one()};
    Fp Z1Z1, YZ, U2, S2;
    fp_mul2(Z1Z1, YZ, p.z, p.z, qy, p.z);
    fp_mul2(U2, S2, qx, Z1Z1, YZ, Z1Z1);
    const Fp H = fp_sub(U2, p.x);
    const Fp rr = fp_dbl(fp_sub(S2, p.y));
    if (fp_is_zero(H)) {
        if (fp_is_zero(rr)) return g1_dbl(p);
        return {fp_one(), fp_one(), fp_zero()};
    }
    Fp HH, RR, ZH;
    const Fp zh = fp_add(p.z, H);
    fp_mul3(HH, RR, ZH, H, H, rr, rr, zh, zh);
    const Fp I = fp_dbl(fp_dbl(HH));
    Fp J, V;
    fp_mul2(J, V, H, I, p.x, I);
    G1 r;
    r.x = fp_sub(fp_sub(RR, J), fp_dbl(V));
    Fp a, b;
    fp_mul2(a, b, rr, fp_sub(V, r.x), p.y, J);
    r.y = fp_sub(a, fp_dbl(b));
    r.z = fp_sub(fp_sub(ZH, Z1Z1), HH);
    return r;
}

BD G1 g1_add(const G1& p, const G1& q) {
    if (fp_is_zero(p.z)) return q;
    if (fp_is_zero(q.z)) return p;
    Fp Z1Z1, Z2Z2, Y1Z2, Y2Z1, U1, U2, S1, S2;
    fp_mul2(Z1Z1, Z2Z2, p.z, p.z, q.z, q.z);
    fp_mul2(Y1Z2, Y2Z1, p.y, q.z, q.y, p.z);
    fp_mul2(U1, U2, p.x, Z2Z2, q.x, Z1Z1);
    fp_mul2(S1, S2, Y1Z2, Z2Z2, Y2Z1, Z1Z1);
    const Fp H = fp_sub(U2, U1);
    const Fp rr = fp_dbl(fp_sub(S2, S1));
    if (fp_is_zero(H)) {
        if (fp_is_zero(rr)) return g1_dbl(p);
        return {fp_one(), fp_one(), fp_zero()};
    }
    Fp I, RR, ZZ;
    const Fp h2 = fp_dbl(H), zz = fp_add(p.z, q.z);
    fp_mul3(I, RR, ZZ, h2, h2, rr, rr, zz, zz);
    Fp J, V;
    fp_mul2(J, V, H, I, U1, I);
    G1 r;
    r.x = fp_sub(fp_sub(RR, J), fp_dbl(V));
    Fp a, b, c;
    fp_mul3(a, b, c, rr, fp_sub(V, r.x), S1, J, fp_sub(fp_sub(ZZ, Z1Z1), Z2Z2), H);
    r.y = fp_sub(a, fp_dbl(b));
    r.z = c;
    return r;
}

BD G1A g1_to_affine(const G1& p) {
    if (fp_is_zero(p.z)) return {fp_zero(), fp_zero(), true};
    const Fp zi = fp_inv(p.z), zi2 = fp_sqr(zi);
    return {fp_mul(p.x, zi2), fp_mul(p.y, fp_mul(zi2, zi)), false};
}

BD bool g1_on_curve(const Fp& x, const Fp& y) {
    return fp_eq(fp_sqr(y), fp_add(fp_mul(fp_sqr(x), x), fp_const(kFour)));
}

// [k]P for a 64-bit scalar (left to right), P affine
BD G1 g1_mul_u64(const Fp& px, const Fp& py, uint64_t k) {
    G1 r = {fp_one(), fp_one(), fp_zero()};
    for (int i = 63; i >= 0; --i) {
        r = g1_dbl(r);
        if ((k >> i) & 1ull) r = g1_add_mixed(r, px, py);
    }
    return r;
}

// [k]P for a 64-bit scalar, P Jacobian (X, Y, Z), Z != 0, k > 0: on the
// isomorphic curve y^2 = x^3 + 4 Z^6 ((x, y) -> (x Z^2, y Z^3); the a = 0
// formulas never read the constant) P is the affine (X, Y) — mixed additions
// — and the result (X', Y', Z') maps back as (X', Y', Z' Z)
BD G1 g1_mul_u64_jac(const G1& p, uint64_t k) {
    const G1 r = g1_mul_u64(p.x, p.y, k);
    return {r.x, r.y, fp_mul(r.z, p.z)};
}

// P in G1  <=>  phi(P) == [-x^2] P,  phi(x, y) = (beta x, y)   (Bowe, eprint 2019/814).
// [x^2]P = [|x|]([|x|]P) stays Jacobian (X, Y, Z); the comparison with the
// affine phi(P) is cross-multiplied (beta x Z^2 == X, y Z^3 == -Y), so no
// field inversion is spent (two ~380-squaring exponentiations saved per point).
BD bool g1_in_subgroup(const Fp& px, const Fp& py) {
    const G1 t = g1_mul_u64(px, py, kBlsX);
    if (fp_is_zero(t.z)) return false;
    const G1 u = g1_mul_u64_jac(t, kBlsX);
    if (fp_is_zero(u.z)) return false;
    const Fp z2 = fp_sqr(u.z), z3 = fp_mul(z2, u.z);
    return fp_eq(fp_mul(fp_mul(px, fp_const(kBeta)), z2), u.x) && fp_eq(fp_mul(py, z3), fp_neg(u.y));
}

// zcash compressed G1 -> affine (Montgomery).  status: 0 ok, else invalid.
BD bool g1_decompress(const uint8_t* b, G1A& out, bool check_subgroup) {
    const uint8_t f = b[0];
    out.x = fp_zero();  // defined on every path (an undefined output lets the
    out.y = fp_zero();  // optimiser drop the early-reject branches)
    out.inf = false;
    if (!(f & 0x80)) return false;
    if (f & 0x40) {  // infinity: everything else must be zero
        bool z = (f & 0x3F) == 0;
        for (int i = 1; i < 48; ++i) z &= b[i] == 0;
        out.inf = true;
        out.x = fp_zero();
        out.y = fp_zero();
        return z;
    }
    Fp raw = fp_from_be(b);
    raw[11] &= 0x1FFFFFFFu;
    if (!fp_raw_lt_p(raw)) return false;
    const Fp x = fp_to_mont(raw);
    bool ok;
    Fp y = fp_sqrt(fp_add(fp_mul(fp_sqr(x), x), fp_const(kFour)), ok);
    if (!ok) return false;
    const Fp ny = fp_neg(y);
    const bool want_greatest = (f & 0x20) != 0;
    const bool y_greatest = fp_gt(y, ny);
    out.x = x;
    out.y = (y_greatest == want_greatest) ? y : ny;
    if (check_subgroup && !g1_in_subgroup(out.x, out.y)) return false;
    return true;
}

BD void g1_compress(uint8_t* b, const G1A& p) {
    if (p.inf) {
        b[0] = 0xC0;
        for (int i = 1; i < 48; ++i) b[i] = 0;
        return;
    }
    fp_to_be(b, fp_from_mont(p.x));
    b[0] |= 0x80;
    if (fp_gt(p.y, fp_neg(p.y))) b[0] |= 0x20;
}

// ---- G2 (y^2 = x^3 + 4(u+1)), Jacobian
BD G2 g2_dbl_v(const G2& p) {
    const Fp2 A = fp2_sqr(p.x), B = fp2_sqr(p.y), C = fp2_sqr(B);
    const Fp2 D = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.x, B)), A), C));
    const Fp2 E = fp2_add(fp2_dbl(A), A);
    const Fp2 F = fp2_sqr(E);
    G2 r;
    r.x = fp2_sub(F, fp2_dbl(D));
    r.y = fp2_sub(fp2_mul(E, fp2_sub(D, r.x)), fp2_dbl(fp2_dbl(fp2_dbl(C))));
    r.z = fp2_dbl(fp2_mul(p.y, p.z));
    return r;
}

// G2 point steps stay out of line (one call per step of a scalar
// multiplication / G2Prepared: keeps the G2 kernels' code and compile time
// bounded).  Only one-wave-per-SIMD kernels call them (TDEC_WAVE1_KERNEL), so
// every caller shares their 512-register budget.  (-DHBG_G2_STEP_INLINE: tool
// builds of tools/ctw_probe.py only, the steps inlined into the kernel.)
#ifdef HBG_G2_STEP_INLINE
#define HBG_G2_STEP BD
#else
#define HBG_G2_STEP __device__ __noinline__
#endif
// (per-function variants of the same tool switch: _DBL, _ADD, _PREP)
#if defined(HBG_G2_STEP_INLINE) || defined(HBG_G2_STEP_INLINE_DBL)
#define HBG_G2_STEP_DBL BD
#else
#define HBG_G2_STEP_DBL __device__ __noinline__
#endif
#if defined(HBG_G2_STEP_INLINE) || defined(HBG_G2_STEP_INLINE_ADD)
#define HBG_G2_STEP_ADD BD
#else
#define HBG_G2_STEP_ADD __device__ __noinline__
#endif
#if defined(HBG_G2_STEP_INLINE) || defined(HBG_G2_STEP_INLINE_PREP)
#define HBG_G2_STEP_PREP BD
#else
#define HBG_G2_STEP_PREP __device__ __noinline__
#endif
HBG_G2_STEP_DBL void g2_dbl_p(G2* r, const G2* p) { *r = g2_dbl_v(*p); }
BD G2 g2_dbl(const G2& p) {
    G2 r;
    g2_dbl_p(&r, &p);
    return r;
}

BD G2 g2_add_mixed_v(const G2& p, const Fp2& qx, const Fp2& qy) {
    if (fp2_is_zero(p.z)) return {qx, qy, fp2_one()};
    const Fp2 Z1Z1 = fp2_sqr(p.z);
    const Fp2 U2 = fp2_mul(qx, Z1Z1);
    const Fp2 S2 = fp2_mul(fp2_mul(qy, p.z), Z1Z1);
    const Fp2 H = fp2_sub(U2, p.x);
    const Fp2 rr = fp2_dbl(fp2_sub(S2, p.y));
    if (fp2_is_zero(H)) {
        if (fp2_is_zero(rr)) return g2_dbl(p);
        return {fp2_one(), fp2_one(), fp2_zero()};
    }
    const Fp2 HH = fp2_sqr(H);
    const Fp2 I = fp2_dbl(fp2_dbl(HH));
    const Fp2 J = fp2_mul(H, I);
    const Fp2 V = fp2_mul(p.x, I);
    G2 r;
    r.x = fp2_sub(fp2_sub(fp2_sqr(rr), J), fp2_dbl(V));
    r.y = fp2_sub(fp2_mul(rr, fp2_sub(V, r.x)), fp2_dbl(fp2_mul(p.y, J)));
    r.z = fp2_sub(fp2_sub(fp2_sqr(fp2_add(p.z, H)), Z1Z1), HH);
    return r;
}

HBG_G2_STEP_ADD void g2_add_mixed_p(G2* r, const G2* p, const Fp2* qx, const Fp2* qy) {
    *r = g2_add_mixed_v(*p, *qx, *qy);
}
BD G2 g2_add_mixed(const G2& p, const Fp2& qx, const Fp2& qy) {
    G2 r;
    g2_add_mixed_p(&r, &p, &qx, &qy);
    return r;
}

BD G2A g2_to_affine(const G2& p) {
    if (fp2_is_zero(p.z)) return {fp2_zero(), fp2_zero(), true};
    const Fp2 zi = fp2_inv(p.z), zi2 = fp2_sqr(zi);
    return {fp2_mul(p.x, zi2), fp2_mul(p.y, fp2_mul(zi2, zi)), false};
}

BD bool g2_on_curve(const Fp2& x, const Fp2& y) {
    const Fp2 b = {fp_const(kB2), fp_const(kB2)};
    return fp2_eq(fp2_sqr(y), fp2_add(fp2_mul(fp2_sqr(x), x), b));
}

BD G2 g2_mul_u64(const Fp2& px, const Fp2& py, uint64_t k) {
    G2 r = {fp2_one(), fp2_one(), fp2_zero()};
    for (int i = 63; i >= 0; --i) {
        r = g2_dbl(r);
        if ((k >> i) & 1ull) r = g2_add_mixed(r, px, py);
    }
    return r;
}

// Q in G2  <=>  psi(Q) == [x] Q   (Scott, eprint 2021/1130)
BD bool g2_in_subgroup(const Fp2& qx, const Fp2& qy) {
    const G2 t = g2_mul_u64(qx, qy, kBlsX);  // [|x|]Q, Jacobian
    if (fp2_is_zero(t.z)) return false;
    const Fp2 psx = fp2_mul(fp2_conj(qx), fp2_const(kPsiX));
    const Fp2 psy = fp2_mul(fp2_conj(qy), fp2_const(kPsiY));
    // psi(Q) == [x]Q = -[|x|]Q, cross-multiplied by Z^2 / Z^3 (no inversion)
    const Fp2 z2 = fp2_sqr(t.z), z3 = fp2_mul(z2, t.z);
    return fp2_eq(fp2_mul(psx, z2), t.x) && fp2_eq(fp2_mul(psy, z3), fp2_neg(t.y));
}

BD bool g2_decompress(const uint8_t* b, G2A& out, bool check_subgroup) {
    const uint8_t f = b[0];
    out.x = fp2_zero();
    out.y = fp2_zero();
    out.inf = false;
    if (!(f & 0x80)) return false;
    if (f & 0x40) {
        bool z = (f & 0x3F) == 0;
        for (int i = 1; i < 96; ++i) z &= b[i] == 0;
        out.inf = true;
        out.x = fp2_zero();
        out.y = fp2_zero();
        return z;
    }
    Fp r1 = fp_from_be(b), r0 = fp_from_be(b + 48);
    r1[11] &= 0x1FFFFFFFu;
    if (!fp_raw_lt_p(r1) || !fp_raw_lt_p(r0)) return false;
    const Fp2 x = {fp_to_mont(r0), fp_to_mont(r1)};
    const Fp2 b2 = {fp_const(kB2), fp_const(kB2)};
    bool ok;
    const Fp2 y = fp2_sqrt(fp2_add(fp2_mul(fp2_sqr(x), x), b2), ok);
    if (!ok) return false;
    const Fp2 ny = fp2_neg(y);
    const bool want = (f & 0x20) != 0;
    out.x = x;
    out.y = (fp2_gt(y, ny) == want) ? y : ny;
    if (check_subgroup && !g2_in_subgroup(out.x, out.y)) return false;
    return true;
}

// ============================================================== pairing pieces
struct LineCoeff {
    Fp2 c0, c1, c2;
};

// G2Prepared doubling step (Algorithm 26, eprint 2010/354; the crate's form)
BD LineCoeff g2_doubling_step_v(G2& r) {
    Fp2 tmp0 = fp2_sqr(r.x);
    Fp2 tmp1 = fp2_sqr(r.y);
    Fp2 tmp2 = fp2_sqr(tmp1);
    Fp2 tmp3 = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(tmp1, r.x)), tmp0), tmp2));
    const Fp2 tmp4 = fp2_add(fp2_dbl(tmp0), tmp0);
    Fp2 tmp6 = fp2_add(r.x, tmp4);
    const Fp2 tmp5 = fp2_sqr(tmp4);
    const Fp2 zsq = fp2_sqr(r.z);
    r.x = fp2_sub(fp2_sub(tmp5, tmp3), tmp3);
    r.z = fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.z, r.y)), tmp1), zsq);
    r.y = fp2_mul(fp2_sub(tmp3, r.x), tmp4);
    tmp2 = fp2_dbl(fp2_dbl(fp2_dbl(tmp2)));
    r.y = fp2_sub(r.y, tmp2);
    tmp3 = fp2_neg(fp2_dbl(fp2_mul(tmp4, zsq)));
    tmp6 = fp2_sub(fp2_sub(fp2_sqr(tmp6), tmp0), tmp5);
    tmp1 = fp2_dbl(fp2_dbl(tmp1));
    tmp6 = fp2_sub(tmp6, tmp1);
    tmp0 = fp2_dbl(fp2_mul(r.z, zsq));
    return {tmp0, tmp3, tmp6};
}

// G2Prepared addition step (Algorithm 27)
HBG_G2_STEP_PREP void g2_doubling_step_p(G2* r, LineCoeff* c) { *c = g2_doubling_step_v(*r); }
BD LineCoeff g2_doubling_step(G2& r) {
    LineCoeff c;
    g2_doubling_step_p(&r, &c);
    return c;
}

BD LineCoeff g2_addition_step_v(G2& r, const Fp2& qx, const Fp2& qy) {
    const Fp2 zsq = fp2_sqr(r.z);
    const Fp2 ysq = fp2_sqr(qy);
    const Fp2 t0 = fp2_mul(zsq, qx);
    const Fp2 t1 = fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(qy, r.z)), ysq), zsq), zsq);
    const Fp2 t2 = fp2_sub(t0, r.x);
    const Fp2 t3 = fp2_sqr(t2);
    const Fp2 t4 = fp2_dbl(fp2_dbl(t3));
    const Fp2 t5 = fp2_mul(t4, t2);
    Fp2 t6 = fp2_sub(fp2_sub(t1, r.y), r.y);
    Fp2 t9 = fp2_mul(t6, qx);
    const Fp2 t7 = fp2_mul(t4, r.x);
    r.x = fp2_sub(fp2_sub(fp2_sub(fp2_sqr(t6), t5), t7), t7);
    r.z = fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.z, t2)), zsq), t3);
    Fp2 t10 = fp2_add(qy, r.z);
    const Fp2 t8 = fp2_mul(fp2_sub(t7, r.x), t6);
    const Fp2 tt0 = fp2_dbl(fp2_mul(r.y, t5));
    r.y = fp2_sub(t8, tt0);
    t10 = fp2_sub(fp2_sqr(t10), ysq);
    const Fp2 ztsq = fp2_sqr(r.z);
    t10 = fp2_sub(t10, ztsq);
    t9 = fp2_sub(fp2_dbl(t9), t10);
    t10 = fp2_dbl(r.z);
    t6 = fp2_neg(t6);
    const Fp2 tt1 = fp2_dbl(t6);
    return {t10, tt1, t9};
}

HBG_G2_STEP_PREP void g2_addition_step_p(G2* r, LineCoeff* c, const Fp2* qx, const Fp2* qy) {
    *c = g2_addition_step_v(*r, *qx, *qy);
}
BD LineCoeff g2_addition_step(G2& r, const Fp2& qx, const Fp2& qy) {
    LineCoeff c;
    g2_addition_step_p(&r, &c, &qx, &qy);
    return c;
}

// number of line coefficients in a G2Prepared: 63 doublings after the leading
// bit of |x|>>1 ... (bits of |x|>>1 below its top bit) + additions + final doubling
constexpr int kMillerSteps = 68;

// ell(f, coeffs, p) of the crate, in place: the line evaluated at affine
// P = (px, py) times the sparse Fp12 (c2, c1 px, c0 py) -> mul_by_014
BD void ell(Fp12& f, const LineCoeff& c, const Fp& px, const Fp& py) {
    fp12_mul_by_014_v(f, c.c2, fp2_mul_fp(c.c1, px), fp2_mul_fp(c.c0, py));
}

// the crate's final_exponentiation, in place
__device__ __noinline__ void final_exponentiation(Fp12* io) {
    Fp12 r, f2, y0, y1, y2, y3;
    fp12_inv_n(&f2, io);
    y3 = fp12_conj(*io);
    fp12_mul_n(&r, &y3, &f2);
    f2 = r;
    fp12_frob_n<2>(&r, &r);
    fp12_mul_n(&r, &r, &f2);
    fp12_cyc_sqr_n(&y0, &r);
    y1 = y0;
    fp12_exp_by_x_inplace(&y1);
    y2 = y1;
    fp12_cyc_pow_conj(&y2, kBlsX >> 1, 62);  // conj(y1^(|x|>>1))
    y3 = fp12_conj(r);
    fp12_mul_n(&y1, &y1, &y3);
    y1 = fp12_conj(y1);
    fp12_mul_n(&y1, &y1, &y2);
    y2 = y1;
    fp12_exp_by_x_inplace(&y2);
    y3 = y2;
    fp12_exp_by_x_inplace(&y3);
    y1 = fp12_conj(y1);
    fp12_mul_n(&y3, &y3, &y1);
    y1 = fp12_conj(y1);
    fp12_frob_n<3>(&y1, &y1);
    fp12_frob_n<2>(&y2, &y2);
    fp12_mul_n(&y1, &y1, &y2);
    y2 = y3;
    fp12_exp_by_x_inplace(&y2);
    fp12_mul_n(&y2, &y2, &y0);
    fp12_mul_n(&y2, &y2, &r);
    fp12_mul_n(&y1, &y1, &y2);
    fp12_frob_n<1>(&y2, &y3);
    fp12_mul_n(io, &y1, &y2);
}

#undef BD

}  // namespace bls
}  // namespace hbg
