// rbc_kernels.hip — gfx950 kernels for hbbft's reliable-broadcast coding path.
//
// Families:
//   1. GF(2^8) coding    rs_encode_const<D,Q>  (a2+a3: Coding::encode, optionally
//                        fused with send_shards' length-prefix/pad/chunk), rs_code_generic
//                        (any matrix: encode for other (D,Q), reconstruct), rs_plan
//                        (a7: first-D-present inverse per instance)
//   2. Keccak/Merkle     merkle_build (a4: MerkleTree::from_vec, levels + root),
//                        merkle_validate (a6: Proof::validate)
//   glue                 rbc_glue_status / rbc_glue_copy (a8: glue_shards + root check),
//                        synth_bytes (seeded inputs)
//
// Device layout: instance k, shard i at
//   shards + (k*N + i)*S,  S % 16 == 0,  L meaningful bytes, [L, S) scratch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <utility>

#include "gf256.h"
#include "keccak.h"
#include "keccak_asm.h"
#include "rbc_kernels.h"

namespace hbg {

// ============================================================== family 1: coding
// Value byte x of an instance (send_shards' buffer): BE u32 length || payload || zeros.
__device__ __forceinline__ uint32_t value_byte(const uint8_t* __restrict__ pay, uint64_t P, uint64_t x) {
    if (x < 4) return (uint32_t)((P >> (8 * (3 - x))) & 0xFF);
    return (x - 4 < P) ? pay[x - 4] : 0u;
}

// 4 value bytes [v, v+4) packed little-endian.  `pay` is 4-byte aligned and
// any 32-bit word holding a byte < P is readable.
__device__ __forceinline__ uint32_t value_word(const uint8_t* __restrict__ pay, uint64_t P, uint64_t v) {
    if (v >= 4 && v + 4 <= P + 4) {
        const uint64_t o = v - 4;
        const uint32_t* w = reinterpret_cast<const uint32_t*>(pay) + (o >> 2);
        const uint32_t s = (uint32_t)(o & 3);
        const uint32_t w0 = w[0];
        const uint32_t w1 = s ? w[1] : 0u;
        return __builtin_amdgcn_alignbyte(w1, w0, s);
    }
    if (v >= P + 4) return 0u;
    return value_byte(pay, P, v) | (value_byte(pay, P, v + 1) << 8) | (value_byte(pay, P, v + 2) << 16) |
           (value_byte(pay, P, v + 3) << 24);
}

template <int D, int Q, int J, int... K>
__device__ __forceinline__ void mac_column(uint32_t (&acc)[Q], const NibPair& T, std::integer_sequence<int, K...>) {
    ((acc[K] = nib_mac<kParity<D, Q>.m[K][J]>(acc[K], T)), ...);
}

// Data words: MODE 0 rows already in place (Coding::encode); 1 from the
// payload, edge-checked (send_shards' prefix, padding, last partial word);
// 2 from the payload, interior block — every row's word lies inside the
// payload, so the address is a wave-uniform row base + p and the byte shift
// (J*L mod 4) is uniform: one dwordx2 load + v_alignbyte per word, no
// per-lane branches.  Loads run kPrefetch columns ahead of the arithmetic.
// 3 as 2 with the D windows loaded by the caller ahead of time (the fused
// kernel issues a pass's loads during the previous pass's Keccak work).
typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));
#ifndef HBG_ENC_PREFETCH
#define HBG_ENC_PREFETCH 6
#endif
constexpr int kPrefetch = HBG_ENC_PREFETCH;

// Raw buffer resource over [p, p + 2^31): loads/stores through it take the
// uniform row offset in an SGPR (soffset) and the lane's offset in a VGPR, so
// the encoder keeps no per-row 64-bit VGPR address.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7FFFFFFF, 0x00020000);
}
constexpr int kBufSc1 = 16;  // buffer aux bit: sc1 (served by L2, not the CU's vector L1)
// Cache policy of the encode / decode kernels' row, payload and level stores
// (buffer aux: 2 = nt, streamed past L2 so they do not evict the rows the
// absorb re-reads; 0 = default).
#ifndef HBG_STORE_AUX
#define HBG_STORE_AUX 2
#endif
constexpr int kStoreAux = HBG_STORE_AUX;
// ... and of the standalone encoders (rs_encode_const, rs_encode_missing):
// nothing re-reads their rows in the same kernel, and the default policy
// writes faster there (configs[1] rs_encode_const + merkle_build 2.60 ->
// 2.43 ms, hbg_rs_encode 0.44 -> 0.35 ms, 8,192 x N = 64 two-launch 28.9 ->
// 27.8 ms; the fused encoder with default-policy stores 26.6 -> 27.0 ms, so
// it keeps nt: gpurun_out r06k4)
#ifndef HBG_STORE_AUX_STANDALONE
#define HBG_STORE_AUX_STANDALONE 0
#endif
constexpr int kStoreAuxStandalone = HBG_STORE_AUX_STANDALONE;

// The rows of one encode: shard rows through `sh` (row J of the instance at
// byte J*S + vsh of the resource; vsh = the lane's instance offset + 4t) and
// the payload through `py` (value byte v of the instance at byte v - 4 +
// vpy).  p0 (wave-uniform) + t is the column: its 4 bytes at 4(p0 + t).
struct EncodeRows {
    __amdgpu_buffer_rsrc_t sh, py;
    uint32_t vsh, vpy;
    uint64_t S, L;
    uint32_t p0, t;
    uint8_t* __restrict__ base;       // MODE 1 only: this lane's instance rows
    const uint8_t* __restrict__ pay;  // MODE 1 only: this lane's payload
    uint64_t P;
    const u32x2_a4* pre;              // MODE 3 only: the D payload windows, loaded ahead (payload_window)
    uint32_t* ring;                   // RING only: parity row 0's word of this lane's column in the LDS ring
    uint32_t rdw;                     // RING only: dwords between consecutive parity rows of the ring
    uint64_t miss0, miss1;            // MASKED only: bit k = parity row k is missing (stored), wave-uniform
};

// MODE 2's payload window of data row J at column p0 + t (8 bytes at the
// 4-aligned payload byte below value byte J*L + 4p): a buffer load.
template <int J>
__device__ __forceinline__ u32x2_a4 payload_window(const EncodeRows& r, uint32_t p0) {
    const uint32_t so = (uint32_t)(((uint64_t)J * r.L + 4 * (uint64_t)p0 - 4) & ~3ull);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r.py, r.vpy, so, 0);
    return u32x2_a4{v[0], v[1]};
}

template <int D, int Q, int MODE, int AUX>
struct EncodeCtx {
    const EncodeRows& r;
    u32x2_a4 buf[kPrefetch];

    template <int J>
    __device__ __forceinline__ void fetch() {
        if constexpr (J < D) {
            if constexpr (MODE == 2) {
                // payload byte of value byte J*L + 4p, rounded down to 4 (the
                // byte shift J*L mod 4 is uniform)
                buf[J % kPrefetch] = payload_window<J>(r, r.p0);
            } else if constexpr (MODE == 0) {
                buf[J % kPrefetch].x =
                    __builtin_amdgcn_raw_buffer_load_b32(r.sh, r.vsh, (uint32_t)((uint64_t)J * r.S + 4 * r.p0), 0);
            }
        }
    }

    template <int J>
    __device__ __forceinline__ uint32_t word() {
        uint32_t w;
        if constexpr (MODE == 2 || MODE == 3) {
            const uint32_t sh = (uint32_t)(((uint64_t)J * r.L) & 3);
            const u32x2_a4 b = MODE == 2 ? buf[J % kPrefetch] : r.pre[J];
            w = __builtin_amdgcn_alignbyte(b.y, b.x, sh);
        } else if constexpr (MODE == 1) {
            w = value_word(r.pay, r.P, (uint64_t)J * r.L + 4 * ((uint64_t)r.p0 + r.t));
        } else {
            w = buf[J % kPrefetch].x;
        }
        if constexpr (MODE != 0)
            __builtin_amdgcn_raw_buffer_store_b32(w, r.sh, r.vsh, (uint32_t)((uint64_t)J * r.S + 4 * r.p0), AUX);
        return w;
    }

    template <int J>
    __device__ __forceinline__ void column(uint32_t (&acc)[Q]) {
        fetch<J + kPrefetch - 1>();
        uint32_t w = word<J>();
        // Column sequencing: the volatile (mutually ordered) empty asms pin this
        // column's tables after the previous column's accumulators, so only one
        // column's 30 table VGPRs are live; they also fence memory ops, which is
        // why the loads are issued explicitly kPrefetch-1 columns ahead above.
        asm volatile("" : "+v"(w));
        const NibPair T = nib_tables(w);
        mac_column<D, Q, J>(acc, T, std::make_integer_sequence<int, Q>{});
#pragma unroll
        for (int k = 0; k < Q; ++k) asm volatile("" : "+v"(acc[k]));
    }

    template <int... J>
    __device__ __forceinline__ void prologue(std::integer_sequence<int, J...>) {
        (fetch<J>(), ...);
    }
    template <int... J>
    __device__ __forceinline__ void columns(uint32_t (&acc)[Q], std::integer_sequence<int, J...>) {
        (column<J>(acc), ...);
    }
};

// Column p0 + t of every row: data words (MODE 1/2: from the payload, stored
// to the data rows) and the Q parity words.
// RING: the parity words also go to the fused kernel's LDS ring (r.ring).
// MASKED: only the parity rows flagged in r.miss0/miss1 are stored (decode:
// the missing parity rows; the present ones stay as received).
template <int D, int Q, int MODE, bool RING = false, bool MASKED = false>
__device__ __forceinline__ void encode_word(const EncodeRows& r) {
    constexpr int AUX = RING ? kStoreAux : kStoreAuxStandalone;  // the fused encoder re-reads its rows
    EncodeCtx<D, Q, MODE, AUX> cx{r, {}};
    uint32_t acc[Q];
#pragma unroll
    for (int k = 0; k < Q; ++k) acc[k] = 0u;
    cx.prologue(std::make_integer_sequence<int, kPrefetch - 1>{});
    cx.columns(acc, std::make_integer_sequence<int, D>{});
#pragma unroll
    for (int k = 0; k < Q; ++k) {
        if constexpr (MASKED) {
            if (!(((k < 64) ? (r.miss0 >> k) : (r.miss1 >> (k & 63))) & 1u)) continue;
        }
        __builtin_amdgcn_raw_buffer_store_b32(acc[k], r.sh, r.vsh, (uint32_t)((uint64_t)(D + k) * r.S + 4 * r.p0),
                                              AUX);
        if constexpr (RING) r.ring[k * r.rdw] = acc[k];
    }
}

// One thread = 4 byte positions of one instance, all N shards; one 256-thread
// block = 1 KiB of every row.  The coding matrix is compile-time, so every
// GF(2^8) product is a split-nibble table lookup resolved at compile time
// (one v_bitop3 per (parity row, data row) pair).
// Workgroups are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8).
// Renumber so XCD x runs the consecutive logical blocks
// [x*per + min(x, rem), ...) of a G-block grid: a bijection on [0, G).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t G) {
    const uint32_t x = b & 7, i = b >> 3, per = G >> 3, rem = G & 7;
    return x * per + (x < rem ? x : rem) + i;
}

template <int D, int Q, bool FROM_PAYLOAD>
__global__ __launch_bounds__(256, 4) void rs_encode_const(uint8_t* __restrict__ shards, uint64_t S, uint64_t L,
                                                       uint64_t n, uint32_t blocks_per_inst,
                                                       const uint8_t* __restrict__ payloads, uint64_t pstride,
                                                       const uint64_t* __restrict__ plen) {
    // XCD-aware block numbering: the G/8 logical blocks an XCD receives are
    // consecutive, so neighbouring 1-KiB slices of a row share that XCD's L2
    // (8,192 x 1 MiB: 35.6 -> 34.1 GB of HBM traffic).
    const uint32_t lb = xcd_block(blockIdx.x, gridDim.x);
    const uint64_t inst = lb / blocks_per_inst;
    if (inst >= n) return;
    uint8_t* base = shards + inst * (uint64_t)(D + Q) * S;
    const uint32_t blk = lb % blocks_per_inst;
    const uint32_t p0 = blk * 256, p = p0 + threadIdx.x;
    const uint8_t* pay = FROM_PAYLOAD ? payloads + inst * pstride : base;
    const uint64_t P = FROM_PAYLOAD ? plen[inst] : 0;
    EncodeRows r{raw_rsrc(base), raw_rsrc(pay), 4 * threadIdx.x, 4 * threadIdx.x, S, L, p0, threadIdx.x, base, pay, P};
    if constexpr (FROM_PAYLOAD) {
        if (!payload_fits(P, pstride, D, L)) return;  // device-mode argument check (flagged by rbc_check_plen)
        const uint64_t end = 4 * (uint64_t)(blk * 256 + 256);  // value-byte end of this block in a row
        // interior: past the length prefix, inside the row, and the last row's
        // dwordx2 window [.., (D-1)L + end + 4) inside the payload (+4 prefix)
        const bool interior = blk > 0 && end <= L && (uint64_t)(D - 1) * L + end + 4 <= P + 4;
        if (interior) {
            encode_word<D, Q, 2>(r);
        } else if (4 * (uint64_t)p < L) {
            encode_word<D, Q, 1>(r);
        }
    } else {
        if (4 * (uint64_t)p < L) encode_word<D, Q, 0>(r);
    }
}

// Reconstruct's second half (rse reconstruct: missing parity rows are encoded
// from the completed data rows): after rs_code_movrel rebuilt the missing data
// rows of a data-only plan (rs_plan max_row = D), the compile-time encoder
// recomputes the parity words and stores only the missing parity rows.
// Instances whose plan failed (too few rows present) or with no missing parity
// row exit at once.
template <int D, int Q>
__global__ __launch_bounds__(256, 4) void rs_encode_missing(uint8_t* __restrict__ shards, uint64_t S, uint64_t L,
                                                         uint64_t n, uint32_t blocks_per_inst,
                                                         const uint8_t* __restrict__ present,
                                                         const uint8_t* __restrict__ plans, uint64_t plan_stride) {
    const uint32_t lb = xcd_block(blockIdx.x, gridDim.x);
    const uint64_t inst = lb / blocks_per_inst;
    if (inst >= n) return;
    if (reinterpret_cast<const CodePlan*>(plans + inst * plan_stride)->status != 0) return;
    const uint8_t* pr = present + inst * (uint64_t)(D + Q) + D;
    uint64_t m0 = 0, m1 = 0;
#pragma unroll
    for (int k = 0; k < Q; ++k) {
        const uint64_t miss = __builtin_amdgcn_readfirstlane((uint32_t)pr[k]) == 0u;
        if (k < 64)
            m0 |= miss << k;
        else
            m1 |= miss << (k & 63);
    }
    if (!(m0 | m1)) return;
    uint8_t* base = shards + inst * (uint64_t)(D + Q) * S;
    const uint32_t blk = lb % blocks_per_inst;
    const uint32_t p0 = blk * 256, p = p0 + threadIdx.x;
    if (4 * (uint64_t)p >= L) return;
    EncodeRows r{raw_rsrc(base), raw_rsrc(base), 4 * threadIdx.x, 4 * threadIdx.x, S, L, p0, threadIdx.x, base, base, 0};
    r.miss0 = m0;
    r.miss1 = m1;
    encode_word<D, Q, 0, false, true>(r);
}

// Pack only (Trivial coding, N <= 3): send_shards' buffer into N rows.
// send_shards' prefix/pad/chunk into the first `rows` (= D) shards of each
// N-shard instance (the parity rows are left to the coder).
__global__ __launch_bounds__(256) void pack_rows(uint8_t* __restrict__ shards, uint64_t S, uint64_t L, uint32_t N,
                                                 uint32_t rows, uint64_t n, uint32_t blocks_per_inst,
                                                 const uint8_t* __restrict__ payloads, uint64_t pstride,
                                                 const uint64_t* __restrict__ plen) {
    const uint64_t inst = blockIdx.x / blocks_per_inst;
    const uint64_t p = (uint64_t)(blockIdx.x % blocks_per_inst) * 256 + threadIdx.x;
    if (inst >= n || 4 * p >= L) return;
    const uint8_t* pay = payloads + inst * pstride;
    const uint64_t P = plen[inst];
    if (!payload_fits(P, pstride, rows, L)) return;  // flagged by rbc_check_plen
    for (uint32_t j = 0; j < rows; ++j)
        reinterpret_cast<uint32_t*>(shards + (inst * N + j) * S)[p] = value_word(pay, P, (uint64_t)j * L + 4 * p);
}

// Device-mode argument check of hbg_rbc_encode_merkle (payload_fits); the
// encode kernels skip an instance that fails it.
__global__ __launch_bounds__(256) void rbc_check_plen(uint64_t n, const uint64_t* __restrict__ plen, uint64_t pstride,
                                                      uint32_t D, uint64_t L, int32_t* __restrict__ err) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n && !payload_fits(plen[k], pstride, D, L)) flag_error(err, HBG_E_ARG);
}

// Coding::Trivial (N <= 3) reconstruct: every shard must be present.
__global__ __launch_bounds__(256) void rbc_trivial_status(uint64_t n, uint32_t N, const uint8_t* __restrict__ present,
                                                          int32_t* __restrict__ status) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int32_t st = 0;
    for (uint32_t i = 0; i < N; ++i)
        if (!present[k * N + i]) st = HBG_E_TOO_FEW_SHARDS_PRESENT;
    status[k] = st;
}

// Generic coding: out_row[o] = XOR_j coef[o][j] * in_row[j] for one instance's
// plan (see rbc_kernels.h CodePlan) — reconstruct (per-instance coefficients)
// and encode for (D, Q) without a compile-time encoder.  Coefficients are
// run-time but wave-uniform; output rows are tiled kGenericTile at a time in
// registers.  kGenericLds: the LDS copy of the split-nibble tables,
// lane-private slots [wave][32 entries][64 lanes] (conflict-free).
constexpr uint32_t kGenericLds = 4 * 32 * 64 * 4;  // 32 KiB per 256-thread block

// The 16 + 16 split-nibble combinations of each data word stay in VGPRs and
// the wave-uniform coefficient (decoded with SALU from the plan's offsets)
// selects them by M0-relative register addressing (v_movrels): 2 selects + 1
// v_bitop3 per MAC-word for the first kMovrelSplit output rows of a tile; the
// rest read an LDS copy of the tables, so the SALU/movrel and LDS pipes run
// side by side.
constexpr int kMovrelSplit = 16;
__global__ __launch_bounds__(256) void rs_code_movrel(uint8_t* __restrict__ shards, uint64_t S, uint64_t L,
                                                      uint32_t N, uint32_t D, uint64_t n,
                                                      uint32_t blocks_per_inst, const uint8_t* __restrict__ plans,
                                                      uint64_t plan_stride) {
    typedef const __attribute__((address_space(4))) uint32_t* cu32;  // scalar (SMEM) loads
    const uint32_t lb = xcd_block(blockIdx.x, gridDim.x);  // XCD-aware (decode 13.25 -> 13.10 ms / 2,048)
    const uint64_t inst = lb / blocks_per_inst;
    const uint32_t p = (lb % blocks_per_inst) * 256 + threadIdx.x;
    if (inst >= n) return;
    const uint32_t Q = N - D, qp = plan_qpad(Q);
    const uint8_t* pbase = plans + inst * plan_stride;
    // the plan through the scalar cache (16-B aligned, wave-uniform): status,
    // n_out and the row-index bytes as s_load_dword — vector loads of them sat
    // on the critical path of every output row's store address
    const cu32 pw = (cu32)pbase;
    if ((int32_t)pw[0] != 0) return;  // CodePlan::status
    const uint32_t n_out = pw[1];
    constexpr uint32_t kInW = offsetof(CodePlan, in_idx) / 4, kOutW = offsetof(CodePlan, out_idx) / 4;
    static_assert(offsetof(CodePlan, in_idx) % 4 == 0 && offsetof(CodePlan, out_idx) % 4 == 0, "dword-aligned");
    auto in_row = [&](uint32_t j) { return (pw[kInW + (j >> 2)] >> (8 * (j & 3))) & 0xFFu; };
    auto out_row = [&](uint32_t o) { return (pw[kOutW + (o >> 2)] >> (8 * (o & 3))) & 0xFFu; };
    const bool active = 4 * (uint64_t)p < L;
    const cu32 offs = (cu32)(pbase + plan_offs_at(D, Q));
    uint8_t* base = shards + inst * (uint64_t)N * S;
    extern __shared__ uint32_t gtab[];
    uint32_t* tab = gtab + (threadIdx.x >> 6) * (32 * 64) + (threadIdx.x & 63);  // entry e at tab[64 e]
    const uint32_t tab_addr = (uint32_t)(uintptr_t)tab;                             // LDS byte address
    tab[0] = 0u;
    tab[16 * 64] = 0u;
    for (uint32_t o0 = 0; o0 < n_out; o0 += kGenericTile) {
        uint32_t acc[kGenericTile];
#pragma unroll
        for (int o = 0; o < (int)kGenericTile; ++o) acc[o] = 0u;
        // wave-uniform row count of this tile: a tile of at most kMovrelSplit
        // rows (a data-only plan: ~D/3 rows) skips the LDS rows and tables
        const uint32_t cnt = (n_out - o0) < (uint32_t)kGenericTile ? (n_out - o0) : (uint32_t)kGenericTile;
        const bool use_lds = cnt > (uint32_t)kMovrelSplit;
        for (uint32_t j = 0; j < D; ++j) {
            const uint32_t w = active ? reinterpret_cast<const uint32_t*>(base + (uint64_t)in_row(j) * S)[p] : 0u;
            const NibPair T = nib_tables(w);
            typedef uint32_t v16 __attribute__((ext_vector_type(16)));
            v16 tl, th;  // vector values: a dynamic uniform index lowers to v_movrels
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                tl[e] = T.lo.t[e];
                th[e] = T.hi.t[e];
            }
            if (kMovrelSplit < (int)kGenericTile && use_lds) {
#pragma unroll
                for (int e = 1; e < 16; ++e) {
                    tab[64 * e] = T.lo.t[e];
                    tab[64 * (16 + e)] = T.hi.t[e];
                }
            }
            const cu32 oj = offs + 2 * ((uint64_t)j * qp + o0);
            typedef const __attribute__((address_space(3))) uint32_t* lds32;
            // offsets are LDS byte offsets 256 * entry (rs_plan); padded rows
            // (o >= cnt) point at entry 0 of both tables, i.e. zero.  Rows below
            // kMovrelSplit select from registers (SALU + v_movrels), the rest read
            // the LDS copy: the two pipes run side by side.
#pragma unroll
            for (int o = 0; o < kMovrelSplit; ++o) {
                const uint32_t lo = oj[2 * o] >> 8, hi = (oj[2 * o + 1] >> 8) - 16u;
                acc[o] = xor3u(acc[o], tl[lo & 15u], th[hi & 15u]);
            }
            // (two straight-line bodies, no early exit: acc[] stays in VGPRs)
            if (use_lds) {
#pragma unroll
                for (int o = kMovrelSplit; o < (int)kGenericTile; ++o)
                    acc[o] = xor3u(acc[o], *(lds32)(uintptr_t)(tab_addr + oj[2 * o]),
                                   *(lds32)(uintptr_t)(tab_addr + oj[2 * o + 1]));
            }
        }
        if (active) {
#pragma unroll
            for (int o = 0; o < (int)kGenericTile; ++o)
                if ((uint32_t)o < cnt) reinterpret_cast<uint32_t*>(base + (uint64_t)out_row(o0 + o) * S)[p] = acc[o];
        }
    }
}

// Per-instance reconstruct plan (rse reconstruct_internal, restated):
// rows_used = first D present rows in index order; dec = inv(M[rows_used]);
// for every missing row r < max_row: coef[r] = M[r] * dec.  max_row = N: one
// pass rebuilds missing data AND parity rows (identical bytes to rse's
// two-pass form: the same linear map of the same D input rows); max_row = D:
// the missing data rows only, and rs_encode_missing then encodes the missing
// parity rows from the completed data rows — rse's own order.
// One 256-thread workgroup per instance; dynamic LDS: aug[D][2D] + row buffer.
__global__ __launch_bounds__(256) void rs_plan(const uint8_t* __restrict__ present, uint32_t D, uint32_t Q,
                                               uint32_t max_row, uint64_t n, const uint8_t* __restrict__ matrix,
                                               uint8_t* __restrict__ plans, uint64_t plan_stride) {
    const uint64_t inst = blockIdx.x;
    if (inst >= n) return;
    const uint32_t N = D + Q;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* lg = lds;           // 256
    uint8_t* ex = lds + 256;     // 512
    uint8_t* aug = lds + 768;    // D * 2D
    __shared__ uint32_t s_rows[256];
    __shared__ uint32_t s_np, s_nout, s_status, s_piv;
    __shared__ uint8_t s_out[256];
    const uint8_t* pr = present + inst * N;
    CodePlan* plan = reinterpret_cast<CodePlan*>(plans + inst * plan_stride);
    uint8_t* coef = reinterpret_cast<uint8_t*>(plan) + sizeof(CodePlan);
    uint32_t* offs = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(plan) + plan_offs_at(D, Q));
    uint16_t* nidx = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(plan) + plan_nidx_at(D, Q));
    const uint32_t qp = plan_qpad(Q);
    const uint32_t t = threadIdx.x;
    // GF tables into LDS
    for (uint32_t i = t; i < 256; i += blockDim.x) lg[i] = kGf.log[i];
    for (uint32_t i = t; i < 510; i += blockDim.x) ex[i] = kGf.exp[i];
    if (t == 0) {
        uint32_t np = 0, no = 0;
        for (uint32_t i = 0; i < N; ++i) {
            if (pr[i]) {
                if (np < D) s_rows[np] = i;
                ++np;
            } else if (i < max_row) {
                s_out[no++] = (uint8_t)i;
            }
        }
        s_np = np;
        s_nout = no;
        s_status = (np < D) ? (uint32_t)(-HBG_E_TOO_FEW_SHARDS_PRESENT) : 0u;
    }
    __syncthreads();
    auto gmul = [&](uint32_t a, uint32_t b) -> uint32_t { return (a && b) ? ex[lg[a] + lg[b]] : 0u; };
    if (s_status != 0 || s_nout == 0) {
        // nothing to rebuild below max_row: the input rows are still the plan's
        // (rbc_decode_merkle re-encodes missing parity rows from them)
        if (s_status == 0)
            for (uint32_t j = t; j < D; j += blockDim.x) plan->in_idx[j] = (uint8_t)s_rows[j];
        if (t == 0) {
            plan->status = s_status ? -(int32_t)s_status : 0;
            plan->n_out = 0;
        }
        return;
    }
    // aug = [M[rows_used] | I]
    const uint32_t W = 2 * D;
    for (uint32_t e = t; e < D * W; e += blockDim.x) {
        const uint32_t r = e / W, c = e % W;
        aug[e] = c < D ? matrix[s_rows[r] * D + c] : (uint8_t)(c - D == r);
    }
    __syncthreads();
    for (uint32_t r = 0; r < D; ++r) {
        if (t == 0) {
            uint32_t piv = r;
            while (piv < D && aug[piv * W + r] == 0) ++piv;
            s_piv = piv;
        }
        __syncthreads();
        const uint32_t piv = s_piv;
        if (piv == D) {  // singular: cannot happen for a Vandermonde-derived M
            if (t == 0) {
                plan->status = HBG_E_SINGULAR_MATRIX;
                plan->n_out = 0;
            }
            return;
        }
        if (piv != r)
            for (uint32_t c = t; c < W; c += blockDim.x) {
                const uint8_t a = aug[r * W + c];
                aug[r * W + c] = aug[piv * W + c];
                aug[piv * W + c] = a;
            }
        __syncthreads();
        const uint32_t s = ex[255 - lg[aug[r * W + r]]];  // inverse of pivot (log of 1 = 0 -> exp[255] = 1)
        __syncthreads();
        for (uint32_t c = t; c < W; c += blockDim.x) aug[r * W + c] = (uint8_t)gmul(s, aug[r * W + c]);
        __syncthreads();
        for (uint32_t e = t; e < D * W; e += blockDim.x) {
            const uint32_t rb = e / W, c = e % W;
            if (rb == r) continue;
            const uint32_t f = aug[rb * W + r];
            if (f && c != r) aug[e] ^= (uint8_t)gmul(f, aug[r * W + c]);
        }
        __syncthreads();
        for (uint32_t rb = t; rb < D; rb += blockDim.x)
            if (rb != r) aug[rb * W + r] = 0;
        __syncthreads();
    }
    // coef[o][c] = sum_t M[out_o][t] * dec[t][c],  dec[t][c] = aug[t*W + D + c]
    const uint32_t no = s_nout;
    for (uint32_t e = t; e < no * D; e += blockDim.x) {
        const uint32_t o = e / D, c = e % D;
        const uint8_t* mrow = matrix + (uint32_t)s_out[o] * D;
        uint32_t acc = 0;
        for (uint32_t k = 0; k < D; ++k) acc ^= gmul(mrow[k], aug[k * W + D + c]);
        coef[o * D + c] = (uint8_t)acc;
        offs[2 * (c * qp + o)] = nib_off_lo(acc);
        offs[2 * (c * qp + o) + 1] = nib_off_hi(acc);
        if (o < plan_nidx_rows(D)) nidx[c * plan_nidx_rows(D) + o] = (uint16_t)nib_idx_pair(acc);
    }
    for (uint32_t e = t; e < (qp - no) * D; e += blockDim.x) {  // padding rows: the zero entries
        const uint32_t o = no + e / D, c = e % D;
        offs[2 * (c * qp + o)] = nib_off_lo(0);
        offs[2 * (c * qp + o) + 1] = nib_off_hi(0);
        if (o < plan_nidx_rows(D)) nidx[c * plan_nidx_rows(D) + o] = (uint16_t)nib_idx_pair(0);
    }
    for (uint32_t j = t; j < D; j += blockDim.x) plan->in_idx[j] = (uint8_t)s_rows[j];
    for (uint32_t o = t; o < no; o += blockDim.x) plan->out_idx[o] = s_out[o];
    if (t == 0) {
        plan->status = 0;
        plan->n_out = no;
    }
}

// ============================================================== family 2: Merkle
// One work-item per leaf; lanes_per_inst = next_pow2(N) (<= 256); tree levels
// built in LDS by the owning lanes.  levels: [n][nodes][32].
// Blocks from b1 on (instances from n1 on) hash each leaf on a lane PAIR
// (sha3_256_aligned8_pair, 2 * lpi lanes an instance): launch_merkle_build
// sends the launch's partial last generation of blocks there, as twice the
// blocks of ~0.63 the duration, so it spreads over every CU instead of
// adding a whole block duration on some of them.
// PAIRS: 0 one-lane blocks only; 1 lane-pair blocks only (no block prefetch,
// 102 VGPRs: fewer than CUs' worth of blocks, latency-bound — 640 x N = 16
// 0.75 -> 0.67 ms, 300 x N = 64 2.89 -> 2.62 ms against the prefetching pair
// path, gpurun_out r06k2); 2 both, split at block b1 (the pairs prefetch)
template <int PAIRS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PAIRS == 1 ? 5 : 1))) void merkle_build(const uint8_t* __restrict__ shards, uint64_t S, uint64_t L,
                                                    uint32_t N, uint32_t lpi, uint32_t nodes, uint64_t n,
                                                    uint8_t* __restrict__ levels, uint32_t b1, uint64_t n1) {
    extern __shared__ __attribute__((aligned(16))) uint32_t mlds[];
    const bool pair = PAIRS == 1 || (PAIRS == 2 && blockIdx.x >= b1);
    const uint32_t lanes = pair ? 2 * lpi : lpi;       // lanes per instance
    const uint32_t li = threadIdx.x / lanes, tl = threadIdx.x % lanes;
    const uint64_t inst = pair ? n1 + (uint64_t)(blockIdx.x - b1) * (256 / lanes) + li
                               : (uint64_t)blockIdx.x * (256 / lpi) + li;
    const bool live = inst < n;
    uint32_t* tree = mlds + (uint64_t)li * nodes * 8;
    uint4* gout = reinterpret_cast<uint4*>(levels + inst * (uint64_t)nodes * 32);
    if (pair) {
        const uint32_t leaf = tl >> 1, half = tl & 1u;
        if (live && leaf < N) {
            uint32_t d[4];
            sha3_256_aligned8_pair<PAIRS == 2>(shards + (inst * N + leaf) * S, L, half, d);
            uint32_t* g = reinterpret_cast<uint32_t*>(gout) + leaf * 8 + half;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                tree[leaf * 8 + 2 * i + half] = d[i];
                g[2 * i] = d[i];
            }
        }
    } else if (PAIRS != 1 && live && tl < N) {
        const uint32_t leaf = tl;
        uint32_t d[8];
        sha3_256_aligned8<1, true>(shards + (inst * N + leaf) * S, L, d);
#pragma unroll
        for (int i = 0; i < 8; ++i) tree[leaf * 8 + i] = d[i];
        gout[2 * leaf] = make_uint4(d[0], d[1], d[2], d[3]);
        gout[2 * leaf + 1] = make_uint4(d[4], d[5], d[6], d[7]);
    }
    __syncthreads();
    const uint32_t leaf = tl;  // the tree levels: one lane a node
    uint32_t base = 0, cnt = N;
    while (cnt > 1) {
        const uint32_t nn = (cnt + 1) / 2;
        if (live && leaf < nn) {
            uint32_t d[8];
            if (2 * leaf + 1 < cnt) {
                uint32_t l[8], r[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    l[i] = tree[(base + 2 * leaf) * 8 + i];
                    r[i] = tree[(base + 2 * leaf + 1) * 8 + i];
                }
                sha3_pair<1>(l, r, d);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) d[i] = tree[(base + 2 * leaf) * 8 + i];
            }
            const uint32_t at = base + cnt + leaf;
#pragma unroll
            for (int i = 0; i < 8; ++i) tree[at * 8 + i] = d[i];
            gout[2 * at] = make_uint4(d[0], d[1], d[2], d[3]);
            gout[2 * at + 1] = make_uint4(d[4], d[5], d[6], d[7]);
        }
        __syncthreads();
        base += cnt;
        cnt = nn;
    }
}

// ============================================================== fused send_shards
// rbc_encode_merkle<D,Q>: hbbft send_shards (a2 prefix/pad/chunk, a3
// Coding::encode, a4 MerkleTree::from_vec) in ONE launch.  A workgroup owns
// IPB instances, LPI = next_pow2(N) lanes each.  The row sweep alternates two
// phases over the same lanes:
//   encode pass  lane = column: LPI 4-byte columns of every row of its
//                instance (the constant-matrix split-nibble coder,
//                encode_word), stored to the shard rows (written once); the
//                Q parity words also go to an LDS ring, row-major;
//   absorb       lane = row: every 136-byte Keccak block that the passes so
//                far have completed is absorbed (Keccak-f, keccak_asm.h) —
//                parity rows read it from the LDS ring (the transpose column ->
//                row happens in LDS, parity bytes never come back from memory),
//                data rows straight from the payload (a data row is payload
//                bytes at a per-row offset: 18 loads + v_alignbyte per block,
//                L2-resident since the encoder loaded the same lines one pass
//                earlier), except the blocks that touch the length prefix or
//                the zero padding, read back from the shard row just stored
//                (sc1 loads served by L2: the vector L1 may hold a stale copy of
//                a line touched before the pass wrote it).
// Measured alternatives (profiles/r03ij, 8,192 x 1 MiB): every data row read
// back from the shard rows 27.8 ms (26.6 as here), all 64 rows in the ring
// 33.5 ms (26 KB LDS per wave: 6 waves per CU), waves_per_eu(3) 37.6 ms
// (spills), no payload prefetch 27.6 ms.
// Ring: R bytes per parity row, R a multiple of 136 (a block never wraps),
// R >= one pass + the previous pass's unabsorbed tail (< 136), R/8 odd (a
// ds_read_b64 of R-strided rows hits 64 distinct banks per 32-lane group).
// The Keccak state stays in registers across encode passes.
// Addressing: raw buffer resources over the workgroup's shard and payload
// blocks, row offsets in SGPRs, the lane's offsets in VGPRs.
// Then the leaf digests and hbbft's tree (odd node promoted) in LDS.
__host__ __device__ constexpr uint32_t fused_ring_bytes(uint32_t pass_bytes) {
    uint32_t r = 136;
    while (r < pass_bytes + 135 || ((r / 8) & 1) == 0) r += 136;
    return r;
}


template <int D, int Q>
struct FusedShape {
    static constexpr uint32_t N = D + Q;
    static constexpr uint32_t LPI = N <= 1 ? 1 : (N <= 2 ? 2 : (N <= 4 ? 4 : (N <= 8 ? 8 : (N <= 16 ? 16 : (N <= 32 ? 32 : (N <= 64 ? 64 : (N <= 128 ? 128 : 256)))))));
    static constexpr uint32_t BLK = LPI < 64 ? 64 : LPI;
    static constexpr uint32_t IPB = BLK / LPI;
    static constexpr uint32_t NODES = merkle_nodes(N);
    static constexpr uint32_t R = fused_ring_bytes(4 * LPI);  // ring bytes per parity row
    static constexpr uint32_t RING = IPB * Q * R;  // the parity rows
    static constexpr uint32_t TREE = IPB * NODES * 32;
    static constexpr uint32_t LDS = RING > TREE ? RING : TREE;
    static constexpr int WPE = 2;  // waves per SIMD the register budget is sized for
};

template <int D, int Q>
__global__ __launch_bounds__((FusedShape<D, Q>::BLK)) __attribute__((amdgpu_waves_per_eu(FusedShape<D, Q>::WPE)))
void rbc_encode_merkle(uint8_t* __restrict__ shards, uint64_t S, uint64_t L, uint64_t n,
                       const uint8_t* __restrict__ payloads, uint64_t pstride, const uint64_t* __restrict__ plen,
                       uint8_t* __restrict__ levels, uint64_t* __restrict__ clk) {
    using F = FusedShape<D, Q>;
    // clock probe (hbg_test_set_clock_probe; null in every product call): the
    // workgroup's shader-clock (s_memtime) and 100 MHz real-time
    // (s_memrealtime) stamps at entry and exit, so the bench can report the
    // core clock the kernel actually ran at beside its roofline fraction
    uint64_t clk_t0 = 0, clk_r0 = 0;
    if (clk) {  // wave-uniform
        clk_t0 = __builtin_amdgcn_s_memtime();
        clk_r0 = __builtin_amdgcn_s_memrealtime();
    }
    constexpr uint32_t N = F::N, LPI = F::LPI, NODES = F::NODES, R = F::R;
    // LDS: the parity ring [IPB][Q][R] during the sweep, then the tree levels
    __shared__ __attribute__((aligned(16))) uint64_t lds[F::LDS / 8];
    uint32_t* ring_all = reinterpret_cast<uint32_t*>(lds);
    uint32_t* tree_all = reinterpret_cast<uint32_t*>(lds);
    // IPB == 1: one instance per workgroup, so every instance quantity is
    // wave-uniform (SGPR bases for the encoder's row addresses)
    const uint32_t sub = F::IPB == 1 ? 0u : threadIdx.x / LPI, t = F::IPB == 1 ? threadIdx.x : threadIdx.x % LPI;
    const uint64_t inst = (uint64_t)blockIdx.x * F::IPB + sub;
    const uint8_t* pay = payloads + inst * pstride;
    const uint64_t P = inst < n ? plen[inst] : 0;
    // device-mode argument check (flagged by rbc_check_plen): such an instance
    // is left unwritten (no shards, no levels)
    const bool live = inst < n && payload_fits(P, pstride, D, L);
    uint8_t* base = shards + inst * (uint64_t)N * S;
    uint32_t* ring = ring_all + sub * (Q * R / 4);  // this instance's parity rows
    uint32_t* tree = tree_all + sub * NODES * 8;
    const uint64_t cols = (L + 3) / 4;
    const uint32_t passes = (uint32_t)((cols + LPI - 1) / LPI);
    const bool row_lane = live && t < N;
    const bool ring_lane = row_lane && t >= (uint32_t)D;
    // buffer resources over the workgroup's first instance (uniform); a lane's
    // instance and column / row are VGPR offsets (host: IPB * N * S and
    // IPB * pstride < 2^31)
    const uint64_t inst0 = (uint64_t)blockIdx.x * F::IPB;
    EncodeRows r{raw_rsrc(shards + inst0 * N * S), raw_rsrc(payloads + inst0 * pstride),
                 (uint32_t)(sub * N * S) + 4 * t, (uint32_t)(sub * pstride) + 4 * t, S, L, 0, t, base, pay, P};
    r.rdw = R / 4;
    const uint32_t vrow = (uint32_t)((sub * N + t) * S);  // absorb: this lane's row
    // absorb (parity lanes): row t - D of the ring, as 8-byte words
    const uint64_t* rrow =
        reinterpret_cast<const uint64_t*>(ring + (ring_lane ? (int)t - D : 0) * (int)(R / 4));
    u64p a[25];
    keccak_zero(a);
    uint32_t done = 0;  // 136-byte blocks absorbed (the same count for every row)
    // interior pass (MODE 2/3 legal): past the length prefix, inside the row,
    // the last row's window inside the payload
    auto interior = [&](uint32_t ps) {
        const uint64_t end = 4ull * ((uint64_t)ps * LPI + LPI);  // value-byte end of the pass in a row
        return ps > 0 && end <= L && (uint64_t)(D - 1) * L + end + 4 <= P + 4;
    };
    // one 136-byte block of this lane's row at byte 136 * done, words [0, nw)
    auto load_block = [&](uint64_t (&w)[17]) {
        if (ring_lane) {
            const uint32_t rp = (136u * done) % R / 8;
#pragma unroll
            for (int i = 0; i < 17; ++i) w[i] = rrow[rp + i];
        } else if ((uint64_t)t * L + 136ull * done >= 4 &&
                   (uint64_t)t * L + 136ull * done + 140 <= P + 4) {
            // data row t's block is payload bytes [o, o + 136), o = t L + 136 done - 4:
            // 35 dwords from the dword below o, then a per-lane byte shift
            const uint64_t o = (uint64_t)t * L + 136ull * done - 4;
            const uint32_t a = (uint32_t)(o & ~3ull), sh8 = (uint32_t)(o & 3);
            uint32_t d[35];
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(r.py, (uint32_t)(sub * pstride) + a + 8 * i, 0, 0);
                d[2 * i] = v[0];
                d[2 * i + 1] = v[1];
            }
            d[34] = __builtin_amdgcn_raw_buffer_load_b32(r.py, (uint32_t)(sub * pstride) + a + 136, 0, 0);
#pragma unroll
            for (int i = 0; i < 17; ++i)
                w[i] = (uint64_t)__builtin_amdgcn_alignbyte(d[2 * i + 1], d[2 * i], sh8) |
                       ((uint64_t)__builtin_amdgcn_alignbyte(d[2 * i + 2], d[2 * i + 1], sh8) << 32);
        } else {
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(r.sh, vrow + 8 * i, 136 * done, kBufSc1);
                w[i] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
            }
        }
    };
    u32x2_a4 pre[D];  // the next interior pass's payload windows, loaded during this pass's Keccak work
    r.pre = pre;
    bool have_pre = false;
    // A data lane's absorb block comes from the payload (payload_block) unless
    // it touches the length prefix or the padding (then the shard row just
    // stored).  The first block a sweep absorbs is loaded at the top of the
    // pass, BEFORE the pass's 64 row stores: vmcnt is one in-order counter, so
    // a load issued after them waits for their (nt, HBM) acknowledgements.
    auto payload_block = [&](uint32_t blk) {
        return (uint64_t)t * L + 136ull * blk >= 4 && (uint64_t)t * L + 136ull * blk + 140 <= P + 4;
    };
    uint32_t pd[35];  // the raw payload dwords of that block (aligned view)
    auto fetch_payload_block = [&](uint32_t blk) {
        const uint64_t o = (uint64_t)t * L + 136ull * blk - 4;
        const uint32_t a0 = (uint32_t)(o & ~3ull);
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(r.py, (uint32_t)(sub * pstride) + a0 + 8 * i, 0, 0);
            pd[2 * i] = v[0];
            pd[2 * i + 1] = v[1];
        }
        pd[34] = __builtin_amdgcn_raw_buffer_load_b32(r.py, (uint32_t)(sub * pstride) + a0 + 136, 0, 0);
    };
    // the first block at which the last data row (the first to leave the
    // payload) reads its shard row: 136 b > P + 4 - 140 - (D - 1) L
    const uint64_t tail_blk = (P + 4 >= (uint64_t)(D - 1) * L + 140)
                                  ? (P + 4 - (uint64_t)(D - 1) * L - 140) / 136 + 1
                                  : 0;
    for (uint32_t ps = 0; ps < passes; ++ps) {
        const uint32_t p0 = ps * LPI, p = p0 + t;  // this lane's column in the encode pass
        r.p0 = p0;
        const uint64_t avail_now = 4ull * LPI * (ps + 1) < L ? 4ull * LPI * (ps + 1) : L;
        const bool first_due = (uint64_t)(done + 1) * 136 <= avail_now;  // wave-uniform
        const bool have_pd = first_due && row_lane && !ring_lane && payload_block(done);
        if (have_pd) fetch_payload_block(done);
        // ring position of this lane's column (wave-uniform pass start; a pass may wrap)
        uint32_t wpos = (uint32_t)(((uint64_t)ps * 4 * LPI) % R) + 4 * t;
        if (wpos >= R) wpos -= R;
        r.ring = ring + wpos / 4;
        if (live) {
            if (have_pre) {
                encode_word<D, Q, 3, true>(r);
            } else if (interior(ps)) {
                encode_word<D, Q, 2, true>(r);
            } else if (4 * (uint64_t)p < L) {
                encode_word<D, Q, 1, true>(r);
            }
        }
        const uint64_t written = 4ull * LPI * (ps + 1);
        const uint64_t avail = written < L ? written : L;
        // a sweep whose blocks include one read back from a shard row (block 0:
        // the length prefix; from tail_blk on: the padding) first waits for the
        // pass's stores; LDS (parity rows) is ordered by the barrier
        const uint32_t last_blk = (uint32_t)(avail / 136);  // exclusive
        if (done == 0 || last_blk > tail_blk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const bool next_pre = live && ps + 1 < passes && interior(ps + 1);
        have_pre = false;
        auto prefetch = [&]() {
            if (next_pre && !have_pre) {
                [&]<int... J>(std::integer_sequence<int, J...>) {
                    ((pre[J] = payload_window<J>(r, p0 + LPI)), ...);
                }(std::make_integer_sequence<int, D>{});
            }
            have_pre = next_pre;
        };
        bool use_pd = have_pd;  // pd holds this block's payload dwords (this lane)
        while ((uint64_t)(done + 1) * 136 <= avail) {
            if (row_lane) {
                uint64_t w[17];
                if (use_pd) {
                    const uint32_t sh8 = (uint32_t)(((uint64_t)t * L + 136ull * done - 4) & 3);
#pragma unroll
                    for (int i = 0; i < 17; ++i)
                        w[i] = (uint64_t)__builtin_amdgcn_alignbyte(pd[2 * i + 1], pd[2 * i], sh8) |
                               ((uint64_t)__builtin_amdgcn_alignbyte(pd[2 * i + 2], pd[2 * i + 1], sh8) << 32);
                } else {
                    load_block(w);
                }
#pragma unroll
                for (int i = 0; i < 17; ++i) {
                    a[i].lo ^= (uint32_t)w[i];
                    a[i].hi ^= (uint32_t)(w[i] >> 32);
                }
            }
            // the sweep's next block (a data lane, from the payload): loaded
            // before this block's permutation, its latency hidden under it
            // (an in-sweep prefetch of the next payload block into pd measured
            // 1.3 % slower: 26.71 against 26.37 ms, gpurun_out r04u)
            use_pd = false;
            // next pass's payload loads: behind this block's loads (vmcnt is
            // in order), ahead of a whole permutation
            prefetch();
            if (row_lane) perm<1>(a);
            ++done;
        }
        prefetch();
        // the next pass overwrites ring bytes this sweep has just absorbed
        __syncthreads();
    }
    uint32_t d[8];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the final block may read a stored shard row
    if (row_lane) {
        // final (possibly empty) block: bytes [136 done, L) + FIPS-202 padding.
        // Reads stay below round_up(L, 8) <= S (rows) / inside the ring.
        const uint32_t rem = (uint32_t)(L - (uint64_t)done * 136);
        uint64_t w[17];
        load_block(w);
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            uint64_t v = 0;
            if ((uint32_t)(8 * i) < rem) {
                v = w[i];
                const uint32_t left = rem - 8 * i;
                if (left < 8) v &= ~0ull >> (64 - 8 * left);
            }
            a[i].lo ^= (uint32_t)v;
            a[i].hi ^= (uint32_t)(v >> 32);
        }
        const uint32_t wi = rem >> 3, sh = (rem & 7) * 8;
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            if ((uint32_t)i == wi) {
                if (sh < 32) a[i].lo ^= 0x06u << sh;
                else a[i].hi ^= 0x06u << (sh - 32);
            }
        }
        a[16].hi ^= 0x80000000u;
        perm<1>(a);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            d[2 * i] = a[i].lo;
            d[2 * i + 1] = a[i].hi;
        }
    }
    uint4* gout = reinterpret_cast<uint4*>(levels + inst * (uint64_t)NODES * 32);
    __syncthreads();  // the tree reuses the ring
    if (row_lane) {
#pragma unroll
        for (int i = 0; i < 8; ++i) tree[t * 8 + i] = d[i];
        gout[2 * t] = make_uint4(d[0], d[1], d[2], d[3]);
        gout[2 * t + 1] = make_uint4(d[4], d[5], d[6], d[7]);
    }
    __syncthreads();
    uint32_t lbase = 0, cnt = N;
    while (cnt > 1) {
        const uint32_t nn = (cnt + 1) / 2;
        if (live && t < nn) {
            uint32_t h[8];
            if (2 * t + 1 < cnt) {
                uint32_t l[8], rr[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    l[i] = tree[(lbase + 2 * t) * 8 + i];
                    rr[i] = tree[(lbase + 2 * t + 1) * 8 + i];
                }
                sha3_pair<1>(l, rr, h);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) h[i] = tree[(lbase + 2 * t) * 8 + i];
            }
            const uint32_t at = lbase + cnt + t;
#pragma unroll
            for (int i = 0; i < 8; ++i) tree[at * 8 + i] = h[i];
            gout[2 * at] = make_uint4(h[0], h[1], h[2], h[3]);
            gout[2 * at + 1] = make_uint4(h[4], h[5], h[6], h[7]);
        }
        __syncthreads();
        lbase += cnt;
        cnt = nn;
    }
    if (clk) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            uint64_t* c = clk + 4ull * blockIdx.x;
            c[0] = clk_t0;
            c[1] = t1;
            c[2] = clk_r0;
            c[3] = r1;
        }
    }
}

// ============================================================== fused decode_from_shards
// rbc_decode_merkle<D,Q>: hbbft decode_from_shards' reconstruct (a7: rse
// reconstruct_shards — missing data rows from the first D present rows with
// the per-instance inverse, then the missing parity rows re-encoded from the
// completed data rows; present rows kept as received) and the Merkle rebuild
// over all N rows (MerkleTree::from_vec) in ONE launch — the decode twin of
// rbc_encode_merkle.  One wave per instance (LPI = 64 = N):
//   coding pass  lane = column: the D input words (first D present rows,
//                rs_plan's data-only plan), the missing data words by the
//                run-time split-nibble coder (wave-uniform coefficients,
//                v_movrels selects, as rs_code_movrel), the data words of the
//                instance (present: an input word, missing: a rebuilt one —
//                uniform register selects), the Q parity words by the
//                compile-time encoder; every MISSING row's word is stored to
//                its shard row and to its slot of the LDS ring (slot = rank of
//                the row among the missing rows: <= Q slots when decodable);
//   absorb       lane = row: every completed 136-byte block — a missing row
//                from the ring, a present row straight from its shard row
//                (not written by this kernel);
// then the leaf digests and the tree in LDS, levels written like
// merkle_build's.  Root check and glue stay in rbc_glue_status / _copy.
// An instance whose plan failed (fewer than D rows present) is left alone
// (no rows, no levels): the glue reports None from the plan status.
// Replaces rs_code_movrel -> rs_encode_missing -> merkle_build, whose
// Merkle pass re-read all N rows (25 GB per 8,192 x 1 MiB).
template <int D, int Q>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
void rbc_decode_merkle(uint8_t* __restrict__ shards, uint64_t S, uint64_t L, uint64_t n,
                       const uint8_t* __restrict__ present, const uint8_t* __restrict__ plans, uint64_t plan_stride,
                       uint8_t* __restrict__ levels, uint8_t* __restrict__ out, uint64_t ostride) {
    static_assert(D + Q == 64, "one wave per instance, lane = row");
    constexpr uint32_t N = D + Q, NODES = merkle_nodes(N);
    constexpr uint32_t R = fused_ring_bytes(4 * 64);
    typedef const __attribute__((address_space(4))) uint32_t* cu32;  // scalar (SMEM) loads
    typedef uint32_t v32 __attribute__((ext_vector_type(32)));      // dynamic uniform index -> v_movrels
    __shared__ __attribute__((aligned(16))) uint64_t lds[(Q * R > NODES * 32 ? Q * R : NODES * 32) / 8];
    __shared__ uint32_t junk[64];  // landing area of the L2-warming loads (never read)
    uint32_t* ring = reinterpret_cast<uint32_t*>(lds);
    uint32_t* tree = reinterpret_cast<uint32_t*>(lds);
    const uint32_t t = threadIdx.x;
    const uint64_t inst = blockIdx.x;
    if (inst >= n) return;
    const uint8_t* pbase = plans + inst * plan_stride;
    const CodePlan* plan = reinterpret_cast<const CodePlan*>(pbase);
    if (__builtin_amdgcn_readfirstlane(plan->status) != 0) return;  // too few present: decode is None
    const uint32_t n_out = __builtin_amdgcn_readfirstlane(plan->n_out);
    const uint64_t miss = __ballot(present[inst * N + t] == 0);      // bit r: row r is missing
    const uint64_t miss_data = miss & ((1ull << D) - 1ull);
    // present rows past the first D present ones (the coding inputs): the
    // absorb reads them straight from HBM, so each pass first pulls its 256-B
    // window of them into L2 (buffer -> LDS loads into `junk`: no VGPR
    // destination, nothing waits on them until the absorb)
    uint64_t warm = ~miss;
#pragma unroll
    for (int j = 0; j < D; ++j) warm &= warm - 1ull;
    const uint64_t pres_data = ~miss & ((1ull << D) - 1ull);
    uint8_t* base = shards + inst * (uint64_t)N * S;
    const __amdgpu_buffer_rsrc_t rows = raw_rsrc(base);
    const __amdgpu_buffer_rsrc_t orow = raw_rsrc(out ? out + inst * ostride : base);  // the glued payload
    const uint32_t qp = plan_qpad(Q);
    const cu32 nidx = (cu32)(pbase + plan_nidx_at(D, Q));  // plan_nidx_rows(D) / 2 dwords per input column
    uint32_t in_off[D];  // byte offset of input row j (wave-uniform)
#pragma unroll
    for (int j = 0; j < D; ++j) in_off[j] = __builtin_amdgcn_readfirstlane((uint32_t)plan->in_idx[j]) * (uint32_t)S;
    const uint64_t cols = (L + 3) / 4;
    const uint32_t passes = (uint32_t)((cols + 63) / 64);
    auto slot_of = [&](uint32_t row) { return (uint32_t)__builtin_popcountll(miss & ((1ull << row) - 1ull)); };
    const bool row_missing = (miss >> t) & 1ull;
    const uint64_t* rrow = reinterpret_cast<const uint64_t*>(ring + (row_missing ? slot_of(t) : 0u) * (R / 4));
    u64p a[25];
    keccak_zero(a);
    uint32_t done = 0;
    // words [0, nw) of the 136-byte block of row t at byte 136 * done (a
    // shard row is read only below round_up(L, 8) <= S)
    auto load_block = [&](uint64_t (&w)[17], uint32_t nw, uint32_t blk) {
        if (row_missing) {
            const uint32_t rp = (136u * blk) % R / 8;
#pragma unroll
            for (int i = 0; i < 17; ++i) w[i] = rrow[rp + i];
        } else {
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                w[i] = 0;
                if ((uint32_t)i < nw) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rows, t * (uint32_t)S + 8 * i, 136 * blk, 0);
                    w[i] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
                }
            }
        }
    };
    uint32_t pre[D];  // the next pass's input words, loaded during this pass's Keccak work
    bool have_pre = false;
    auto load_inputs = [&](uint32_t p0, uint32_t (&w)[D]) {
        const uint32_t vo = 4 * t;
#pragma unroll
        for (int j = 0; j < D; ++j) w[j] = __builtin_amdgcn_raw_buffer_load_b32(rows, vo, in_off[j] + 4 * p0, 0);
    };
    for (uint32_t ps = 0; ps < passes; ++ps) {
        const uint32_t p0 = ps * 64, p = p0 + t;
        const bool active = 4 * (uint64_t)p < L;
        uint32_t wpos = (uint32_t)(((uint64_t)ps * 256) % R) + 4 * t;
        if (wpos >= R) wpos -= R;
        uint32_t* rcol = ring + wpos / 4;
        // the sweep's first block is loaded after the barrier (loading a
        // present row's block here, before the pass's stores, measured 1.8 %
        // slower: 39.2 against 38.6 ms, gpurun_out r04u)
        uint64_t w[17];
        bool have_w = false;
        if (have_w) load_block(w, 17, done);
        for (uint64_t m = warm; m; m &= m - 1ull) {  // uniform loop, per-lane guard inside
            const uint32_t r = (uint32_t)__builtin_ctzll(m);
            const uint32_t so = __builtin_amdgcn_readfirstlane(r * (uint32_t)S + 4 * p0);
            if (active)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rows, (__attribute__((address_space(3))) void*)junk, 4, 4 * t, so, 0, 0);
        }
        if (active) {
            uint32_t win[D];
            if (have_pre) {
#pragma unroll
                for (int j = 0; j < D; ++j) win[j] = pre[j];
            } else {
                load_inputs(p0, win);
            }

            // ---- missing data rows: run-time coefficients over the D inputs.
            // The accumulators are plain registers (static indices); the one
            // 32-entry table of an input word (lo nibbles 0..15, hi 16..31, the
            // plan's offsets index it directly) is the only dynamically indexed
            // vector, so the group branches below merge scalars, not vectors.
            uint32_t acc[D];
#pragma unroll
            for (int o = 0; o < D; ++o) acc[o] = 0u;
            if (n_out) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    uint32_t wj = win[j];
                    asm volatile("" : "+v"(wj));
                    const NibPair T = nib_tables(wj);
                    v32 tab;
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        tab[e] = T.lo.t[e];
                        tab[16 + e] = T.hi.t[e];
                    }
                    // the column's index pairs for every output row, loaded up front
                    // (unconditional scalar loads: their latency hides under the table build)
                    const cu32 nj = nidx + (uint64_t)j * (plan_nidx_rows(D) / 2);
                    uint32_t ix[(D + 1) / 2];
#pragma unroll
                    for (int i = 0; i < (D + 1) / 2; ++i) ix[i] = nj[i];
                    // rows in groups of 4, a group only while o0 < n_out (wave-uniform);
                    // rows o >= n_out inside a group point at the zero entries (rs_plan's padding)
#pragma unroll
                    for (int o0 = 0; o0 < D; o0 += 4) {
                        if ((uint32_t)o0 < n_out) {
#pragma unroll
                            for (int o = o0; o < (o0 + 4 < D ? o0 + 4 : D); ++o) {
                                const uint32_t pr = ix[o / 2] >> (16 * (o & 1));
                                acc[o] = xor3u(acc[o], tab[pr & 31u], tab[(pr >> 8) & 31u]);
                            }
                        }
                    }
#pragma unroll
                    for (int o = 0; o < D; ++o) asm volatile("" : "+v"(acc[o]));
                }
            }
            v32 accv, winv;
#pragma unroll
            for (int o = 0; o < 32; ++o) {
                accv[o] = o < D ? acc[o] : 0u;
                winv[o] = o < D ? win[o] : 0u;
            }
            // ---- the instance's data words: present -> its input word, missing -> rebuilt;
            // every data word also goes to the glued payload (value byte 4 on)
            const bool tail_pass = 4 * (uint64_t)(p0 + 64) > L;  // this pass holds the rows' last word
            uint32_t d[D];
#pragma unroll
            for (int J = 0; J < D; ++J) {
                const uint32_t below = (uint32_t)((1ull << J) - 1ull);
                if ((miss_data >> J) & 1ull) {
                    d[J] = accv[(uint32_t)__builtin_popcountll(miss_data & below) & 31u];
                    __builtin_amdgcn_raw_buffer_store_b32(d[J], rows, 4 * t, J * (uint32_t)S + 4 * p0, kStoreAux);
                    rcol[slot_of(J) * (R / 4)] = d[J];
                } else {
                    d[J] = winv[(uint32_t)__builtin_popcountll(pres_data & below) & 31u];
                }
                if (out) {
                    // payload byte J*L + 4p - 4 (row 0's first word is the length
                    // prefix: offset 2^32 - 4 lies past the resource, the store is
                    // dropped).  Unaligned dword stores; the last word of a row
                    // stores only its bytes below L, since the bytes past it are
                    // the next row's, written in the first pass.
                    const uint32_t vo = 4 * p + (uint32_t)J * (uint32_t)L - 4u;
                    if (!tail_pass || 4 * (uint64_t)p + 4 <= L) {
                        __builtin_amdgcn_raw_buffer_store_b32(d[J], orow, vo, 0, kStoreAux);
                    } else {
#pragma unroll
                        for (uint32_t b = 0; b < 3; ++b)
                            if (4 * (uint64_t)p + b < L)
                                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(d[J] >> (8 * b)), orow, vo + b, 0,
                                                                     kStoreAux);
                    }
                }
            }
            // ---- parity: the compile-time encoder over the data words; missing rows stored
            uint32_t accp[Q];
#pragma unroll
            for (int k = 0; k < Q; ++k) accp[k] = 0u;
            [&]<int... J>(std::integer_sequence<int, J...>) {
                (([&] {
                    uint32_t w = d[J];
                    asm volatile("" : "+v"(w));
                    const NibPair T = nib_tables(w);
                    mac_column<D, Q, J>(accp, T, std::make_integer_sequence<int, Q>{});
#pragma unroll
                    for (int k = 0; k < Q; ++k) asm volatile("" : "+v"(accp[k]));
                }()), ...);
            }(std::make_integer_sequence<int, D>{});
#pragma unroll
            for (int k = 0; k < Q; ++k) {
                if ((miss >> (D + k)) & 1ull) {
                    __builtin_amdgcn_raw_buffer_store_b32(accp[k], rows, 4 * t, (D + k) * (uint32_t)S + 4 * p0,
                                                          kStoreAux);
                    rcol[slot_of(D + k) * (R / 4)] = accp[k];
                }
            }
        }
        __syncthreads();  // the pass's ring words are visible to every row lane
        const uint64_t written = 256ull * (ps + 1);
        const uint64_t avail = written < L ? written : L;
        const bool next_pre = ps + 1 < passes && 4 * (uint64_t)(p0 + 64 + t) < L;
        have_pre = false;
        auto prefetch = [&]() {
            if (next_pre && !have_pre) load_inputs(p0 + 64, pre);
            have_pre = next_pre;
        };
        // the next block of the same sweep is loaded before this block's
        // permutation (its latency hides under it)
        while ((uint64_t)(done + 1) * 136 <= avail) {
            if (!have_w) load_block(w, 17, done);
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                a[i].lo ^= (uint32_t)w[i];
                a[i].hi ^= (uint32_t)(w[i] >> 32);
            }
            prefetch();
            have_w = (uint64_t)(done + 2) * 136 <= avail;
            if (have_w) load_block(w, 17, done + 1);
            perm<1>(a);
            ++done;
        }
        prefetch();
        __syncthreads();  // the next pass overwrites ring bytes this sweep has just absorbed
    }
    uint32_t dg[8];
    {
        // final (possibly empty) block: bytes [136 done, L) + FIPS-202 padding
        const uint32_t rem = (uint32_t)(L - (uint64_t)done * 136);
        uint64_t w[17];
        load_block(w, (rem + 7) / 8, done);
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            uint64_t v = 0;
            if ((uint32_t)(8 * i) < rem) {
                v = w[i];
                const uint32_t left = rem - 8 * i;
                if (left < 8) v &= ~0ull >> (64 - 8 * left);
            }
            a[i].lo ^= (uint32_t)v;
            a[i].hi ^= (uint32_t)(v >> 32);
        }
        const uint32_t wi = rem >> 3, sh = (rem & 7) * 8;
#pragma unroll
        for (int i = 0; i < 17; ++i) {
            if ((uint32_t)i == wi) {
                if (sh < 32) a[i].lo ^= 0x06u << sh;
                else a[i].hi ^= 0x06u << (sh - 32);
            }
        }
        a[16].hi ^= 0x80000000u;
        perm<1>(a);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            dg[2 * i] = a[i].lo;
            dg[2 * i + 1] = a[i].hi;
        }
    }
    uint4* gout = reinterpret_cast<uint4*>(levels + inst * (uint64_t)NODES * 32);
    __syncthreads();  // the tree reuses the ring
#pragma unroll
    for (int i = 0; i < 8; ++i) tree[t * 8 + i] = dg[i];
    gout[2 * t] = make_uint4(dg[0], dg[1], dg[2], dg[3]);
    gout[2 * t + 1] = make_uint4(dg[4], dg[5], dg[6], dg[7]);
    __syncthreads();
    uint32_t lbase = 0, cnt = N;
    while (cnt > 1) {
        const uint32_t nn = (cnt + 1) / 2;
        if (t < nn) {
            uint32_t h[8];
            if (2 * t + 1 < cnt) {
                uint32_t l[8], rr[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    l[i] = tree[(lbase + 2 * t) * 8 + i];
                    rr[i] = tree[(lbase + 2 * t + 1) * 8 + i];
                }
                sha3_pair<1>(l, rr, h);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) h[i] = tree[(lbase + 2 * t) * 8 + i];
            }
            const uint32_t at = lbase + cnt + t;
#pragma unroll
            for (int i = 0; i < 8; ++i) tree[at * 8 + i] = h[i];
            gout[2 * at] = make_uint4(h[0], h[1], h[2], h[3]);
            gout[2 * at + 1] = make_uint4(h[4], h[5], h[6], h[7]);
        }
        __syncthreads();
        lbase += cnt;
        cnt = nn;
    }
}

// Proof::validate(N) — one work-item per proof.  Work-item q validates proof
// k = q % n_base of the table (n_base = n: every proof once; n = views *
// n_base: each view's own validation of the whole table, ok view-major —
// hbg_merkle_validate_views), so views need no copies of the table.
__global__ __launch_bounds__(256) void merkle_validate(uint32_t N, uint64_t len, const uint8_t* __restrict__ values,
                                                       uint64_t vstride, const uint32_t* __restrict__ index,
                                                       const uint8_t* __restrict__ digests, uint32_t depth,
                                                       const uint32_t* __restrict__ ndig,
                                                       const uint8_t* __restrict__ roots, uint8_t* __restrict__ ok,
                                                       uint64_t n, uint64_t n_base) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const uint64_t k = q < n_base ? q : q % n_base;
    uint32_t d[8];
    sha3_256_aligned8<1>(values + k * vstride, len, d);
    uint32_t li = index[k], ln = N, used = 0;
    const uint32_t nd = ndig[k];
    const uint32_t* dg = reinterpret_cast<const uint32_t*>(digests + k * (uint64_t)depth * 32);
    bool good = true;
    while (ln > 1) {
        if ((li ^ 1u) < ln) {
            if (used >= nd || used >= depth) {
                good = false;
                break;
            }
            uint32_t s[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) s[i] = dg[used * 8 + i];
            ++used;
            if (li & 1u) sha3_pair<1>(s, d, d);
            else sha3_pair<1>(d, s, d);
        }
        li >>= 1;
        ln = (ln + 1) >> 1;
    }
    if (good && used != nd) good = false;
    if (good) {
        const uint32_t* rt = reinterpret_cast<const uint32_t*>(roots + k * 32);
#pragma unroll
        for (int i = 0; i < 8; ++i) good &= (rt[i] == d[i]);
    }
    ok[q] = good ? 1 : 0;
}

// ============================================================== glue (a8)
// status/length per instance: root check + BE u32 length of the glued value.
__global__ void rbc_glue_status(const uint8_t* __restrict__ shards, uint64_t S, uint64_t L, uint32_t N, uint32_t D,
                                uint64_t n, const uint8_t* __restrict__ levels, uint32_t nodes,
                                const uint8_t* __restrict__ roots, const int32_t* __restrict__ rstatus,
                                uint64_t* __restrict__ plen, uint8_t* __restrict__ status) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    bool good = rstatus ? (rstatus[k] == 0) : true;
    if (good) {
        const uint32_t* a = reinterpret_cast<const uint32_t*>(levels + (k * nodes + nodes - 1) * 32);
        const uint32_t* b = reinterpret_cast<const uint32_t*>(roots + k * 32);
#pragma unroll
        for (int i = 0; i < 8; ++i) good &= (a[i] == b[i]);
    }
    const uint64_t tot = (uint64_t)D * L;
    if (good && tot < 4) good = false;
    uint64_t len = 0;
    if (good) {
        const uint8_t* inst = shards + k * N * S;
        uint32_t v = 0;
        for (uint32_t x = 0; x < 4; ++x) v = (v << 8) | inst[(x / L) * S + x % L];
        len = v;
        if (len > tot - 4) len = tot - 4;  // `take(len)` truncates silently
    }
    plen[k] = len;
    status[k] = good ? HBG_DECODE_OK : HBG_DECODE_NONE;
}

// payload byte q = value byte q+4 of the concatenated data rows; one thread per
// 16 output bytes: 5 aligned dword loads + 4 v_alignbyte, one 16-B store when the
// destination allows it (byte loop only where a window crosses a row end or
// the payload end).
__global__ __launch_bounds__(256) void rbc_glue_copy(const uint8_t* __restrict__ shards, uint64_t S, uint64_t L,
                                                     uint32_t N, uint64_t n, uint32_t blocks_per_inst,
                                                     const uint64_t* __restrict__ plen,
                                                     const uint8_t* __restrict__ status, uint8_t* __restrict__ out,
                                                     uint64_t ostride) {
    const uint64_t inst = blockIdx.x / blocks_per_inst;
    const uint64_t q = ((uint64_t)(blockIdx.x % blocks_per_inst) * 256 + threadIdx.x) * 16;
    if (inst >= n || status[inst] != HBG_DECODE_OK) return;
    const uint64_t len = plen[inst];
    if (q >= len) return;
    const uint8_t* base = shards + inst * N * S;
    const uint32_t Lw = (uint32_t)L;
    const uint32_t x = (uint32_t)(q + 4);
    const uint32_t r = x / Lw, c = x - r * Lw;
    uint8_t* dst = out + inst * ostride + q;
    if (c + 16 <= Lw && q + 16 <= len) {
        const uint32_t* pw = reinterpret_cast<const uint32_t*>(base + (uint64_t)r * S) + (c >> 2);
        const uint32_t s = c & 3;
        uint32_t v[5];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = pw[i];
        v[4] = s ? pw[4] : 0u;  // pw[4] lies inside the row (c + 16 <= L) when s != 0
        uint4 w;
        w.x = __builtin_amdgcn_alignbyte(v[1], v[0], s);
        w.y = __builtin_amdgcn_alignbyte(v[2], v[1], s);
        w.z = __builtin_amdgcn_alignbyte(v[3], v[2], s);
        w.w = __builtin_amdgcn_alignbyte(v[4], v[3], s);
        if (((uintptr_t)dst & 15u) == 0) {
            *reinterpret_cast<uint4*>(dst) = w;
        } else {  // ostride % 4 == 0
            uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
            d4[0] = w.x;
            d4[1] = w.y;
            d4[2] = w.z;
            d4[3] = w.w;
        }
        return;
    }
    for (uint32_t b = 0; b < 16 && q + b < len; ++b) {
        const uint32_t xb = x + b, rb = xb / Lw, cb = xb - rb * Lw;
        dst[b] = base[(uint64_t)rb * S + cb];
    }
}

// A NONE instance's payload row is zeroed over the span a decode may have
// written ([0, D*L)): the fused N = 64 decoder stores the glued bytes before
// the root comparison, so without this a NONE row would hold bytes that
// failed authentication.  One workgroup per instance; an OK instance returns
// at once (include/hbgpu.h, hbg_rbc_decode).
__global__ __launch_bounds__(256) void rbc_glue_clear(uint64_t n, uint64_t span, const uint8_t* __restrict__ status,
                                                      uint8_t* __restrict__ out, uint64_t ostride) {
    const uint64_t inst = blockIdx.x;
    if (inst >= n || status[inst] == HBG_DECODE_OK) return;
    uint32_t* row = reinterpret_cast<uint32_t*>(out + inst * ostride);  // ostride % 4 == 0, out 4-aligned
    const uint64_t words = span / 4;
    for (uint64_t w = threadIdx.x; w < words; w += 256) row[w] = 0u;
    for (uint64_t b = words * 4 + threadIdx.x; b < span; b += 256) out[inst * ostride + b] = 0;
}

// ============================================================== synthetic inputs
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_bytes(uint32_t tag, uint64_t first, uint64_t nbytes,
                                                   uint8_t* __restrict__ out, uint64_t ostride, uint64_t n,
                                                   uint32_t blocks_per_row) {
    const uint64_t row = blockIdx.x / blocks_per_row;
    const uint64_t w = (uint64_t)(blockIdx.x % blocks_per_row) * 256 + threadIdx.x;
    if (row >= n || 8 * w >= nbytes) return;
    const uint64_t seed = 0x48424247ull ^ ((uint64_t)tag << 48) ^ (first + row);
    const uint64_t v = mix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull);
    uint8_t* dst = out + row * ostride + 8 * w;
    if (8 * w + 8 <= nbytes && (ostride % 8) == 0) {
        *reinterpret_cast<uint64_t*>(dst) = v;
    } else {
        for (uint64_t b = 0; b < 8 && 8 * w + b < nbytes; ++b) dst[b] = (uint8_t)(v >> (8 * b));
    }
}

// ============================================================== launchers
template <int D, int Q>
static hipError_t launch_encode_const(uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                      const uint8_t* payloads, uint64_t pstride, const uint64_t* plen,
                                      hipStream_t st) {
    const uint32_t bpi = (uint32_t)(((L + 3) / 4 + 255) / 256);
    const uint64_t blocks = n * bpi;
    HBG_GRID_CHECK(blocks, 256);
    if (payloads)
        rs_encode_const<D, Q, true><<<dim3((uint32_t)blocks), dim3(256), 0, st>>>(shards, S, L, n, bpi, payloads,
                                                                                   pstride, plen);
    else
        rs_encode_const<D, Q, false><<<dim3((uint32_t)blocks), dim3(256), 0, st>>>(shards, S, L, n, bpi, nullptr, 0,
                                                                                    nullptr);
    return hipGetLastError();
}

bool has_const_encoder(uint32_t D, uint32_t Q) {
    return (D == 2 && Q == 2) || (D == 6 && Q == 10) || (D == 22 && Q == 42) || (D == 44 && Q == 84);
}

// The constant encoders address rows through raw buffer resources of 2^31
// bytes (raw_rsrc): a workgroup's shard block and payload block must fit.
bool const_encoder_fits(uint32_t D, uint32_t Q, uint64_t S, uint64_t pstride, bool fused) {
    uint64_t ipb = 1;
    if (fused) {
        uint32_t lpi = 1;
        while (lpi < D + Q) lpi <<= 1;
        ipb = lpi < 64 ? 64 / lpi : 1;
    }
    const uint64_t lim = 1ull << 31;
    return has_const_encoder(D, Q) && ipb * (D + Q) * S < lim && ipb * (pstride + 16) < lim;
}

template <int D, int Q>
static hipError_t launch_missing(uint8_t* shards, uint64_t S, uint64_t L, uint64_t n, const uint8_t* present,
                                 const uint8_t* plans, uint64_t plan_stride, hipStream_t st) {
    const uint32_t bpi = (uint32_t)(((L + 3) / 4 + 255) / 256);
    HBG_GRID_CHECK(n * bpi, 256);
    rs_encode_missing<D, Q><<<dim3((uint32_t)(n * bpi)), dim3(256), 0, st>>>(shards, S, L, n, bpi, present, plans,
                                                                             plan_stride);
    return hipGetLastError();
}

hipError_t launch_rs_encode_missing(uint32_t D, uint32_t Q, uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                    const uint8_t* present, const uint8_t* plans, uint64_t plan_stride,
                                    hipStream_t st) {
    if (D == 2 && Q == 2) return launch_missing<2, 2>(shards, S, L, n, present, plans, plan_stride, st);
    if (D == 6 && Q == 10) return launch_missing<6, 10>(shards, S, L, n, present, plans, plan_stride, st);
    if (D == 22 && Q == 42) return launch_missing<22, 42>(shards, S, L, n, present, plans, plan_stride, st);
    if (D == 44 && Q == 84) return launch_missing<44, 84>(shards, S, L, n, present, plans, plan_stride, st);
    return hipErrorInvalidValue;
}

hipError_t launch_rs_encode_const(uint32_t D, uint32_t Q, uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                  const uint8_t* payloads, uint64_t pstride, const uint64_t* plen,
                                  hipStream_t st) {
    if (D == 2 && Q == 2) return launch_encode_const<2, 2>(shards, S, L, n, payloads, pstride, plen, st);
    if (D == 6 && Q == 10) return launch_encode_const<6, 10>(shards, S, L, n, payloads, pstride, plen, st);
    if (D == 22 && Q == 42) return launch_encode_const<22, 42>(shards, S, L, n, payloads, pstride, plen, st);
    if (D == 44 && Q == 84) return launch_encode_const<44, 84>(shards, S, L, n, payloads, pstride, plen, st);
    return hipErrorInvalidValue;
}

template <int D, int Q>
static hipError_t launch_fused(uint8_t* shards, uint64_t S, uint64_t L, uint64_t n, const uint8_t* payloads,
                               uint64_t pstride, const uint64_t* plen, uint8_t* levels, hipStream_t st,
                               uint64_t* clk, uint64_t clk_cap) {
    using F = FusedShape<D, Q>;
    const uint64_t blocks = (n + F::IPB - 1) / F::IPB;
    HBG_GRID_CHECK(blocks, F::BLK);
    if (blocks > clk_cap) clk = nullptr;  // the probe buffer holds clk_cap workgroups
    rbc_encode_merkle<D, Q><<<dim3((uint32_t)blocks), dim3(F::BLK), 0, st>>>(shards, S, L, n, payloads, pstride,
                                                                             plen, levels, clk);
    return hipGetLastError();
}

hipError_t launch_rbc_encode_merkle(uint32_t D, uint32_t Q, uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                    const uint8_t* payloads, uint64_t pstride, const uint64_t* plen, uint8_t* levels,
                                    hipStream_t st, uint64_t* clk, uint64_t clk_cap) {
    if (D == 2 && Q == 2) return launch_fused<2, 2>(shards, S, L, n, payloads, pstride, plen, levels, st, clk, clk_cap);
    if (D == 6 && Q == 10)
        return launch_fused<6, 10>(shards, S, L, n, payloads, pstride, plen, levels, st, clk, clk_cap);
    if (D == 22 && Q == 42)
        return launch_fused<22, 42>(shards, S, L, n, payloads, pstride, plen, levels, st, clk, clk_cap);
    if (D == 44 && Q == 84)
        return launch_fused<44, 84>(shards, S, L, n, payloads, pstride, plen, levels, st, clk, clk_cap);
    return hipErrorInvalidValue;
}

bool has_fused_decoder(uint32_t D, uint32_t Q) { return D == 22 && Q == 42; }

hipError_t launch_rbc_decode_merkle(uint32_t D, uint32_t Q, uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                    const uint8_t* present, const uint8_t* plans, uint64_t plan_stride,
                                    uint8_t* levels, uint8_t* out, uint64_t ostride, hipStream_t st) {
    if (!(D == 22 && Q == 42)) return hipErrorInvalidValue;
    HBG_GRID_CHECK(n, 64);
#ifdef HBG_DEC_NO_PAYLOAD  // diagnostic variant (tools/build_variant.py): the payload stores left out
    out = nullptr;
#endif
    rbc_decode_merkle<22, 42><<<dim3((uint32_t)n), dim3(64), 0, st>>>(shards, S, L, n, present, plans, plan_stride,
                                                                    levels, out, ostride);
    return hipGetLastError();
}

hipError_t launch_pack_rows(uint8_t* shards, uint64_t S, uint64_t L, uint32_t N, uint32_t rows, uint64_t n,
                            const uint8_t* payloads, uint64_t pstride, const uint64_t* plen, hipStream_t st) {
    const uint32_t bpi = (uint32_t)(((L + 3) / 4 + 255) / 256);
    HBG_GRID_CHECK(n * bpi, 256);
    pack_rows<<<dim3((uint32_t)(n * bpi)), dim3(256), 0, st>>>(shards, S, L, N, rows, n, bpi, payloads, pstride,
                                                               plen);
    return hipGetLastError();
}

hipError_t launch_rs_code_generic(uint8_t* shards, uint64_t S, uint64_t L, uint32_t N, uint32_t D, uint64_t n,
                                  const uint8_t* plans, uint64_t plan_stride, hipStream_t st) {
    const uint32_t bpi = (uint32_t)(((L + 3) / 4 + 255) / 256);
    HBG_GRID_CHECK(n * bpi, 256);
    rs_code_movrel<<<dim3((uint32_t)(n * bpi)), dim3(256), kGenericLds, st>>>(shards, S, L, N, D, n, bpi, plans,
                                                                            plan_stride);
    return hipGetLastError();
}

hipError_t launch_rs_plan(const uint8_t* present, uint32_t D, uint32_t Q, uint32_t max_row, uint64_t n,
                          const uint8_t* matrix, uint8_t* plans, uint64_t plan_stride, hipStream_t st) {
    const size_t lds = 768 + (size_t)D * 2 * D;
    HBG_GRID_CHECK(n, 256);
    rs_plan<<<dim3((uint32_t)n), dim3(256), lds, st>>>(present, D, Q, max_row, n, matrix, plans, plan_stride);
    return hipGetLastError();
}

// Compute units of the current device (the partial-generation split below).
static uint32_t device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 0;
    return (uint32_t)cus;
}

// The blocks past the last whole generation (one block a CU) — when they
// would fill at most half of the CUs — hash on lane pairs instead: twice the
// blocks, each ~0.63 of a block's duration, one a CU.  configs[1] (N = 16,
// 10 k instances: 625 blocks on 256 CUs): 2 + 0.63 block durations instead of
// 3.  Whole generations (the headline shapes, the epoch's chunks) are
// unchanged.  split = 0: one-lane blocks only, 1: lane pairs only (tests).
hipError_t launch_merkle_build(const uint8_t* shards, uint64_t S, uint64_t L, uint32_t N, uint64_t n,
                               uint8_t* levels, hipStream_t st, int split) {
    uint32_t lpi = 1;
    while (lpi < N) lpi <<= 1;
    const uint32_t nodes = merkle_nodes(N);
    const uint32_t ipb = 256 / lpi;
    const uint64_t blocks = (n + ipb - 1) / ipb;
    uint64_t b1 = blocks, b2 = 0;
    if (lpi <= 128 && split != 0) {
        const uint32_t cus = device_cus();
        const uint64_t gen = cus ? blocks / cus * cus : blocks;  // blocks in whole generations
        const uint64_t tail = n - std::min<uint64_t>(n, gen * ipb), tb = (tail + ipb / 2 - 1) / (ipb / 2);
        if (split == 1) {
            b1 = 0;
            b2 = (n + ipb / 2 - 1) / (ipb / 2);
        } else if (cus && tail && tb <= cus) {
            b1 = gen;
            b2 = tb;
        }
    }
    const size_t lds = (size_t)ipb * nodes * 32;
    HBG_GRID_CHECK(b1 + b2, 256);
    const dim3 grid((uint32_t)(b1 + b2)), blk(256);
    if (b2 == 0)
        merkle_build<0><<<grid, blk, lds, st>>>(shards, S, L, N, lpi, nodes, n, levels, (uint32_t)b1, b1 * ipb);
    else if (b1 == 0)
        merkle_build<1><<<grid, blk, lds, st>>>(shards, S, L, N, lpi, nodes, n, levels, 0u, 0u);
    else
        merkle_build<2><<<grid, blk, lds, st>>>(shards, S, L, N, lpi, nodes, n, levels, (uint32_t)b1, b1 * ipb);
    return hipGetLastError();
}

hipError_t launch_merkle_validate(uint32_t N, uint64_t len, const uint8_t* values, uint64_t vstride,
                                  const uint32_t* index, const uint8_t* digests, uint32_t depth,
                                  const uint32_t* ndig, const uint8_t* roots, uint8_t* ok, uint64_t n,
                                  hipStream_t st, uint32_t views) {
    const uint64_t total = n * views;
    HBG_GRID_CHECK((total + 255) / 256, 256);
    merkle_validate<<<dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, st>>>(N, len, values, vstride, index,
                                                                               digests, depth, ndig, roots, ok, total,
                                                                               n);
    return hipGetLastError();
}

hipError_t launch_rbc_glue(const uint8_t* shards, uint64_t S, uint64_t L, uint32_t N, uint32_t D, uint64_t n,
                           const uint8_t* levels, const uint8_t* roots, const int32_t* rstatus, uint64_t* plen,
                           uint8_t* status, uint8_t* out, uint64_t ostride, hipStream_t st, bool copy) {
    const uint32_t nodes = merkle_nodes(N);
    const uint64_t maxlen = (uint64_t)D * L;
    const uint32_t bpi = (uint32_t)(((maxlen + 15) / 16 + 255) / 256);
    HBG_GRID_CHECK(n * bpi, 256);  // every grid of this call, before the first launch
    HBG_GRID_CHECK(n, 256);
    rbc_glue_status<<<dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st>>>(shards, S, L, N, D, n, levels, nodes,
                                                                            roots, rstatus, plen, status);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    rbc_glue_clear<<<dim3((uint32_t)n), dim3(256), 0, st>>>(n, maxlen, status, out, ostride);
    e = hipGetLastError();
    if (e != hipSuccess || !copy) return e;
    rbc_glue_copy<<<dim3((uint32_t)(n * bpi)), dim3(256), 0, st>>>(shards, S, L, N, n, bpi, plen, status, out,
                                                                    ostride);
    return hipGetLastError();
}

hipError_t launch_rbc_check_plen(uint64_t n, const uint64_t* plen, uint64_t pstride, uint32_t D, uint64_t L,
                                 int32_t* err, hipStream_t st) {
    if (n == 0) return hipSuccess;
    HBG_GRID_CHECK((n + 255) / 256, 256);
    rbc_check_plen<<<dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st>>>(n, plen, pstride, D, L, err);
    return hipGetLastError();
}

hipError_t launch_rbc_trivial_status(uint64_t n, uint32_t N, const uint8_t* present, int32_t* status,
                                     hipStream_t st) {
    if (n == 0) return hipSuccess;
    HBG_GRID_CHECK((n + 255) / 256, 256);
    rbc_trivial_status<<<dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st>>>(n, N, present, status);
    return hipGetLastError();
}

hipError_t launch_synth(uint32_t tag, uint64_t first, uint64_t nbytes, uint8_t* out, uint64_t ostride, uint64_t n,
                        hipStream_t st) {
    const uint32_t bpr = (uint32_t)(((nbytes + 7) / 8 + 255) / 256);
    HBG_GRID_CHECK(n * bpr, 256);
    synth_bytes<<<dim3((uint32_t)(n * bpr)), dim3(256), 0, st>>>(tag, first, nbytes, out, ostride, n, bpr);
    return hipGetLastError();
}

}  // namespace hbg
