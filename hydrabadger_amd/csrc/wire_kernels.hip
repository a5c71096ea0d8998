// wire_kernels.hip — SURVEY.md §8(f4): hbbft broadcast wire format on gfx950.
//
// bincode 1.x (default config: little-endian fixed-width integers, u64
// sequence lengths, u32 enum variant index) of hbbft `broadcast::Message`
// [EXT, VegeBun-csj/hbbft master, src/broadcast/message.rs]:
//   Value(Proof<Vec<u8>>) = 0, Echo(Proof<Vec<u8>>) = 1, Ready(Digest) = 2,
//   CanDecode(Digest) = 3, EchoHash(Digest) = 4
// and `Proof<T> { value: T, index: usize, digests: Vec<Digest>, root_hash: Digest }`
// [EXT, src/broadcast/merkle.rs]; `Digest = [u8; 32]` is a serde tuple (no
// length).  A Value/Echo message for leaf i of an N-leaf tree is therefore
//   u32 tag | u64 L | value[L] | u64 i | u64 k | k x digest[32] | root[32]
// with k = hbg_proof_digests(N, i).  The reference builds these one at a time
// in `Broadcast::send_shards` / `handle_value` (proof -> Message -> bincode in
// hydrabadger's `WireMessages::start_send`, src/lib.rs:432-446) and parses
// them in `WireMessages::poll` (src/lib.rs:397-404).
//
// Both kernels are HBM byte movers (no arithmetic): every thread owns one
// 16-byte chunk of the destination, the value body is moved with aligned dword
// loads + v_alignbyte and 16-B stores, header/trailer bytes (≤ 0.6 % of a
// message at N=64, 1 MiB) go through a byte path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rbc_kernels.h"

namespace hbg {

__host__ __device__ inline uint32_t proof_digests(uint32_t N, uint32_t i) {
    if (i >= N) return 0;
    uint32_t k = 0, ln = N;
    while (ln > 1) {
        if ((i ^ 1u) < ln) ++k;
        i >>= 1;
        ln = (ln + 1) >> 1;
    }
    return k;
}

// flat-levels node of the j-th sibling digest of proof(i) (MerkleTree::proof's walk)
__device__ inline uint32_t sibling_node(uint32_t N, uint32_t i, uint32_t j) {
    uint32_t off = 0, ln = N, k = 0;
    while (ln > 1) {
        if ((i ^ 1u) < ln) {
            if (k == j) return off + (i ^ 1u);
            ++k;
        }
        off += ln;
        i >>= 1;
        ln = (ln + 1) >> 1;
    }
    return 0;
}

__device__ __forceinline__ uint8_t le_byte(uint64_t v, uint32_t b) { return (uint8_t)(v >> (8 * b)); }

// Byte o of message (tag, proof(inst, i)); value bytes come from the shard row.
__device__ inline uint8_t proof_msg_byte(uint64_t o, uint32_t tag, uint64_t L, const uint8_t* __restrict__ row,
                                         const uint8_t* __restrict__ lev, uint32_t nodes, uint32_t N, uint32_t i,
                                         uint32_t k) {
    if (o < 4) return le_byte(tag, (uint32_t)o);
    if (o < 12) return le_byte(L, (uint32_t)(o - 4));
    if (o < 12 + L) return row[o - 12];
    const uint64_t t = o - 12 - L;
    if (t < 8) return le_byte(i, (uint32_t)t);
    if (t < 16) return le_byte(k, (uint32_t)(t - 8));
    const uint64_t d = t - 16;
    if (d < 32ull * k) return lev[(uint64_t)sibling_node(N, i, (uint32_t)(d >> 5)) * 32 + (d & 31)];
    return lev[(uint64_t)(nodes - 1) * 32 + (d - 32ull * k)];
}

// 16 bytes starting at an arbitrary byte address p: one dwordx4 load at the
// dword-aligned address below p (+ one dword when p is not dword aligned) and
// 4 v_alignbyte.  Every dword read contains at least one byte of [p, p + 16).
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ uint4 load16_unaligned(const uint8_t* p) {
    const uint32_t s = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3);
    const u32x4_a4 v = *reinterpret_cast<const u32x4_a4*>(w);
    const uint32_t v4 = s ? w[4] : 0u;
    uint4 r;
    r.x = __builtin_amdgcn_alignbyte(v.y, v.x, s);
    r.y = __builtin_amdgcn_alignbyte(v.z, v.y, s);
    r.z = __builtin_amdgcn_alignbyte(v.w, v.z, s);
    r.w = __builtin_amdgcn_alignbyte(v4, v.w, s);
    return r;
}

// Every thread of the byte movers below owns kChunks 16-B chunks, 256 apart
// (coalesced per pass); a block covers kChunks * 4 KiB of one message.
constexpr uint32_t kChunks = 4;
constexpr uint32_t kBlockBytes = 256 * 16 * kChunks;

// grid: m messages x blocks_per_msg; thread = one 16-B destination chunk.
__global__ __launch_bounds__(256) void rbc_write_proof_msgs(uint32_t N, uint64_t L, const uint8_t* __restrict__ shards,
                                                            uint64_t S, const uint8_t* __restrict__ levels,
                                                            uint32_t nodes, uint64_t n, uint32_t tag, uint64_t m,
                                                            const uint64_t* __restrict__ inst,
                                                            const uint32_t* __restrict__ index,
                                                            uint8_t* __restrict__ out,
                                                            const uint64_t* __restrict__ out_off,
                                                            uint32_t blocks_per_msg, int32_t* __restrict__ err) {
    const uint64_t j = blockIdx.x / blocks_per_msg;
    if (j >= m) return;
    const uint32_t i = index[j];
    const uint64_t ki = inst[j];
    const uint32_t k = proof_digests(N, i);
    const uint64_t start = out_off[j], end = out_off[j + 1];
    // device-mode argument check (host mode rejects these up front): the message stays unwritten
    if (i >= N || ki >= n || end < start || end - start != 12 + L + 16 + 32ull * k + 32) {
        if (blockIdx.x % blocks_per_msg == 0 && threadIdx.x == 0) flag_error(err, HBG_E_ARG);
        return;
    }
    const uint8_t* row = shards + (ki * N + i) * S;
    const uint8_t* lev = levels + ki * nodes * 32ull;
    const uint64_t c0 = (uint64_t)(blockIdx.x % blocks_per_msg) * 256 * kChunks + threadIdx.x;
#pragma unroll
    for (uint32_t q = 0; q < kChunks; ++q) {
        const uint64_t A = (start & ~15ull) + 16 * (c0 + 256 * q);  // byte offset in out of this chunk
        if (A >= end) return;
        if (A >= start + 12 && A + 16 <= start + 12 + L) {  // interior of the value: 16-B move
            *reinterpret_cast<uint4*>(out + A) = load16_unaligned(row + (A - start - 12));
            continue;
        }
        const uint64_t lo = A > start ? A : start, hi = A + 16 < end ? A + 16 : end;
        for (uint64_t b = lo; b < hi; ++b) out[b] = proof_msg_byte(b - start, tag, L, row, lev, nodes, N, i, k);
    }
}

__device__ __forceinline__ uint64_t rd_le(const uint8_t* p, int nb) {
    uint64_t v = 0;
    for (int b = 0; b < nb; ++b) v |= (uint64_t)p[b] << (8 * b);
    return v;
}

// Parse message j: the bincode checks hbbft's deserialisation makes (EOF,
// variant index) plus the layout this batch table can hold (value length ==
// L).  Returns status; fills the header fields.
struct MsgHdr {
    int32_t status;
    uint32_t tag;
    uint64_t vlen, index, k, trailer;  // trailer = byte offset of the index field
};

__device__ inline MsgHdr parse_hdr(const uint8_t* __restrict__ msg, uint64_t len, uint64_t L) {
    MsgHdr h{0, 0xFFFFFFFFu, 0, 0, 0, 0};
    if (len < 4) {
        h.status = HBG_E_WIRE_EOF;
        return h;
    }
    h.tag = (uint32_t)rd_le(msg, 4);
    if (h.tag > HBG_MSG_ECHO_HASH) {
        h.status = HBG_E_WIRE_TAG;
        return h;
    }
    if (h.tag >= HBG_MSG_READY) {
        if (len < 36) h.status = HBG_E_WIRE_EOF;
        return h;
    }
    if (len < 12) {
        h.status = HBG_E_WIRE_EOF;
        return h;
    }
    h.vlen = rd_le(msg + 4, 8);
    if (h.vlen > len - 12 || len - 12 - h.vlen < 16) {
        h.status = HBG_E_WIRE_EOF;
        return h;
    }
    h.trailer = 12 + h.vlen;
    h.index = rd_le(msg + h.trailer, 8);
    h.k = rd_le(msg + h.trailer + 8, 8);
    const uint64_t rest = len - h.trailer - 16;
    if (h.k > rest / 32 || rest - 32 * h.k < 32) {
        h.status = HBG_E_WIRE_EOF;
        return h;
    }
    if (h.vlen != L) h.status = HBG_E_INCORRECT_SHARD_SIZE;
    return h;
}

// grid: m messages x blocks_per_msg; thread = one 16-B chunk of the value row.
__global__ __launch_bounds__(256) void rbc_read_msgs(uint64_t L, const uint8_t* __restrict__ msgs,
                                                     const uint64_t* __restrict__ msg_off, uint64_t m,
                                                     uint32_t* __restrict__ tag_out, uint8_t* __restrict__ values,
                                                     uint64_t vstride, uint32_t* __restrict__ index_out,
                                                     uint8_t* __restrict__ digests, uint32_t depth,
                                                     uint32_t* __restrict__ ndig_out, uint8_t* __restrict__ roots,
                                                     int32_t* __restrict__ status, uint32_t blocks_per_msg) {
    const uint64_t j = blockIdx.x / blocks_per_msg;
    if (j >= m) return;
    const uint64_t start = msg_off[j], len = msg_off[j + 1] - start;
    const uint8_t* msg = msgs + start;
    __shared__ MsgHdr sh;  // parsed once per block (byte loads of a uniform header)
    if (threadIdx.x == 0) sh = parse_hdr(msg, len, L);
    __syncthreads();
    const MsgHdr h = sh;
    const uint64_t c0 = (uint64_t)(blockIdx.x % blocks_per_msg) * 256 * kChunks + threadIdx.x;
    if (c0 == 0) {
        status[j] = h.status;
        tag_out[j] = h.tag;
        const bool proof = h.tag <= HBG_MSG_ECHO && (h.status == 0 || h.status == HBG_E_INCORRECT_SHARD_SIZE);
        const bool digest = h.tag >= HBG_MSG_READY && h.tag <= HBG_MSG_ECHO_HASH && h.status == 0;
        index_out[j] = proof ? (h.index > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)h.index) : 0u;
        uint32_t nd = 0;
        if (proof) nd = h.k > depth ? 0xFFFFFFFFu : (uint32_t)h.k;  // more than any valid proof: validate -> false
        ndig_out[j] = nd;
        uint8_t* rt = roots + j * 32;
        if (proof) {
            const uint8_t* src = msg + h.trailer + 16 + 32 * h.k;
            for (int b = 0; b < 32; ++b) rt[b] = src[b];
            if (nd != 0xFFFFFFFFu)
                for (uint32_t b = 0; b < 32 * nd; ++b) digests[j * depth * 32ull + b] = msg[h.trailer + 16 + b];
        } else if (digest) {
            for (int b = 0; b < 32; ++b) rt[b] = msg[4 + b];
        } else {
            for (int b = 0; b < 32; ++b) rt[b] = 0;
        }
    }
    if (h.status != 0 || h.tag > HBG_MSG_ECHO) return;
#pragma unroll
    for (uint32_t q = 0; q < kChunks; ++q) {
        const uint64_t o = 16 * (c0 + 256 * q);  // value byte offset of this chunk
        if (o >= L) return;
        uint8_t* dst = values + j * vstride + o;
        const uint8_t* src = msg + 12 + o;
        if (o + 16 <= L) {
            *reinterpret_cast<uint4*>(dst) = load16_unaligned(src);
            continue;
        }
        for (uint64_t b = 0; o + b < L; ++b) dst[b] = src[b];
    }
}

// WireMessages::start_send framing: u32 BE (8 + len + 96) | u64 LE len |
// message | sig96 (sig from bls_sign into a [n][96] table).  One 256-thread
// block per frame, thread = one 16-B destination chunk per pass (frames are
// sized from the device offsets: no host round trip in device mode).  A frame
// whose slot size is wrong, or whose body exceeds the codec's 8 MiB limit,
// stays unwritten and flags HBG_E_ARG / HBG_E_WIRE_FRAME.
__global__ __launch_bounds__(256) void wire_frame_pack(uint64_t n, const uint8_t* __restrict__ msg,
                                                       const uint64_t* __restrict__ msg_off,
                                                       const uint8_t* __restrict__ sig96, uint8_t* __restrict__ frames,
                                                       const uint64_t* __restrict__ frame_off,
                                                       int32_t* __restrict__ err) {
    const uint64_t k = blockIdx.x;
    if (k >= n) return;
    const uint64_t len = msg_off[k + 1] - msg_off[k];
    const uint64_t start = frame_off[k], end = frame_off[k + 1];
    const uint64_t body = 8 + len + 96;
    if (msg_off[k + 1] < msg_off[k] || end < start || end - start != 12 + len + 96 || body > (uint64_t)HBG_WIRE_MAX_FRAME) {
        if (threadIdx.x == 0) flag_error(err, body > (uint64_t)HBG_WIRE_MAX_FRAME ? HBG_E_WIRE_FRAME : HBG_E_ARG);
        return;
    }
    const uint8_t* m = msg + msg_off[k];
    for (uint64_t c = threadIdx.x;; c += 256) {
        const uint64_t A = (start & ~15ull) + 16 * c;
        if (A >= end) return;
        if (A >= start + 12 && A + 16 <= start + 12 + len) {
            *reinterpret_cast<uint4*>(frames + A) = load16_unaligned(m + (A - start - 12));
            continue;
        }
        const uint64_t lo = A > start ? A : start, hi = A + 16 < end ? A + 16 : end;
        for (uint64_t b = lo; b < hi; ++b) {
            const uint64_t o = b - start;
            uint8_t v;
            if (o < 4) v = (uint8_t)(body >> (8 * (3 - o)));
            else if (o < 12) v = le_byte(len, (uint32_t)(o - 4));
            else if (o < 12 + len) v = m[o - 12];
            else v = sig96[96 * k + (o - 12 - len)];
            frames[b] = v;
        }
    }
}

hipError_t launch_wire_frame_pack(uint64_t n, const uint8_t* msg, const uint64_t* msg_off, const uint8_t* sig96,
                                  uint8_t* frames, const uint64_t* frame_off, int32_t* err, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(wire_frame_pack, dim3((uint32_t)n), dim3(256), 0, st, n, msg, msg_off, sig96, frames, frame_off,
                       err);
    return hipGetLastError();
}

hipError_t launch_rbc_write_proof_msgs(uint32_t N, uint64_t L, const uint8_t* shards, uint64_t S,
                                       const uint8_t* levels, uint64_t n, uint32_t tag, uint64_t m,
                                       const uint64_t* inst, const uint32_t* index, uint8_t* out,
                                       const uint64_t* out_off, int32_t* err, hipStream_t st) {
    if (m == 0) return hipSuccess;
    const uint64_t max_len = 12 + L + 16 + 32ull * merkle_depth(N) + 32;
    const uint32_t bpm = (uint32_t)((max_len + 32 + kBlockBytes - 1) / kBlockBytes);
    hipLaunchKernelGGL(rbc_write_proof_msgs, dim3((uint32_t)(m * bpm)), dim3(256), 0, st, N, L, shards, S, levels,
                       merkle_nodes(N), n, tag, m, inst, index, out, out_off, bpm, err);
    return hipGetLastError();
}

hipError_t launch_rbc_read_msgs(uint32_t N, uint64_t L, const uint8_t* msgs, const uint64_t* msg_off, uint64_t m,
                                uint32_t* tag, uint8_t* values, uint64_t vstride, uint32_t* index,
                                uint8_t* digests, uint32_t* ndig, uint8_t* roots, int32_t* status,
                                hipStream_t st) {
    if (m == 0) return hipSuccess;
    const uint32_t bpm = (uint32_t)((L + kBlockBytes - 1) / kBlockBytes + (L == 0 ? 1 : 0));
    hipLaunchKernelGGL(rbc_read_msgs, dim3((uint32_t)(m * (bpm ? bpm : 1))), dim3(256), 0, st, L, msgs, msg_off,
                       m, tag, values, vstride, index, digests, merkle_depth(N), ndig, roots, status,
                       bpm ? bpm : 1u);
    return hipGetLastError();
}

uint32_t host_proof_digests(uint32_t N, uint32_t i) { return proof_digests(N, i); }

}  // namespace hbg
