// ubench.hip — gfx950 VALU issue-rate microbenchmarks for the integer ops the
// Keccak / GF(2^8) kernels are built from, plus the in-kernel clock
// (s_memtime / s_memrealtime, MI355X_MICROARCH.md 'DVFS give-back' item 6).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench tools/ubench.hip && tools/ubench
//
// Each kernel runs 8 independent dependency chains per lane (ILP 8) so the
// issue rate, not the dependent latency, is measured.  Reported: cycles per
// wave64 instruction per SIMD = (clock * time * SIMDs) / (instructions issued).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
#define CH 8

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t err_ = (x);                                                       \
        if (err_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t* out, uint32_t seed, uint64_t* clk) {
    uint32_t a[CH], b = seed ^ threadIdx.x, c = seed * 3 + blockIdx.x;
    uint64_t m[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        a[i] = seed + i * 77 + threadIdx.x;
        m[i] = a[i];
    }
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
            if constexpr (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b));
            if constexpr (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if constexpr (OP == 4) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(m[i]) : "v"(b), "v"(c) : "vcc");
            if constexpr (OP == 5) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if constexpr (OP == 6) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if constexpr (OP == 7) asm volatile("v_alignbit_b32 %0, %1, %0, 7" : "+v"(a[i]) : "v"(b));
            if constexpr (OP == 8) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if constexpr (OP == 10) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if constexpr (OP == 11) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a[i]) : "v"(b));
            if constexpr (OP == 9) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) s ^= a[i] ^ (uint32_t)m[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int OP>
int run(const char* name, int insts_per_chain_step, int blocks_per_cu, uint32_t* out, uint64_t* clk) {
    int dev = 0;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, dev));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * blocks_per_cu;
    hipEvent_t s, e;
    CHECK(hipEventCreate(&s));
    CHECK(hipEventCreate(&e));
    k_op<OP><<<blocks, 256>>>(out, 1, clk);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(s));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) k_op<OP><<<blocks, 256>>>(out, r + 2, clk);
    CHECK(hipEventRecord(e));
    CHECK(hipEventSynchronize(e));
    float ms;
    CHECK(hipEventElapsedTime(&ms, s, e));
    uint64_t hc[2];
    CHECK(hipMemcpy(hc, clk, sizeof hc, hipMemcpyDeviceToHost));
    const double ghz = (double)hc[0] / (double)hc[1] * 0.1;  // memrealtime = 100 MHz
    const double waves = (double)blocks * 4 * reps;
    const double insts = waves * ITERS * CH * insts_per_chain_step;
    const double simds = cus * 4.0;
    const double cyc_per_inst = (ms * 1e-3) * ghz * 1e9 * simds / insts;
    const double lane_ops = insts * 64 / (ms * 1e-3);
    printf("%-16s waves/SIMD=%d  %.3f ms  clock %.3f GHz  %.2f cyc/wave-inst/SIMD  %.1f Tlane-op/s\n", name,
           blocks_per_cu, ms / reps, ghz, cyc_per_inst, lane_ops / 1e12);
    return 0;
}

int main() {
    uint32_t* out;
    uint64_t* clk;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    printf("device %s CUs=%d clock(prop)=%d kHz\n", p.name, p.multiProcessorCount, p.clockRate);
    CHECK(hipMalloc(&out, sizeof(uint32_t) * 256 * p.multiProcessorCount * 8));
    CHECK(hipMalloc(&clk, 16));
    for (int w : {1, 2, 4, 8}) {
        run<0>("xor(VOP2)", 1, w, out, clk);
        run<1>("bitop3", 1, w, out, clk);
        run<2>("alignbit", 1, w, out, clk);
        run<3>("add_u32", 1, w, out, clk);
    }
    run<4>("mad_u64_u32", 1, 4, out, clk);
    run<5>("mul_lo_u32", 1, 4, out, clk);
    run<6>("perm_b32", 1, 4, out, clk);
    run<7>("alignbit(b,a)", 1, 4, out, clk);
    run<8>("xor_e64", 1, 4, out, clk);
    run<10>("add3_u32", 1, 4, out, clk);
    run<11>("bitop3(2 regs)", 1, 4, out, clk);
    run<9>("mul_hi_u32", 1, 4, out, clk);
    return 0;
}
