// ubench6 — issue rate of the fixed-register Montgomery subroutines
// (bls_fp_sub.h: hbg_fpmul1 / hbg_fpmul3) at one and two waves per SIMD.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++20 -I hydrabadger_amd/csrc tools/ubench6.hip -o tools/ubench6
//   ./tools/ubench6            # one JSON line per probe
//
// Each lane runs a dependent chain of `reps` calls (mul1: one product per
// call; mul3: three independent products per call); the grid is one (WPE 1)
// or two (WPE 2) waves per SIMD on the 1,024 SIMDs.  Reported: products per
// second chip-wide and wave-cycles per product at the 2.4 GHz nominal clock.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "bls.h"

using namespace hbg::bls;

#define PROBE(NAME, WPE, BODY)                                                                              \
    __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void NAME(uint32_t* out,     \
                                                                                        uint32_t reps) {    \
        const uint32_t g = blockIdx.x * 64 + threadIdx.x;                                                   \
        Fp a, b, c, x, y, z;                                                                                \
        for (int i = 0; i < 12; ++i) {                                                                      \
            a[i] = (g * 2654435761u + i) & 0x0FFFFFFFu;                                                     \
            b[i] = a[i] ^ 0x1234567u;                                                                       \
            c[i] = a[i] ^ 0x7654321u;                                                                       \
            x[i] = (i * 77u + 5u) & 0x0FFFFFFFu;                                                            \
            y[i] = x[i] ^ 0x2468ACEu;                                                                       \
            z[i] = x[i] ^ 0x1357BDFu;                                                                       \
        }                                                                                                   \
        for (uint32_t r = 0; r < reps; ++r) { BODY; }                                                       \
        uint32_t h = 0;                                                                                     \
        for (int i = 0; i < 12; ++i) h ^= a[i] ^ b[i] ^ c[i];                                               \
        out[g] = h;                                                                                         \
    }

PROBE(mul1_w1, 1, a = fp_mul(a, x))
PROBE(mul1_w2, 2, a = fp_mul(a, x))
PROBE(mul3_w1, 1, fp_mul3(a, b, c, a, x, b, y, c, z))
PROBE(mul3_w2, 2, fp_mul3(a, b, c, a, x, b, y, c, z))

int main() {
    uint32_t* out;
    if (hipMalloc(&out, 2048 * 64 * sizeof(uint32_t)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct P {
        const char* name;
        void (*k)(uint32_t*, uint32_t);
        int waves_per_simd, products_per_call;
    } probes[] = {{"mul1", mul1_w1, 1, 1}, {"mul1", mul1_w2, 2, 1}, {"mul3", mul3_w1, 1, 3}, {"mul3", mul3_w2, 2, 3}};
    const uint32_t reps = 2000;
    for (const P& p : probes) {
        const uint32_t blocks = 1024u * p.waves_per_simd;
        p.k<<<blocks, 64>>>(out, 16);  // warm
        (void)hipEventRecord(e0);
        p.k<<<blocks, 64>>>(out, reps);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double products = (double)blocks * 64 * reps * p.products_per_call;
        const double per_s = products / (ms * 1e-3);
        // wave-cycles per product on one SIMD: SIMD-cycles / (products per SIMD / 64 lanes)
        const double cyc = 2.4e9 * ms * 1e-3 / ((double)p.waves_per_simd * reps * p.products_per_call);
        printf("{\"probe\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"G_products_per_s\": %.2f, "
               "\"simd_cycles_per_wave_product\": %.0f}\n",
               p.name, p.waves_per_simd, ms, per_s / 1e9, cyc);
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
