// tdec_kernels_lat.hip — the latency build of the BLS12-381 kernels: the same
// source as tdec_kernels.hip compiled into namespace hbg::bls_lat with three
// interleaved accumulators per Fp multiplication column (HBG_FP_LAT,
// bls_fp_mul.h) and a one-wave-per-SIMD register budget.  tdec_kernels.hip's launchers hand launches of at most
// kLatLanes lanes to these kernels ("latency build").
#define HBG_FP_LAT 1
// one wave per SIMD: the latency build takes launches of at most one wave per
// SIMD, so every kernel gets the whole register file (fewer scratch spills)
#define HBG_TDEC_WPE 1
#define HBG_TDEC_LAT_TU 1
#define bls bls_lat
#include "tdec_kernels.hip"
