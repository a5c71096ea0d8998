// tdec_kernels_lat.hip — the latency build of the BLS12-381 kernels: the same
// source as tdec_kernels.hip compiled into namespace hbg::bls_lat with a
// one-wave-per-SIMD register budget for EVERY kernel (the throughput build
// gives it only to the pairing / G2 kernels).  tdec_kernels.hip's launchers
// hand launches of at most g_lat_lanes lanes to these kernels (DESIGN.md §4,
// "latency build").
// one wave per SIMD: the latency build takes launches of at most one wave per
// SIMD, so every kernel gets the whole register file (fewer scratch spills)
#define HBG_TDEC_WPE 1
#define HBG_TDEC_LAT_TU 1
#define bls bls_lat
#include "tdec_kernels.hip"
