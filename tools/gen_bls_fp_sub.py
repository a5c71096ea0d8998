#!/usr/bin/env python3
"""Generates hydrabadger_amd/csrc/bls_fp_sub.h: BLS12-381 Montgomery
multiplication as gfx950 leaf SUBROUTINES with a fixed register interface,
and the inline-asm call wrappers fp_mul / fp_sqr / fp_mul2 / fp_mul3.

Why ("register-resident tower"): with the standard AMDGPU call
ABI every fp_mul call clobbers the ~150 caller-saved VGPRs, so only ~108
VGPRs of an Fp6 / Fp12 computation survive a call; round 3 therefore passed
Fp6 / Fp12 operands through scratch (295 KB of HBM traffic per verified
share).  Here a call is an inline-asm `s_swappc_b64` whose constraints bind the
operands to fixed VGPRs and whose clobber list names exactly the registers the
subroutine writes, so the compiler keeps everything else live across it.

Subroutine hbg_fpmul<N> (N = 1, 2, 3) computes N independent products
    R_k = X_k * Y_k * 2^-384 mod p,   k < N,
with X_k in v[24k, 24k+11], Y_k in v[24k+12, 24k+23] (12 x u32 LE limbs,
Montgomery form, < p), R_k written over X_k.  Temporaries per slot k (base
T = 24N): accumulator v[T+2k : T+2k+1], carry count v[T+2N+k], Montgomery
quotients m_k[0..11] at v[T+3N+12k ..].  SGPRs: p limbs s[64:75], -p^-1 mod
2^32 s76, carries s[78+2k : 79+2k] and s[88+2k : 89+2k] (alternating), reduction
mask s[84:85], call target s[86:87], return address s[30:31].  The N products run interleaved (product
scanning, one v_mad_u64_u32 + carry count per partial product): with N = 3
a carry SGPR is read two instructions after its write, so no wait states are
spent and a lone wave per SIMD still issues back to back (three independent
chains) — fp2_mul's three Karatsuba products are one hbg_fpmul3 call.

Hazards (gfx950): a VALU write of an SGPR read back by a VALU (carry-in)
needs 2 wait states; the emitter tracks every SGPR pair and pads with s_nop.

    python tools/gen_bls_fp_sub.py
"""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
P_LIMBS = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(12)]
N0 = (-pow(P, -1, 1 << 32)) % (1 << 32)
assert N0 == 0xFFFCFFFD

S_P = 64        # s[64:75] modulus limbs
S_N0 = 76
S_CARRY = 78    # s[78+2k : 79+2k]
S_MASK = 84     # s[84:85]
S_TGT = 86      # s[86:87] call target
S_CARRY2 = 88   # s[88+2k : 89+2k]: the second carry set (partial products alternate sets)
VALU_SGPR_WAIT = 2  # wait states between a VALU SGPR write and a VALU read of it
PIPELINE = True     # --no-pipeline: count each product's carries right after its mads (round 3's order)


class Emitter:
    def __init__(self):
        self.lines: list[str] = []
        self.pos = 0                 # wait-state position
        self.sgpr_w: dict[int, int] = {}  # sgpr pair base -> position of the last VALU write

    def _need(self, reads):
        wait = 0
        for s in reads:
            if s in self.sgpr_w:
                d = self.pos - self.sgpr_w[s] - 1
                wait = max(wait, VALU_SGPR_WAIT - d)
        if wait > 0:
            self.lines.append(f"s_nop {wait - 1}")
            self.pos += wait

    def valu(self, text, reads=(), writes=()):
        self._need(reads)
        self.lines.append(text)
        for s in writes:
            self.sgpr_w[s] = self.pos
        self.pos += 1

    def salu(self, text):
        self.lines.append(text)
        self.pos += 1

    def nop(self, k):
        self.lines.append(f"s_nop {k}")
        self.pos += k + 1


def v(i):
    return f"v{i}"


def vp(i):
    return f"v[{i}:{i + 1}]"


def sp(i):
    return f"s[{i}:{i + 1}]"


def regs(N):
    T = 24 * N
    slots = []
    for k in range(N):
        slots.append({
            "x": 24 * k, "y": 24 * k + 12,
            "acc": T + 2 * k, "t2": T + 2 * N + k, "m": T + 3 * N + 12 * k,
            "sc": S_CARRY + 2 * k, "sc2": S_CARRY2 + 2 * k,
        })
    return slots, 39 * N


def gen_sub(N: int) -> str:
    slots, nv = regs(N)
    e = Emitter()
    for i in range(12):
        e.salu(f"s_mov_b32 s{S_P + i}, 0x{P_LIMBS[i]:08x}")
    e.salu(f"s_mov_b32 s{S_N0}, 0x{N0:08x}")
    for s in slots:
        e.valu(f"v_mov_b32 {v(s['acc'])}, 0")
        e.valu(f"v_mov_b32 {v(s['acc'] + 1)}, 0")
        e.valu(f"v_mov_b32 {v(s['t2'])}, 0")

    def mac(prods):
        """prods: list of (xkind, xi, ykind, yi); kinds 'x' | 'y' | 'm' | 'p'.

        Software-pipelined carry counts: partial product q's carries go to
        carry set q % 2 and are counted (v_addc into t2) after product q+1's
        mads, so a carry SGPR is read 2N instructions after its write instead
        of N (a lone wave's mad -> addc latency), and the two sets never
        overlap.  The last product's counts are drained at the end."""
        def carry(s, cs):
            return s["sc"] if cs == 0 else s["sc2"]

        def counts(cs):
            for s in slots:
                c = carry(s, cs)
                e.valu(f"v_addc_co_u32_e64 {v(s['t2'])}, {sp(c)}, {v(s['t2'])}, 0, {sp(c)}",
                       reads=(c,), writes=(c,))

        pending = None
        for q, (xk, xi, yk, yi) in enumerate(prods):
            cs = q % 2 if PIPELINE else 0
            for s in slots:
                def op(kind, i):
                    if kind == "p":
                        return f"s{S_P + i}"
                    return v(s[kind] + i)
                c = carry(s, cs)
                e.valu(f"v_mad_u64_u32 {vp(s['acc'])}, {sp(c)}, {op(xk, xi)}, {op(yk, yi)}, {vp(s['acc'])}",
                       writes=(c,))
            if pending is not None:
                counts(pending)
            pending = cs
            if not PIPELINE:
                counts(cs)
                pending = None
        if pending is not None:
            counts(pending)

    for i in range(24):
        prods = []
        lo = 0 if i < 12 else i - 11
        hi = i if i < 12 else 11
        for j in range(lo, hi + 1):
            if i < 12 and j == i:
                continue
            prods.append(("x", j, "y", i - j))
            if i >= 12 or j < i:
                prods.append(("m", j, "p", i - j))
        if i < 12:
            prods.append(("x", i, "y", 0))
        mac(prods)
        if i < 12:
            for s in slots:
                e.valu(f"v_mul_lo_u32 {v(s['m'] + i)}, {v(s['acc'])}, s{S_N0}")
            mac([("m", i, "p", 0)])
        else:
            for s in slots:
                e.valu(f"v_mov_b32 {v(s['x'] + i - 12)}, {v(s['acc'])}")
        for s in slots:
            e.valu(f"v_mov_b32 {v(s['acc'])}, {v(s['acc'] + 1)}")
            e.valu(f"v_mov_b32 {v(s['acc'] + 1)}, {v(s['t2'])}")
            e.valu(f"v_mov_b32 {v(s['t2'])}, 0")
    # r = (o + carry * 2^384) >= p ? o - p : o, with the carry word in acc.lo;
    # p is copied into the (dead) quotient registers, which then hold o - p
    for s in slots:
        for i in range(12):
            e.valu(f"v_mov_b32 {v(s['m'] + i)}, s{S_P + i}")
    for i in range(12):
        for s in slots:
            if i == 0:
                e.valu(f"v_sub_co_u32_e64 {v(s['m'])}, {sp(s['sc'])}, {v(s['x'])}, {v(s['m'])}",
                       writes=(s["sc"],))
            else:
                e.valu(f"v_subb_co_u32_e64 {v(s['m'] + i)}, {sp(s['sc'])}, {v(s['x'] + i)}, {v(s['m'] + i)}, "
                       f"{sp(s['sc'])}", reads=(s["sc"],), writes=(s["sc"],))
    for s in slots:
        e.valu(f"v_cmp_ne_u32_e64 {sp(S_MASK)}, 0, {v(s['acc'])}", writes=(S_MASK,))
        e.nop(4)
        e.salu(f"s_orn2_b64 {sp(S_MASK)}, {sp(S_MASK)}, {sp(s['sc'])}")  # carry | no borrow
        e.nop(4)
        for i in range(12):
            e.valu(f"v_cndmask_b32_e64 {v(s['x'] + i)}, {v(s['x'] + i)}, {v(s['m'] + i)}, {sp(S_MASK)}")
    e.salu("s_setpc_b64 s[30:31]")
    body = "\n".join("\t" + ln for ln in e.lines)
    return f"\t.p2align 6\n\t.hidden hbg_fpmul{N}\n\t.globl hbg_fpmul{N}\nhbg_fpmul{N}:\n{body}\n", nv


def clobbers(N: int, nv: int) -> str:
    # VGPRs the subroutine writes besides the outputs X_k: all temporaries
    vs = [f'"v{i}"' for i in range(24 * N, nv)]
    top = S_CARRY2 + 6 if PIPELINE else S_TGT + 2
    ss = [f'"s{i}"' for i in range(S_P, top)] + ['"s30"', '"s31"', '"scc"']
    return ", ".join(vs + ss)


OUT = None


def main():
    subs, cl = [], {}
    for N in (1, 2, 3):
        s, nv = gen_sub(N)
        subs.append(s)
        cl[N] = clobbers(N, nv)
        n_mad = s.count("v_mad_u64_u32")
        n_all = len([ln for ln in s.split("\n") if ln.startswith("\t") and not ln.startswith("\t.")])
        print(f"hbg_fpmul{N}: {n_all} instructions, {n_mad} v_mad_u64_u32, {s.count('s_nop')} s_nop, {nv} VGPRs")
    call = (r'"s_getpc_b64 s[86:87]\n\ts_add_u32 s86, s86, " SUB "@rel32@lo+4\n\t'
            r's_addc_u32 s87, s87, " SUB "@rel32@hi+12\n\ts_swappc_b64 s[30:31], s[86:87]"')
    out = [
        "// Generated by tools/gen_bls_fp_sub.py — do not edit.\n",
        "// BLS12-381 Montgomery multiplication as fixed-register gfx950 subroutines\n",
        "// (hbg_fpmul1/2/3: 1, 2 or 3 interleaved products) and their call wrappers.\n",
        "// Interface and rationale: the generator's docstring and DESIGN.md §4.\n",
        "#pragma once\n#include <hip/hip_runtime.h>\n#include <stdint.h>\n\n",
        "namespace hbg {\nnamespace bls {\n\n",
        "typedef uint32_t Fp __attribute__((ext_vector_type(12)));\n\n",
        "// The subroutine bodies: never called as a function; the labels inside are\n",
        "// the entry points (hidden, so the kernels' rel32 calls resolve at link time).\n",
        "__device__ __noinline__ __attribute__((used)) void hbg_fp_subroutines() {\n",
        "    asm volatile(R\"(\n",
        "".join(subs),
        ")\");\n}\n\n",
        "#define HBG_FP_SUB_CALL(SUB) " + call + "\n",
        f"#define HBG_FP_SUB1_CLOBBERS {cl[1]}\n",
        f"#define HBG_FP_SUB2_CLOBBERS {cl[2]}\n",
        f"#define HBG_FP_SUB3_CLOBBERS {cl[3]}\n\n",
        "}  // namespace bls\n}  // namespace hbg\n",
    ]
    path = OUT or os.path.join(ROOT, "hydrabadger_amd", "csrc", "bls_fp_sub.h")
    with open(path, "w") as f:
        f.write("".join(out))
    print(path)


if __name__ == "__main__":
    import sys
    OUT = None
    if "--no-pipeline" in sys.argv:
        PIPELINE = False
    if "--out" in sys.argv:
        OUT = sys.argv[sys.argv.index("--out") + 1]
    main()
