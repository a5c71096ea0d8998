#!/usr/bin/env python3
"""Generates hydrabadger_amd/csrc/keccak_asm.h: Keccak-f[1600] as one inline-asm
block with a hand-placed VGPR layout for gfx950.

Why: on gfx950 `v_bitop3_b32` issues at full rate (2.34 cyc/wave-instr) only
when its three VGPR sources sit in distinct register banks (index mod 4) and at
3.8-4.3 cyc otherwise; `v_alignbit_b32` is half rate regardless
(profiles/r01/ubench2.txt).  The compiler does not bank-allocate, so the
compiled round ran at ~4.2 cyc/instr.  This layout makes every bitop3
conflict-free except one chi per row-half (a 5-cycle of consecutive triples
cannot be 3-coloured distinctly with 4 banks).

Round (x, y lane coordinates, lane L = x + 5y, each lane = lo/hi VGPR pair):
  C[x]   = A[x,0]^A[x,1]^A[x,2] (bitop3) ^ A[x,3]^A[x,4] (bitop3)   banks(A[x,y]) = (x+y) mod 4
  D[x]   = C[x-1] ^ rotl1(C[x+1])          2 alignbit + 2 xor per column
  A[L]  ^= D[x]                            VOP2 xor (no bank constraint)
  B[y, 2x+3y] = rotl(A[x,y], r[x,y])       2 alignbit (B[0,0] aliases A[0,0])
  A[x,y] = B[x,y] ^ (~B[x+1,y] & B[x+2,y]) bitop3, banks(B[., y]) = [0,1,2,3,1] + y
  A[0,0] ^= RC[round]                       SGPR operands from a constant table
24 rounds run as a scalar loop inside the asm (one round body in the
I-cache).  Register budget: 50 A + 48 B (theta temporaries reuse B registers) = 98.
    python tools/gen_keccak_asm.py
"""
from __future__ import annotations

import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# option: rho rotations by a multiple of 8 (56 and 8: four funnel shifts a round) as
# v_perm_b32 instead of the half-rate v_alignbit_b32
BYTE_PERM = os.environ.get("KECCAK_BYTE_PERM", "0") == "1"  # measured slower (r05c1): off

ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61], [28, 55, 25, 21, 56], [27, 20, 39, 8, 14]]
# ROT[x][y]


class Alloc:
    def __init__(self, start=0):
        self.used = set()
        self.start = start

    def take(self, bank):
        i = self.start
        while True:
            if i % 4 == bank and i not in self.used:
                self.used.add(i)
                return i
            i += 1


def layout(hshift: int = 0):
    """Returns (round body lines, A[x][y][h] register map, registers used).
    hshift: bank offset of a lane's hi word relative to its lo word (2 puts
    the two halves in different banks, so the rho v_alignbit reading both
    halves has no source bank conflict)."""
    al = Alloc(0)
    # A[x][y][h]: bank (x + y) mod 4 — column triples y=0,1,2 distinct, y=3,4
    # distinct, partial-C bank free; spreads the state evenly over the banks
    A = [[[al.take((x + y + hshift * h) % 4) for h in range(2)] for y in range(5)] for x in range(5)]
    bbank = [0, 1, 2, 3, 1]  # per row, rotated by y below
    B = [[[None, None] for y in range(5)] for x in range(5)]
    for x in range(5):
        for y in range(5):
            for h in range(2):
                if x == 0 and y == 0:
                    B[x][y][h] = A[0][0][h]  # alias (rotation 0)
                else:
                    B[x][y][h] = al.take((bbank[x] + y + hshift * h) % 4)
    # theta temporaries live only before B is written: they reuse B registers.
    pool = [B[x][y][h] for x in range(5) for y in range(5) for h in range(2) if not (x == 0 and y == 0)]

    def from_pool(banks, avoid):
        for r in pool:
            if r % 4 in banks and r not in avoid:
                avoid.add(r)
                return r
        raise RuntimeError("pool exhausted")

    taken = set()
    Cp = [[from_pool({(x + 1 + hshift * h) % 4, (x + 2 + hshift * h) % 4}, taken) for h in range(2)]
          for x in range(5)]  # partial C
    C = [[from_pool({0, 1, 2, 3} if not hshift else {(2 * h) % 4, (2 * h + 1) % 4}, taken) for h in range(2)]
         for x in range(5)]
    T = [[from_pool({0, 1, 2, 3}, taken), from_pool({0, 1, 2, 3}, taken)] for x in range(5)]
    D = Cp  # D is written after Cp is dead (no bank constraint on D)
    regs_used = sorted(al.used)
    nreg = max(regs_used) + 1

    def v(i):
        return f"v{i}"

    L = []
    # theta: column parities
    for x in range(5):
        for h in range(2):
            L.append(f"v_bitop3_b32 {v(Cp[x][h])}, {v(A[x][0][h])}, {v(A[x][1][h])}, {v(A[x][2][h])} bitop3:0x96")
    for x in range(5):
        for h in range(2):
            L.append(f"v_bitop3_b32 {v(C[x][h])}, {v(Cp[x][h])}, {v(A[x][3][h])}, {v(A[x][4][h])} bitop3:0x96")
    # D[x] = C[x-1] ^ rotl1(C[x+1]);  rotl1(lo, hi) = (alignbit(lo, hi, 31), alignbit(hi, lo, 31))
    for x in range(5):
        c1 = C[(x + 1) % 5]
        c0 = C[(x + 4) % 5]
        L.append(f"v_alignbit_b32 {v(T[x][0])}, {v(c1[0])}, {v(c1[1])}, 31")
        L.append(f"v_alignbit_b32 {v(T[x][1])}, {v(c1[1])}, {v(c1[0])}, 31")
        L.append(f"v_xor_b32 {v(D[x][0])}, {v(c0[0])}, {v(T[x][0])}")
        L.append(f"v_xor_b32 {v(D[x][1])}, {v(c0[1])}, {v(T[x][1])}")
    # theta apply + rho + pi
    for x in range(5):
        for y in range(5):
            for h in range(2):
                L.append(f"v_xor_b32 {v(A[x][y][h])}, {v(A[x][y][h])}, {v(D[x][h])}")
    for x in range(5):
        for y in range(5):
            r = ROT[x][y]
            dx, dy = y, (2 * x + 3 * y) % 5
            lo, hi = A[x][y]
            blo, bhi = B[dx][dy]
            if r == 0:
                continue  # B[0,0] aliases A[0,0]
            amt = 32 - r if r < 32 else 64 - r
            if BYTE_PERM and amt % 8 == 0 and r != 32:
                # a byte-multiple funnel shift as a full-rate v_perm_b32
                # (selector from an SGPR: no VOP3 literal on gfx9)
                s0, s1 = (lo, hi) if r < 32 else (hi, lo)
                L.append(f"v_perm_b32 {v(blo)}, {v(s0)}, {v(s1)}, %[p{amt}]")
                L.append(f"v_perm_b32 {v(bhi)}, {v(s1)}, {v(s0)}, %[p{amt}]")
                continue
            if r < 32:
                L.append(f"v_alignbit_b32 {v(blo)}, {v(lo)}, {v(hi)}, {32 - r}")
                L.append(f"v_alignbit_b32 {v(bhi)}, {v(hi)}, {v(lo)}, {32 - r}")
            elif r == 32:
                L.append(f"v_mov_b32 {v(blo)}, {v(hi)}")
                L.append(f"v_mov_b32 {v(bhi)}, {v(lo)}")
            else:
                L.append(f"v_alignbit_b32 {v(blo)}, {v(hi)}, {v(lo)}, {64 - r}")
                L.append(f"v_alignbit_b32 {v(bhi)}, {v(lo)}, {v(hi)}, {64 - r}")
    # chi, row by row; row 0 writes A[0,0] (aliasing B[0,0]) last
    for y in range(5):
        order = [1, 2, 3, 4, 0] if y == 0 else [0, 1, 2, 3, 4]
        for x in order:
            for h in range(2):
                a, b, c = B[x][y][h], B[(x + 1) % 5][y][h], B[(x + 2) % 5][y][h]
                # a ^ (~b & c): truth table over (S0=a, S1=b, S2=c) with index (a<<2)|(b<<1)|c
                L.append(f"v_bitop3_b32 {v(A[x][y][h])}, {v(a)}, {v(b)}, {v(c)} bitop3:0xd2")
    return L, A, sorted(al.used)


def _parse(line):
    op, rest = line.split(None, 1)
    regs = [t.strip() for t in rest.split(" bitop3")[0].split(",")]
    regs = [int(t[1:]) for t in regs if t.startswith("v")]
    return op, regs[0], regs[1:]


def schedule(lines, lat=2, gap=2):
    """Greedy list schedule of one round: spreads the half-rate v_alignbit ops
    between full-rate ops (at most one alignbit per `gap` full-rate ops when
    both are ready) and keeps `lat` slots between a producer and its consumer
    where possible; ties broken by critical-path length.  Register RAW/WAR/WAW
    dependencies are preserved exactly."""
    n = len(lines)
    info = [_parse(x) for x in lines]
    preds = [set() for _ in range(n)]
    raw = [set() for _ in range(n)]
    last_w, readers = {}, {}
    for i, (op, d, srcs) in enumerate(info):
        for r in srcs:
            if r in last_w:
                preds[i].add(last_w[r])
                raw[i].add(last_w[r])
        for j in readers.get(d, []):
            if j != i:
                preds[i].add(j)
        if d in last_w:
            preds[i].add(last_w[d])
        for r in srcs:
            readers.setdefault(r, []).append(i)
        last_w[d] = i
        readers[d] = []
    succs = [[] for _ in range(n)]
    for i in range(n):
        for j in preds[i]:
            succs[j].append(i)
    half = [info[i][0] == "v_alignbit_b32" for i in range(n)]
    cp = [0] * n
    for i in reversed(range(n)):
        w = 2 if half[i] else 1
        cp[i] = w + max((cp[j] for j in succs[i]), default=0)
    done_at = {}
    out = []
    since_half = gap
    remaining = set(range(n))
    t = 0
    while remaining:
        ready = [i for i in remaining if all(p in done_at for p in preds[i])]
        def key(i):
            stall = any(t - done_at[p] < lat for p in raw[i])
            want_half = since_half >= gap
            cls = 0 if half[i] == want_half else 1
            return (stall, cls, -cp[i], i)
        i = min(ready, key=key)
        out.append(lines[i])
        done_at[i] = t
        remaining.discard(i)
        since_half = 0 if half[i] else since_half + 1
        t += 1
    return out


def main():
    L, A, regs_used = layout()
    if os.environ.get("KECCAK_SCHED", "0") == "1":  # measured no faster: off
        L = schedule(L)
    nreg = max(regs_used) + 1

    def v(i):
        return f"v{i}"

    # iota: RC from the scalar table, loop control
    body = "\\n\\t".join(L)
    asm_lines = [
        "s_mov_b32 %[cnt], 0",
        ".Lkround%=:",
        "s_load_dword %[rl], %[tab], %[cnt]",
        "s_load_dword %[rh], %[tab4], %[cnt]",
        body,
        "s_waitcnt lgkmcnt(0)",
        f"v_xor_b32 {v(A[0][0][0])}, %[rl], {v(A[0][0][0])}",
        f"v_xor_b32 {v(A[0][0][1])}, %[rh], {v(A[0][0][1])}",
        "s_add_u32 %[cnt], %[cnt], 8",
        "s_cmp_lg_u32 %[cnt], 192",
        "s_cbranch_scc1 .Lkround%=",
    ]
    # operands: state pinned to its registers
    outs = []
    for x in range(5):
        for y in range(5):
            L_ = x + 5 * y
            outs.append(f'"+{{{v(A[x][y][0])}}}"(a[{L_}].lo)')
            outs.append(f'"+{{{v(A[x][y][1])}}}"(a[{L_}].hi)')
    state_regs = {A[x][y][h] for x in range(5) for y in range(5) for h in range(2)}
    clob = [f'"{v(i)}"' for i in regs_used if i not in state_regs]
    asm_text = "\\n\\t".join(asm_lines)
    perm_ops = ', [p8] "s"(0x04030201u), [p24] "s"(0x06050403u)' if BYTE_PERM else ""
    hdr = f"""// Generated by tools/gen_keccak_asm.py — do not edit.
// Keccak-f[1600] for gfx950 with a bank-conflict-aware VGPR layout (see the
// generator's docstring).  Uses v0..v{nreg - 1}; state pinned to fixed VGPRs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keccak.h"

namespace hbg {{

// 24 x (RC lo, RC hi) for the scalar loads inside the asm loop
__device__ __constant__ static const uint32_t kKeccakRC_asm[48] = {{
    0x00000001u, 0x00000000u, 0x00008082u, 0x00000000u, 0x0000808au, 0x80000000u, 0x80008000u, 0x80000000u,
    0x0000808bu, 0x00000000u, 0x80000001u, 0x00000000u, 0x80008081u, 0x80000000u, 0x00008009u, 0x80000000u,
    0x0000008au, 0x00000000u, 0x00000088u, 0x00000000u, 0x80008009u, 0x00000000u, 0x8000000au, 0x00000000u,
    0x8000808bu, 0x00000000u, 0x0000008bu, 0x80000000u, 0x00008089u, 0x80000000u, 0x00008003u, 0x80000000u,
    0x00008002u, 0x80000000u, 0x00000080u, 0x80000000u, 0x0000800au, 0x00000000u, 0x8000000au, 0x80000000u,
    0x80008081u, 0x80000000u, 0x00008080u, 0x80000000u, 0x80000001u, 0x00000000u, 0x80008008u, 0x80000000u}};

__device__ __forceinline__ void keccak_f_asm(u64p (&a)[25]) {{
    uint32_t cnt, rl, rh;
    const uint32_t* tab = kKeccakRC_asm;
    const uint32_t* tab4 = kKeccakRC_asm + 1;
    asm volatile("{asm_text}"
        : {", ".join(outs)}, [cnt] "=&s"(cnt), [rl] "=&s"(rl), [rh] "=&s"(rh)
        : [tab] "s"(tab), [tab4] "s"(tab4){perm_ops}
        : {", ".join(clob)}, "scc", "memory");
}}

template <>
__device__ __forceinline__ void perm<1>(u64p (&a)[25]) {{
    keccak_f_asm(a);
}}

}}  // namespace hbg
"""
    path = os.path.join(ROOT, "hydrabadger_amd", "csrc", "keccak_asm.h")
    with open(path, "w") as f:
        f.write(hdr)
    print(path, "vgprs", nreg)


if __name__ == "__main__":
    main()
