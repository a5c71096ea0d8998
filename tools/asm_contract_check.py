#!/usr/bin/env python3
"""Static check of the fixed-register multiplication contract (bls.h /
bls_fp_sub.h; DESIGN.md §4 "The HBG_FP_COUNT fault") over gfx950 assembly.

    hipcc ... --cuda-device-only -S hydrabadger_amd/csrc/tdec_kernels.hip -o t.s
    python tools/asm_contract_check.py t.s [--only NAME]

For every function of the file it builds the control-flow graph (labels,
s_branch / s_cbranch_*, s_setpc / s_endpgm), computes backward liveness of
every VGPR, SGPR and SCC, and reports

  * each inline-asm call of a subroutine hbg_fpmul<N> after which a register
    of its clobber set (the temporaries v[24N, 39N), s[64, 94), s30/s31,
    SCC) is live — a value the compiler expects to survive the call;
  * each real call (s_swappc to a function of the file) after which a
    register the callee writes — transitively, its own callees' and its
    subroutine calls' clobbers included, minus what its prologue saves and
    its epilogue restores — is live (the interprocedural clobber masks the
    compiler uses for internal functions).

AGPRs (a0..a255, the compiler's VGPR spill space on gfx950) are tracked like
VGPRs (round 6).  Register-level only: lanes are not modelled (a VALU write under a partial
EXEC is taken as a whole-register definition, v_writelane as a partial one).
Exit status 1 if anything is reported.
"""
from __future__ import annotations

import argparse
import re
import sys

CLOB_V = {1: range(24, 39), 2: range(48, 78), 3: range(72, 117)}
CLOB_S = set(range(64, 94)) | {30, 31}
SCC = ("c", 0)

_SCC_W = re.compile(r"^s_(add|sub|addc|subb|and|or|xor|andn2|orn2|nand|nor|xnor|lshl|lshr|ashr|bfe|cmp|bitcmp|abs|min|"
                    r"max|not|bcnt|quadmask|wqm|absdiff)")
_SCC_R = re.compile(r"^s_(cbranch_scc|cselect|addc|subb|cmov)")
_NODEF = re.compile(r"^(s_cbranch|s_branch|s_waitcnt|s_nop|s_endpgm|s_setpc|global_store|flat_store|scratch_store|"
                    r"buffer_store|ds_write|global_atomic|s_cmp|v_cmp_|s_bitcmp|v_cmpx)")
_TWO_DST = re.compile(r"v_(mad_u64_u32|mad_i64_i32|add_co_u32_e64|sub_co_u32_e64|subrev_co_u32_e64|addc_co_u32_e64|"
                      r"subb_co_u32_e64|subbrev_co_u32_e64)")


def regs(tok: str) -> list:
    out = []
    for m in re.finditer(r"\b(vcc|vcc_lo|vcc_hi|m0)\b", tok):  # named registers a call may clobber
        out.append(("n", {"vcc_lo": "vcc", "vcc_hi": "vcc"}.get(m.group(1), m.group(1))))
    for m in re.finditer(r"\b([vsa])(\d+)\b|\b([vsa])\[(\d+):(\d+)\]", tok):
        if m.group(1):
            out.append((m.group(1), int(m.group(2))))
        else:
            out += [(m.group(3), i) for i in range(int(m.group(4)), int(m.group(5)) + 1)]
    return out


def parse(line: str):
    """(op, defs, uses) of one instruction line, or None."""
    t = line.split(";")[0].strip()
    if not t or t.startswith(".") or t.endswith(":"):
        return None
    op, _, rest = t.partition(" ")
    args = [a.strip() for a in rest.split(",")] if rest else []
    if op == "v_writelane_b32":  # one lane: a partial definition, the register stays live above it
        d, u = regs(args[0]), regs(",".join(args))
    elif op.startswith(("global_atomic", "flat_atomic", "buffer_atomic")) and re.search(r"\b(sc0|glc)\b", rest):
        d, u = regs(args[0]), regs(",".join(args[1:]))  # a returning atomic writes its first operand
    elif _NODEF.match(op):
        d, u = [], regs(rest)
        if op.startswith("v_cmp_") and ("_e64" in op or (args and args[0] in ("vcc", "vcc_lo"))):
            d, u = regs(args[0]), regs(",".join(args[1:]))
    else:
        nd = 2 if _TWO_DST.match(op) else 1
        d, u = regs(",".join(args[:nd])), regs(",".join(args[nd:]))
    if op.endswith("_e32") and len(args) >= 2 and args[1] == "vcc" and "_co_" in op:
        # VOP2 carry ops: the second operand is the carry-out (a def); a carry-in is the last operand
        d = list(d) + [("n", "vcc")]
        u = [r for r in u if r != ("n", "vcc")] + ([("n", "vcc")] if args[-1] == "vcc" and len(args) > 4 else [])
    if _SCC_R.match(op):
        u = list(u) + [SCC]
    if _SCC_W.match(op):
        d = list(d) + [SCC]
    return op, d, u


def functions(lines: list):
    starts = [i for i, t in enumerate(lines) if re.match(r"^_Z\w*:", t.strip())]
    for s in starts:
        e = next((j for j in range(s, len(lines)) if lines[j].startswith(".Lfunc_end")), len(lines))
        yield lines[s].strip().split(":")[0], s, e


def sub_clobbers(n: int) -> set:
    return set(("v", r) for r in CLOB_V[n]) | set(("s", r) for r in CLOB_S) | {SCC}


def instructions(lines: list, s: int, e: int):
    """Instruction tuples (kind, info, defs, uses, line) with asm blocks and calls collapsed."""
    ins, target, i = [], {}, s + 1
    while i < e:
        t = lines[i].strip()
        if t.startswith(";;#ASMSTART"):
            j = i
            while not lines[j].strip().startswith(";;#ASMEND"):
                j += 1
            m = re.search(r"hbg_fpmul(\d)", " ".join(lines[i:j]))
            if m:
                n = int(m.group(1))
                outs = set(("v", r) for k in range(n) for r in range(24 * k, 24 * k + 12))
                ins_ = set(("v", r) for k in range(n) for r in range(24 * k, 24 * k + 24))
                ins.append(("ASM", n, sub_clobbers(n) | outs, ins_, i + 1))
            else:
                for k in range(i + 1, j):
                    p = parse(lines[k])
                    if p:
                        ins.append((p[0], None, set(p[1]), set(p[2]), k + 1))
            i = j + 1
            continue
        lm = re.match(r"^([_.A-Za-z0-9$]+):", t)
        if lm:
            ins.append(("LABEL", lm.group(1), set(), set(), i + 1))
            i += 1
            continue
        m = re.match(r"s_add_u32 (s\d+), s\d+, (_Z\w+)@rel32@lo", t)
        if m:
            target[int(m.group(1)[1:])] = m.group(2)
        m = re.match(r"s_swappc_b64 s\[30:31\], s\[(\d+):\d+\]", t)
        if m and int(m.group(1)) in target:
            ins.append(("CALL", target[int(m.group(1))], set(), set(), i + 1))
            i += 1
            continue
        p = parse(lines[i])
        if p:
            ins.append((p[0], None, set(p[1]), set(p[2]), i + 1))
        i += 1
    return ins


def callee_writes(lines: list, funcs: list) -> dict:
    w, calls = {}, {}
    for name, s, e in funcs:
        ws, cs = set(), set()
        txt = lines[s:e]
        for x in instructions(lines, s, e):
            ws |= x[2]
            if x[0] == "CALL":
                cs.add(x[1])
        calls[name] = cs
        # restored by the function itself: whole-wave saved VGPRs, s30/s31 (return address), SP/FP/BP
        joined = "\n".join(txt)
        for m in re.finditer(r"scratch_store_dword off, ([va]\d+), s3[23]( offset:\d+)?\s*; 4-byte Folded Spill\n"
                             r"\s*s_mov_b64 exec", joined):
            ws.discard((m.group(1)[0], int(m.group(1)[1:])))
        for r in (30, 31, 32, 33, 34):
            ws.discard(("s", r))
        w[name] = ws
    changed = True
    while changed:
        changed = False
        for name in w:
            for c in calls[name]:
                if c in w and not w[c] <= w[name]:
                    w[name] |= w[c]
                    changed = True
    return w


def check(path: str, only: str = "") -> int:
    lines = open(path).read().split("\n")
    funcs = list(functions(lines))
    writes = callee_writes(lines, funcs)
    bad = 0
    for name, s, e in funcs:
        if only not in name or name.endswith("hbg_fp_subroutinesEv"):
            continue
        ins = [list(x) for x in instructions(lines, s, e)]
        written = set()
        for x in ins:  # a call's argument uses: v0..v31 set up in its own block before it
            if x[0] == "LABEL":
                written = set()
            elif x[0] == "CALL":
                x[2] = set(writes.get(x[1], set())) | {SCC}
                x[3] = {r for r in written if r[0] == "v" and r[1] < 32} | {("s", 32)}
                written = set()
            else:
                written |= x[2]
        blocks, cur = [], []
        for x in ins:
            if x[0] == "LABEL":
                if cur:
                    blocks.append(cur)
                cur = [x]
                continue
            cur.append(x)
            if x[0].startswith(("s_branch", "s_cbranch")) or x[0] in ("s_setpc_b64", "s_endpgm"):
                blocks.append(cur)
                cur = []
        if cur:
            blocks.append(cur)
        lab = {b[0][1]: k for k, b in enumerate(blocks) if b[0][0] == "LABEL"}
        succ = []
        for k, b in enumerate(blocks):
            last = b[-1]
            sc = []
            if last[0].startswith(("s_branch", "s_cbranch")):
                t = re.search(r"(\.LBB\w+)", lines[last[4] - 1])
                if t and t.group(1) in lab:
                    sc.append(lab[t.group(1)])
            if not last[0].startswith("s_branch") and last[0] not in ("s_setpc_b64", "s_endpgm") and k + 1 < len(blocks):
                sc.append(k + 1)
            succ.append(sc)
        ud = []
        for b in blocks:
            use, df = set(), set()
            for x in b:
                if x[0] != "LABEL":
                    use |= x[3] - df
                    df |= x[2]
            ud.append((use, df))
        li = [set() for _ in blocks]
        lo = [set() for _ in blocks]
        changed = True
        while changed:
            changed = False
            for k in range(len(blocks) - 1, -1, -1):
                o = set().union(*[li[j] for j in succ[k]]) if succ[k] else set()
                n_ = ud[k][0] | (o - ud[k][1])
                if o != lo[k] or n_ != li[k]:
                    lo[k], li[k] = o, n_
                    changed = True
        for k, b in enumerate(blocks):
            live = set(lo[k])
            for x in reversed(b):
                if x[0] == "LABEL":
                    continue
                if x[0] in ("ASM", "CALL"):
                    clob = sub_clobbers(x[1]) if x[0] == "ASM" else x[2]
                    hit = live & clob
                    if hit:
                        bad += 1
                        what = f"hbg_fpmul{x[1]}" if x[0] == "ASM" else x[1][:60]
                        print(f"{path}:{x[4]}: in {name[:60]}: {what}: live across the call: {sorted(hit)[:12]}")
                live -= x[2]
                live |= x[3]
    n_asm = sum(1 for t in lines if "hbg_fpmul" in t and "s_add_u32" in t)
    print(f"checked {len(funcs)} functions, {n_asm} subroutine calls: {bad} violation(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    sys.exit(check(a.asm, a.only))
