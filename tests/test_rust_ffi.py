"""The Rust FFI crate (rust/hbgpu-sys/src/lib.rs) against the C header
(include/hbgpu.h): every prototype bound once with the same parameter and
return types, and every HBG_* constant with the same value.  cargo is absent
in this image, so this diff is what keeps the crate honest.
"""
from __future__ import annotations

import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hbgpu.h")
LIB_RS = os.path.join(ROOT, "rust", "hbgpu-sys", "src", "lib.rs")

# C parameter / return type -> the Rust type the crate must use
C_TO_RUST = {
    "int": "c_int", "uint32_t": "u32", "uint64_t": "u64", "int32_t": "i32", "void": None,
    "hbg_ctx*": "*mut hbg_ctx", "hbg_ctx**": "*mut *mut hbg_ctx", "void*": "*mut c_void",
    "const hbg_ctx*": "*const hbg_ctx",
    "const char*": "*const c_char", "char*": "*mut c_char",
    "const uint8_t*": "*const u8", "uint8_t*": "*mut u8",
    "const uint32_t*": "*const u32", "uint32_t*": "*mut u32",
    "const uint64_t*": "*const u64", "uint64_t*": "*mut u64",
    "const int32_t*": "*const i32", "int32_t*": "*mut i32",
}


def _strip_c_comments(s: str) -> str:
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _c_type(decl: str) -> tuple:
    """'const uint8_t *shards' -> ('const uint8_t*', 'shards')."""
    decl = " ".join(decl.replace("*", " * ").split())
    m = re.match(r"^(.*?)(\w+)$", decl)
    ty, name = m.group(1).strip(), m.group(2)
    if not ty:  # unnamed parameter: 'void'
        ty, name = name, ""
    return ty.replace(" *", "*").replace(" *", "*"), name


def header_prototypes() -> dict:
    src = _strip_c_comments(open(HEADER).read())
    src = "\n".join(line for line in src.splitlines() if not line.lstrip().startswith("#"))
    out = {}
    for stmt in re.split(r"[;{}]", src):
        m = re.fullmatch(r"\s*([A-Za-z_][\w\s\*]*?)\b(hbg_\w+)\s*\(([^()]*)\)\s*", stmt, flags=re.S)
        if not m:
            continue
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ret_t = _c_type(ret.strip() + " x")[0]
        ps = [] if params.strip() in ("", "void") else [_c_type(p)[0] for p in params.split(",")]
        out[name] = (ret_t, ps)
    return out


def rust_prototypes() -> dict:
    src = open(LIB_RS).read()
    block = re.search(r'extern "C" \{(.*?)\n\}', src, flags=re.S).group(1)
    out = {}
    for m in re.finditer(r"pub fn (\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        name, params, ret = m.group(1), m.group(2), m.group(3)
        ps = [" ".join(p.split(":", 1)[1].split()) for p in params.split(",") if p.strip()]
        out[name] = (ret.strip() if ret else None, ps)
    return out


def _eval_const(expr: str) -> int:
    expr = re.sub(r"\b(0[xX][0-9a-fA-F]+|\d+)[uU]\b", r"\1", expr.strip())
    assert re.fullmatch(r"(0[xX][0-9a-fA-F]+|[\d\s\(\)\*\+\-])+", expr), expr
    return int(eval(expr))  # integer literals and arithmetic only (asserted above)


def header_constants() -> dict:
    src = _strip_c_comments(open(HEADER).read())
    return {m.group(1): _eval_const(m.group(2))
            for m in re.finditer(r"#define (HBG_\w+)\s+([^\n]+)", src) if re.search(r"\d", m.group(2))}


def rust_constants() -> dict:
    src = open(LIB_RS).read()
    return {m.group(1): _eval_const(m.group(2).replace("_", ""))
            for m in re.finditer(r"pub const (HBG_\w+): \w+ = ([^;]+);", src)}


def test_every_prototype_bound_with_matching_types():
    h, r = header_prototypes(), rust_prototypes()
    assert len(h) >= 30, sorted(h)
    assert set(h) == set(r), {"header only": sorted(set(h) - set(r)), "rust only": sorted(set(r) - set(h))}
    for name, (ret, ps) in h.items():
        rret, rps = r[name]
        assert C_TO_RUST[ret] == rret, (name, ret, rret)
        assert len(ps) == len(rps), (name, ps, rps)
        for i, (c, rust) in enumerate(zip(ps, rps)):
            assert C_TO_RUST[c] == rust, (name, i, c, rust)


def test_every_constant_matches():
    h, r = header_constants(), rust_constants()
    missing = sorted(set(h) - set(r))
    assert not missing, missing
    for k, v in r.items():
        assert k in h, k
        assert h[k] == v, (k, h[k], v)


def test_safe_wrappers_reference_bound_symbols():
    """safe.rs calls only functions the extern block declares."""
    safe = open(os.path.join(ROOT, "rust", "hbgpu-sys", "src", "safe.rs")).read()
    called = set(re.findall(r"\b(hbg_\w+)\(", safe))
    assert called, "no FFI calls in safe.rs"
    assert called <= set(rust_prototypes()), sorted(called - set(rust_prototypes()))


@pytest.mark.parametrize("decl,expect", [("const uint8_t *shards", ("const uint8_t*", "shards")),
                                         ("hbg_ctx **out", ("hbg_ctx**", "out")), ("void", ("void", ""))])
def test_c_type_parser(decl, expect):
    assert _c_type(decl) == expect


def test_kat_gen_payload_generator_matches_oracle():
    """rust/kat-gen restates oracle/synth.py's payload stream: same constants."""
    from oracle import synth
    src = open(os.path.join(ROOT, "rust", "kat-gen", "src", "main.rs")).read()
    consts = {m.group(1): int(m.group(2).replace("_", ""), 16)
              for m in re.finditer(r"const (\w+): u64 = 0x([0-9A-Fa-f_]+);", src)}
    assert consts["BASE_SEED"] == synth.BASE_SEED and consts["GAMMA"] == synth.GAMMA
    assert re.search(r"const TAG_PAYLOAD: u64 = (\d+);", src).group(1) == str(synth.TAG_PAYLOAD)
    for c in ("0xBF58_476D_1CE4_E5B9", "0x94D0_49BB_1331_11EB"):
        assert c in src
