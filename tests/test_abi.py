"""CPU-side checks of the C ABI boundary: libhbgpu.so loads, exports every
symbol include/hbgpu.h declares (with the binding's signature table in sync),
and its pure host functions (no GPU needed) agree with the oracle."""
from __future__ import annotations

import os
import re

import numpy as np
import pytest

from oracle import gf256, merkle, rbc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = []
    for h in os.listdir(os.path.join(ROOT, "include")):
        if h.endswith(".h"):
            src = open(os.path.join(ROOT, "include", h)).read()
            names += re.findall(r"^\s*(?:const\s+)?\w+[\s\*]+(hbg_\w+)\s*\(", src, re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    from hydrabadger_amd import _lib
    l = _lib.lib()
    declared = _declared()
    assert len(declared) >= 18
    for name in declared:
        assert hasattr(l, name), name
    assert set(declared) == set(_lib.SIGNATURES), set(declared) ^ set(_lib.SIGNATURES)
    assert l.hbg_version().startswith(b"hbgpu")


def test_error_strings():
    from hydrabadger_amd import _lib
    assert _lib.lib().hbg_strerror(_lib.HBG_E_TOO_FEW_SHARDS_PRESENT) == b"TooFewShardsPresent"


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 16, 64, 100, 128, 255, 256])
def test_shape_helpers_match_oracle(n):
    from hydrabadger_amd import _lib
    assert _lib.merkle_nodes(n) == merkle.num_nodes(n)
    assert _lib.merkle_depth(n) == merkle.depth(n)
    assert _lib.num_faulty(n) == rbc.num_faulty(n)
    for P in [0, 1, 1 << 16, 1 << 20]:
        d, _ = rbc.shard_counts(n)
        assert _lib.shard_len(n, P) == rbc.shard_len(P, d)


@pytest.mark.parametrize("D,Q", [(2, 2), (6, 10), (22, 42), (44, 84), (1, 1), (86, 170), (255, 1), (3, 253)])
def test_coding_matrix_matches_oracle(D, Q):
    from hydrabadger_amd import _lib
    assert np.array_equal(_lib.coding_matrix(D, Q), np.array(gf256.build_matrix(D, Q), np.uint8))


def test_coding_new_errors():
    from hydrabadger_amd import broadcast as bc
    for (d, q), kind in [((0, 2), "TooFewDataShards"), ((200, 57), "TooManyShards")]:
        with pytest.raises(bc.RseError) as e:
            bc.Coding(d, q)
        assert e.value.kind == kind
    assert bc.Coding(3, 0).parity_shard_count() == 0  # Trivial


def test_no_cpu_fallback_without_device():
    """The product path must fail loudly (not compute on the CPU) when no GPU
    is present; in this container hbg_init must error."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from hydrabadger_amd import _lib
    with pytest.raises(_lib.HbgError):
        _lib.Context()


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "hydrabadger_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dp, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f
                assert "liborc" not in src, f


def test_workload_generator_matches_oracle_statement():
    from hydrabadger_amd import workload
    from oracle import synth
    for inst in [0, 1, 77, 2 ** 33]:
        for n, e in [(64, 42), (16, 10), (4, 2), (128, 84)]:
            assert workload.erasure_mask(inst, n, e) == synth.erasure_mask(inst, n, e)


def test_selftest_vectors_match_the_fixture(tmp_path):
    """The power-on self-test's known answers (csrc/selftest_vectors.h,
    api.hip run_self_test) are exactly what tools/gen_selftest_vectors.py
    derives from the committed tests/golden/tdec_golden.json."""
    import subprocess
    import sys
    out = tmp_path / "v.h"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_selftest_vectors.py"), "--out", str(out)],
                   check=True, capture_output=True)
    assert out.read_text() == open(os.path.join(ROOT, "hydrabadger_amd", "csrc", "selftest_vectors.h")).read()
