"""GF(2^8) Reed-Solomon restatement (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Restates reed-solomon-erasure [EXT, version unpinned; v3..v6 share the math],
reached from hbbft ``Broadcast::new`` -> ``Coding::new(data, parity)`` and
``send_shards`` -> ``Coding::encode`` / ``decode_from_shards`` ->
``Coding::reconstruct_shards``, which the
reference reaches through ``src/hydrabadger/state.rs:484`` (``dhb.propose``) and
``state.rs:486-487`` (``dhb.handle_message``).

Field: polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2 (rse ``galois_8``).
Coding matrix: M = V · inv(V[0..D]) with V[r][c] = r^c (0^0 = 1), N x D
(rse ``build_matrix``).  Pinned by the Backblaze JavaReedSolomon known answer
(tests/test_oracle_rbc.py::test_backblaze_kat).
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D
FIELD = 256

# --- tables (rse galois_8: gen_log_table / gen_exp_table) -----------------
LOG = [0] * 256
EXP = [0] * 510
_b = 1
for _l in range(255):
    LOG[_b] = _l
    EXP[_l] = _b
    EXP[_l + 255] = _b
    _b <<= 1
    if _b >= FIELD:
        _b ^= POLY
del _b, _l

MUL = np.zeros((256, 256), dtype=np.uint8)
for _a in range(1, 256):
    for _c in range(1, 256):
        MUL[_a, _c] = EXP[LOG[_a] + LOG[_c]]
del _a, _c


def gmul(a: int, b: int) -> int:
    if a == 0 or b == 0:
        return 0
    return EXP[LOG[a] + LOG[b]]


def gdiv(a: int, b: int) -> int:
    if b == 0:
        raise ZeroDivisionError("GF(2^8) division by zero")
    if a == 0:
        return 0
    return EXP[(LOG[a] - LOG[b]) % 255]


def gexp(a: int, n: int) -> int:
    """rse ``galois_8::exp``: a^n with 0^0 = 1."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return EXP[(LOG[a] * n) % 255]


# --- matrices ---------------------------------------------------------------
class SingularMatrix(Exception):
    pass


def invert(m: list[list[int]]) -> list[list[int]]:
    """Gauss-Jordan inverse over GF(2^8).  The inverse is unique, so any pivot
    order gives the same bytes as rse ``Matrix::invert``."""
    n = len(m)
    a = [list(row) + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(m)]
    for r in range(n):
        if a[r][r] == 0:
            for rb in range(r + 1, n):
                if a[rb][r] != 0:
                    a[r], a[rb] = a[rb], a[r]
                    break
        if a[r][r] == 0:
            raise SingularMatrix()
        if a[r][r] != 1:
            s = gdiv(1, a[r][r])
            a[r] = [gmul(s, x) for x in a[r]]
        for rb in range(n):
            if rb != r and a[rb][r] != 0:
                s = a[rb][r]
                a[rb] = [x ^ gmul(s, y) for x, y in zip(a[rb], a[r])]
    return [row[n:] for row in a]


def matmul(a: list[list[int]], b: list[list[int]]) -> list[list[int]]:
    out = []
    for row in a:
        o = []
        for c in range(len(b[0])):
            acc = 0
            for k, x in enumerate(row):
                acc ^= gmul(x, b[k][c])
            o.append(acc)
        out.append(o)
    return out


class TooFewDataShards(Exception):
    pass


class TooFewParityShards(Exception):
    pass


class TooManyShards(Exception):
    pass


class TooFewShards(Exception):
    pass


class TooFewShardsPresent(Exception):
    pass


class IncorrectShardSize(Exception):
    pass


class EmptyShard(Exception):
    pass


def build_matrix(data: int, parity: int) -> list[list[int]]:
    """rse ``ReedSolomon::new`` -> ``build_matrix(data, total)``: N x D."""
    if data == 0:
        raise TooFewDataShards()
    if parity == 0:
        raise TooFewParityShards()
    total = data + parity
    if total > 256:
        raise TooManyShards()
    vand = [[gexp(r, c) for c in range(data)] for r in range(total)]
    top_inv = invert([row[:] for row in vand[:data]])
    return matmul(vand, top_inv)


def code_rows(rows: list[list[int]], inputs: np.ndarray) -> np.ndarray:
    """out[k] = XOR_j rows[k][j] * inputs[j]  (inputs: [J][L] uint8)."""
    out = np.zeros((len(rows), inputs.shape[1]), dtype=np.uint8)
    for k, row in enumerate(rows):
        acc = out[k]
        for j, c in enumerate(row):
            if c:
                acc ^= MUL[c][inputs[j]]
    return out


class ReedSolomon:
    """rse ``ReedSolomon`` (encode / reconstruct), numpy-vectorised over bytes."""

    def __init__(self, data: int, parity: int):
        self.data = data
        self.parity = parity
        self.total = data + parity
        self.matrix = build_matrix(data, parity)
        self.parity_rows = self.matrix[data:]

    def encode(self, shards: np.ndarray) -> None:
        """In place: shards [N][L]; rows D..N-1 overwritten with parity."""
        if shards.shape[0] != self.total:
            raise TooManyShards() if shards.shape[0] > self.total else TooFewShards()
        if shards.shape[1] == 0:
            raise EmptyShard()
        shards[self.data:] = code_rows(self.parity_rows, shards[: self.data])

    def reconstruct(self, shards: list) -> None:
        """In place on a list of Optional[np.ndarray]; rse ``reconstruct``.

        Uses the FIRST D present rows in index order (rse reconstruct_internal)
        — the decode matrix is unique for that row set, and the present shards
        are kept exactly as received."""
        if len(shards) != self.total:
            raise TooManyShards() if len(shards) > self.total else TooFewShards()
        present = [i for i, s in enumerate(shards) if s is not None]
        sizes = {len(shards[i]) for i in present}
        if len(sizes) > 1:
            raise IncorrectShardSize()
        if len(present) == self.total:
            return
        if len(present) < self.data:
            raise TooFewShardsPresent()
        L = sizes.pop()
        if L == 0:
            raise EmptyShard()
        rows_used = present[: self.data]
        sub = [self.matrix[r][:] for r in rows_used]
        dec = invert(sub)
        sub_shards = np.stack([shards[r] for r in rows_used])
        missing_data = [i for i in range(self.data) if shards[i] is None]
        if missing_data:
            rec = code_rows([dec[i] for i in missing_data], sub_shards)
            for k, i in enumerate(missing_data):
                shards[i] = rec[k]
        missing_par = [i for i in range(self.data, self.total) if shards[i] is None]
        if missing_par:
            data_shards = np.stack([shards[i] for i in range(self.data)])
            rec = code_rows([self.matrix[i] for i in missing_par], data_shards)
            for k, i in enumerate(missing_par):
                shards[i] = rec[k]


def decode_matrix(data: int, parity: int, present_mask: list[bool]) -> tuple[list[int], list[list[int]]]:
    """Helper used by tests: (rows_used, inverse of their D x D submatrix)."""
    m = build_matrix(data, parity)
    rows = [i for i, p in enumerate(present_mask) if p][:data]
    return rows, invert([m[r][:] for r in rows])
