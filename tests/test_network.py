"""configs[4] rehearsal: one simulated N-node network spanning ranks with the
all-gather Value/Echo exchange (hydrabadger_amd/network.py).

CPU (gloo, world size 2 and 4): the product's SpanningEpoch orchestration with
an oracle-backed engine standing in for the GPU kernels (test-only: the oracle
is the checker here, never the shipped path).  Every rank must decode every
node's proposal bit-exactly, a tampered echo must be caught by its proof and
dropped, and the result must equal a single-process run.  GPU: the same epoch
through DeviceEngine on cuda:0 (world 1) against the oracle.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hydrabadger_amd import network
from oracle import corc, merkle as omerkle, synth

N_NODES, P = 16, 5000


class OracleEngine:
    """CPU stand-in for DeviceEngine built on the oracle (tests only)."""

    def synth_payloads(self, first, m, P):
        return torch.from_numpy(np.stack([corc.synth_bytes(synth.TAG_PAYLOAD, first + k, P) for k in range(m)]))

    def encode_merkle(self, N, pay, P):
        L = corc.shard_len(N, P)
        out = [corc.rbc_encode_merkle(N, pay[k, :P].numpy().copy()) for k in range(pay.shape[0])]
        return (torch.from_numpy(np.stack([s[:, :L] for s, _ in out])),
                torch.from_numpy(np.stack([lv for _, lv in out])))

    def validate(self, N, L, shards, levels, sib, nd):
        sh, lv = shards.numpy(), levels.numpy()
        ok = np.zeros((sh.shape[0], N), np.uint8)
        for i in range(sh.shape[0]):
            for j in range(N):
                p = omerkle.Proof(sh[i, j, :L].tobytes(), j, [lv[i, sib[j, k]].tobytes() for k in range(nd[j])],
                                  lv[i, -1].tobytes())
                ok[i, j] = p.validate(N)
        return torch.from_numpy(ok)

    def decode(self, N, L, shards, present, roots):
        outs, lens, st = [], [], []
        for i in range(shards.shape[0]):
            r = corc.rbc_decode(N, L, shards[i].numpy().copy(), present[i].numpy(), roots[i].numpy().tobytes())
            outs.append(r or b"")
            lens.append(len(r) if r is not None else 0)
            st.append(1 if r is not None else 0)
        w = max(len(o) for o in outs)
        buf = np.zeros((len(outs), max(w, 1)), np.uint8)
        for i, o in enumerate(outs):
            buf[i, :len(o)] = np.frombuffer(o, np.uint8)
        return torch.from_numpy(buf), torch.tensor(lens), torch.tensor(st, dtype=torch.uint8)

    def sync(self):
        pass


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_rank(rank, world, port, q, tamper):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = OracleEngine()
        ep = network.SpanningEpoch(N_NODES, P, eng)
        pay = eng.synth_payloads(ep.rank * ep.m, ep.m, P)
        if tamper:
            real = eng.encode_merkle
            def bad(N, p, PP):  # rank 0 proposer 1's shard 5 corrupted after its tree is built
                sh, lv = real(N, p, PP)
                if rank == 0:
                    sh[1, 5, 0] ^= 0xFF
                return sh, lv
            eng.encode_merkle = bad
        res = ep.run(pay)
        q.put((rank, res.payloads[:, :P].numpy().copy(), res.lengths.tolist(), res.status.tolist(),
               res.echo_ok.numpy().copy(), res.exchange_bytes))
    finally:
        dist.destroy_process_group()


def _spawn(world, tamper=False):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_run_rank, args=(r, world, port, q, tamper)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=300) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def _expected():
    return np.stack([corc.synth_bytes(synth.TAG_PAYLOAD, i, P) for i in range(N_NODES)])


def test_proof_index_map_matches_merkle_proofs():
    for n in (1, 2, 3, 4, 7, 16, 64, 100, 128):
        sib, nd = network.proof_index_map(n)
        values = [bytes([i]) * 3 for i in range(n)]
        t = omerkle.MerkleTree.from_vec(values)
        flat = t.flat_levels()
        for j in range(n):
            pr = t.proof(j)
            assert [flat[sib[j, k]] for k in range(nd[j])] == list(pr.digests)


def test_arrival_mask_drops_f():
    for i in range(5):
        m = network.arrival_mask(i, 128)
        assert sum(m) == 128 - 42


@pytest.mark.parametrize("world", [2, 4])
def test_spanning_epoch_gloo(world):
    got = _spawn(world)
    exp = _expected()
    for r in range(world):
        pays, lens, st, ok, recv = got[r]
        assert st == [1] * N_NODES and lens == [P] * N_NODES
        assert np.array_equal(pays, exp)
        assert ok.all()
        assert recv > 0
    # world 1 (no collective) gives the same batch
    single = network.SpanningEpoch(N_NODES, P, OracleEngine())
    res = single.run(OracleEngine().synth_payloads(0, N_NODES, P))
    assert np.array_equal(res.payloads[:, :P].numpy(), exp) and res.exchange_bytes == 0


def test_spanning_epoch_tampered_echo_dropped():
    """A shard changed after its tree was built fails Proof::validate on every
    rank; the instance still decodes from the remaining echoes (f absent + 1
    invalid still leaves >= N-2f), identically everywhere."""
    got = _spawn(2, tamper=True)
    exp = _expected()
    for r in range(2):
        pays, lens, st, ok, _ = got[r]
        assert ok[1, 5] == 0 and ok.sum() == N_NODES * N_NODES - 1
        assert st == [1] * N_NODES and np.array_equal(pays, exp)


@pytest.mark.gpu
def test_spanning_epoch_device_world1():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda:0")
    eng = network.DeviceEngine(dev)
    try:
        N, PP = 128, 1 << 16
        ep = network.SpanningEpoch(N, PP, eng)
        res = ep.run(eng.synth_payloads(0, N, PP))
        assert res.status.cpu().tolist() == [1] * N
        assert res.lengths.cpu().tolist() == [PP] * N
        assert bool(res.echo_ok.all())
        out = res.payloads[:, :PP].cpu().numpy()
        for i in (0, 77, N - 1):
            assert np.array_equal(out[i], corc.synth_bytes(synth.TAG_PAYLOAD, i, PP))
    finally:
        eng.ctx.close()
