"""SURVEY.md §8 f4 + a18: one HoneyBadger epoch (hydrabadger_amd/epoch.py)
against oracle/epoch.py, the node-by-node restatement of hbbft's Broadcast
(Value -> Echo -> Ready with the N-f / 2f+1 / N-2f thresholds) and
ThresholdDecrypt over the wire-format messages.

CPU: the product orchestration with the oracle-backed engine, world 1 and
gloo world 2 (the all_gather_into_tensor branch RCCL takes), honest and with
faulty nodes.  GPU: the same epochs through DeviceEngine on cuda:0.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hydrabadger_amd import epoch as hbe
from oracle import epoch as oep
from oracle import synth

FAULTS = {
    "honest": {},
    # a crashed node, a Value corrupted for one recipient, a node echoing garbage,
    # a node sending shares made with another node's key, a corrupted ciphertext
    "faulty": dict(silent={3}, bad_value={(0, 1)}, bad_echo={2}, bad_share={5}, bad_ct={6}),
}


def _faults(spec, mod):
    return mod.Faults(**{k: frozenset(v) for k, v in spec.items()})


def _np(t):
    return t.cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def compare(res: hbe.EpochResult, exp: oep.EpochOut, P: int):
    """Bit-exact agreement of the batched epoch with the node-by-node oracle."""
    N = len(exp.delivered)
    assert _np(res.value_ok).astype(bool).tolist() == exp.value_ok
    assert _np(res.echo_ok).astype(bool).tolist() == exp.echo_ok
    assert _np(res.echo_count).tolist() == exp.echo_count
    assert _np(res.ready_count).tolist() == exp.ready_count
    assert _np(res.delivered).astype(bool).tolist() == exp.delivered
    pays = _np(res.payloads)
    C = hbe.ct_bytes(P)
    for p in range(N):
        if exp.payloads[p] is not None:
            assert pays[p, :C].tobytes() == exp.payloads[p], p
    assert res.accepted == exp.accepted
    # TDec views: this rank's nodes (each its own ThresholdDecrypt with its own
    # arrival order) or the shared view
    assert len(res.views) == _np(res.ct_status).shape[0]
    for vi, node in enumerate(res.views):
        ei = exp.views.index(None if node < 0 else node)
        assert _np(res.ct_status)[vi].tolist() == exp.ct_status[ei], node
        pts = _np(res.plaintexts)[vi]
        for q, pt in enumerate(exp.plaintexts[ei]):
            if pt is not None:
                assert pts[q].tobytes() == pt, (node, q)
        assert _np(res.share_outcome)[vi].tolist() == exp.share_outcome[ei], node


# ----------------------------------------------------------------------------- oracle sanity
def test_oracle_epoch_honest_delivers_every_contribution():
    N, P = 4, 40
    out = oep.run_epoch(N, P, seed=3)
    assert out.delivered == [True] * N and out.accepted == list(range(N))
    assert out.views == list(range(N))
    for v in range(N):  # every node decrypts every contribution
        assert out.ct_status[v] == [0] * N
        for p in range(N):
            assert out.plaintexts[v][p] == synth.synth_bytes(oep.TAG_CONTRIB, oep.instance_id(0, p), P)
        f = (N - 1) // 3
        for oc in out.share_outcome[v]:  # exactly t+1 = f+1 accepted, the rest ignored
            assert oc.count(1) == f + 1 and oc.count(3) == N - f - 1
    # each node handles shares in its own arrival order: the views differ
    assert len({str(out.share_outcome[v]) for v in range(N)}) > 1


def test_oracle_epoch_shared_view_is_one_instance_per_ciphertext():
    out = oep.run_epoch(4, 40, seed=3, per_node=False)
    assert out.views == [None] and len(out.ct_status) == 1 and out.ct_status[0] == [0] * 4


def test_oracle_epoch_fault_semantics():
    N, P = 7, 24
    out = oep.run_epoch(N, P, seed=2, faults=_faults(FAULTS["faulty"], oep))
    assert not out.value_ok[0][1]                    # the corrupted Value fails its proof
    assert not any(out.echo_ok[2])                   # node 2's echoes all fail
    assert not any(out.echo_ok[3])                   # the silent node echoes nothing
    assert not out.delivered[3]                      # ... and proposes nothing
    k6 = out.accepted.index(6)
    for v in out.views:
        assert out.ct_status[v][k6] == oep.T.E_INVALID_CIPHERTEXT
        for q, p in enumerate(out.accepted):
            if p != 6:
                assert out.ct_status[v][q] == 0
                # silent: no share, except in its own view (start_decryption inserts the own share)
                assert out.share_outcome[v][q][3] == (1 if v == 3 else 0)
                # bad share: fault if processed, never accepted — except its own (true) share in its own view
                assert out.share_outcome[v][q][5] in ((1,) if v == 5 else (0, 2, 3))


# ----------------------------------------------------------------------------- product orchestration on CPU
@pytest.mark.parametrize("per_node", [True, False])
@pytest.mark.parametrize("name,N,P", [("honest", 4, 40), ("faulty", 7, 24)])
def test_epoch_world1_oracle_engine(name, N, P, per_node):
    from tests.oracle_engine import OracleEngine
    ep = hbe.HoneyBadgerEpoch(N, P, OracleEngine(), seed=2)
    res = ep.run(epoch=1, faults=_faults(FAULTS[name], hbe), per_node=per_node)
    compare(res, oep.run_epoch(N, P, seed=2, epoch=1, faults=_faults(FAULTS[name], oep), per_node=per_node), P)
    assert res.exchange_bytes == 0
    nv = N if per_node else 1
    assert res.views == (list(range(N)) if per_node else [-1])
    assert res.work["echo_validations"] == nv * N * N and res.work["decodes"] == nv * N
    assert res.work["value_validations"] == N * N


def test_epoch_gloo_world1_group_runs_the_collective():
    """A one-rank process group takes the all_gather_into_tensor branch (the
    path the GPU test drives through RCCL) and agrees with the oracle."""
    from tests.oracle_engine import OracleEngine
    dist.init_process_group("gloo", rank=0, world_size=1, store=dist.HashStore())
    try:
        calls = []
        real = dist.all_gather_into_tensor
        def spy(*a, **k):
            calls.append(1)
            return real(*a, **k)
        dist.all_gather_into_tensor = spy
        try:
            res = hbe.HoneyBadgerEpoch(7, 24, OracleEngine(), seed=2).run(epoch=1, faults=_faults(FAULTS["faulty"], hbe))
        finally:
            dist.all_gather_into_tensor = real
        assert calls
        compare(res, oep.run_epoch(7, 24, seed=2, epoch=1, faults=_faults(FAULTS["faulty"], oep)), 24)
    finally:
        dist.destroy_process_group()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q, N, P, name):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.oracle_engine import OracleEngine
        res = hbe.HoneyBadgerEpoch(N, P, OracleEngine(), seed=2).run(epoch=1, faults=_faults(FAULTS[name], hbe))
        # tensors -> numpy: a queued tensor is shared through a handle that dies with this process
        plain = {k: (v.numpy().copy() if isinstance(v, torch.Tensor) else v) for k, v in vars(res).items()}
        q.put((rank, hbe.EpochResult(**plain)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,N,P", [("honest", 4, 40), ("faulty", 8, 24)])
def test_epoch_gloo_world2(name, N, P):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q, N, P, name)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=600) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = oep.run_epoch(N, P, seed=2, epoch=1, faults=_faults(FAULTS[name], oep))
    m = N // 2
    for r in range(2):
        compare(got[r], exp, P)
        assert got[r].exchange_bytes > 0
        assert got[r].views == list(range(r * m, (r + 1) * m))
        # each rank validates only the Values addressed to its own nodes (N per
        # node), every echo once per local node, and decodes / decrypts per node
        assert got[r].work["value_validations"] == N * m
        assert got[r].work["echo_validations"] == m * N * N
        assert got[r].work["decodes"] == m * N
        assert got[r].work["tdec_instances"] == m * len(exp.accepted)


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name,N,P,per_node", [("honest", 4, 40, True), ("faulty", 7, 24, True),
                                               ("faulty", 16, 300, True), ("faulty", 16, 300, False)])
def test_epoch_device_world1(name, N, P, per_node):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hydrabadger_amd import network
    eng = network.DeviceEngine(torch.device("cuda:0"))
    try:
        res = hbe.HoneyBadgerEpoch(N, P, eng, seed=2).run(epoch=1, faults=_faults(FAULTS[name], hbe),
                                                           per_node=per_node)
        compare(res, oep.run_epoch(N, P, seed=2, epoch=1, faults=_faults(FAULTS[name], oep), per_node=per_node), P)
    finally:
        eng.ctx.close()


@pytest.mark.gpu
def test_epoch_device_rccl_world1():
    """The RCCL branch on hardware: a one-rank "nccl" process group, so every
    message round goes through all_gather_into_tensor on device tensors (RCCL
    refuses two ranks on one GPU: "Duplicate GPU detected", tools/rccl_probe.py),
    same results as the oracle epoch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hydrabadger_amd import network
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=dev)
    eng = network.DeviceEngine(dev)
    try:
        assert dist.get_backend() == "nccl"
        res = hbe.HoneyBadgerEpoch(16, 300, eng, seed=2).run(epoch=1, faults=_faults(FAULTS["faulty"], hbe))
        compare(res, oep.run_epoch(16, 300, seed=2, epoch=1, faults=_faults(FAULTS["faulty"], oep)), 300)
    finally:
        eng.ctx.close()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_epoch_device_n64_honest_plaintexts():
    """configs[3]/[4] shape: N=64, every contribution decrypted to its bytes
    (size-independent property: no oracle epoch at this size)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hydrabadger_amd import network
    eng = network.DeviceEngine(torch.device("cuda:0"))
    try:
        N, P = 64, 4096
        res = hbe.HoneyBadgerEpoch(N, P, eng, seed=5).run(epoch=2)
        assert bool(res.delivered.all()) and res.accepted == list(range(N))
        assert res.views == list(range(N)) and (_np(res.ct_status) == 0).all()
        pts = _np(res.plaintexts)
        for v in (0, 17, 63):
            for p in (0, 31, 63):
                assert pts[v, p].tobytes() == synth.synth_bytes(hbe.TAG_CONTRIB, hbe.instance_id(2, p), P)
        oc = _np(res.share_outcome)
        assert ((oc == 1).sum(2) == 22).all() and ((oc == 3).sum(2) == N - 22).all()
    finally:
        eng.ctx.close()


@pytest.mark.parametrize("N", [1, 2, 3, 5])
@pytest.mark.parametrize("spec", [{}, {"silent": {0}}, {"bad_share": {1}, "bad_echo": {0}}])
def test_epoch_small_networks_oracle_engine(N, spec):
    """Trivial coding (N <= 3: no parity), a single node, and crashed / faulty
    nodes in networks too small to tolerate them: same outcome as the oracle."""
    from tests.oracle_engine import OracleEngine
    spec = {k: {x % N for x in v} for k, v in spec.items()}
    res = hbe.HoneyBadgerEpoch(N, 17, OracleEngine(), seed=4).run(epoch=3, faults=_faults(spec, hbe))
    compare(res, oep.run_epoch(N, 17, seed=4, epoch=3, faults=_faults(spec, oep)), 17)


@pytest.mark.gpu
def test_epoch_device_configs4_size():
    """BASELINE.json configs[4] at full size on one GPU: a 128-node epoch (RS
    44+84, t = 42) with 1 MiB contributions — every contribution delivered,
    accepted and decrypted to its bytes, t+1 shares held per ciphertext
    (size-independent properties; no oracle epoch at this size)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hydrabadger_amd import network
    eng = network.DeviceEngine(torch.device("cuda:0"))
    try:
        N, P = 128, 1 << 20
        res = hbe.HoneyBadgerEpoch(N, P, eng, seed=7).run(epoch=3)
        assert bool(res.delivered.all()) and res.accepted == list(range(N))
        assert res.views == list(range(N)) and (_np(res.ct_status) == 0).all()
        want = eng.synth(hbe.TAG_CONTRIB, hbe.instance_id(3, 0), N, P)
        assert len(res.views) == N and all(torch.equal(res.plaintexts[v], want) for v in range(N))
        oc = _np(res.share_outcome)
        assert ((oc == 1).sum(2) == 43).all() and ((oc == 3).sum(2) == N - 43).all()
    finally:
        eng.ctx.close()
