"""World-size-2 (gloo, CPU) rehearsal of bench.py's multi-GPU structure
(SURVEY.md §8(e)): each rank owns a contiguous block of instance ids, builds
its inputs from the per-instance SplitMix64 streams (no data exchange), and
only the timing max / rate sum cross ranks.  The per-rank results (oracle C
port standing in for the device) must equal a single-process run over all
instances, which is what makes the sharded bench's work identical to N=1."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hydrabadger_amd import shard

N_NODES, P, PER_RANK = 16, 3000, 3


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _roots_for(ids):
    from oracle import corc
    out = []
    for k in ids:
        pay = corc.synth_bytes(1, k, P)
        _, levels = corc.rbc_encode_merkle(N_NODES, pay)[:2]
        out.append(bytes(levels[-1]))
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = shard.instance_block(rank, world, PER_RANK)
        roots = _roots_for(ids)
        mx = shard.max_over_ranks(float(rank + 1))
        sm = shard.sum_over_ranks(float(10 * (rank + 1)))
        gathered = [None] * world
        dist.all_gather_object(gathered, (list(ids), roots))
        if rank == 0:
            q.put((gathered, mx, sm))
    finally:
        dist.destroy_process_group()


def test_instance_blocks_and_partition():
    assert list(shard.instance_block(1, 4, 5)) == [5, 6, 7, 8, 9]
    for n, w in ((10, 3), (7, 8), (2048, 8)):
        parts = [shard.partition(n, r, w) for r in range(w)]
        assert sum(len(p) for p in parts) == n
        assert [i for p in parts for i in p] == list(range(n))
    with pytest.raises(ValueError):
        shard.instance_block(2, 2, 1)


def test_world2_gloo_matches_single_process():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, mx, sm = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mx == 2.0 and sm == 30.0
    ids = [i for g in gathered for i in g[0]]
    assert ids == list(range(world * PER_RANK))  # disjoint, contiguous, complete
    roots = [r for g in gathered for r in g[1]]
    assert roots == _roots_for(range(world * PER_RANK))
    assert len(set(roots)) == len(roots)
