"""CPU rehearsal of bench.py's multi-rank path: the same
init_distributed / run_timed / Legs code the driver runs under torchrun with
RCCL, here with the gloo backend and 2 ranks.  The timed region must be the
max over ranks (the slowest rank's wall time) on every rank, and a failing leg
must be reported, not crash the line."""
from __future__ import annotations

import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

import bench


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    w, r = bench.init_distributed("gloo", 0)
    try:
        assert (w, r) == (world, rank)
        calls = []

        def step():
            calls.append(1)
            time.sleep(0.04 * (rank + 1))
        dt = bench.run_timed(step, 3, 2, lambda: None, torch.device("cpu"))
        from hydrabadger_amd import shard
        total = shard.sum_over_ranks(float(rank + 1), torch.device("cpu"))
        info = bench.dist_info(True)
        assert info == {"backend": "gloo", "world_size_seen": world, "rccl_version": None}
        q.put((rank, dt, len(calls), total))
    finally:
        torch.distributed.destroy_process_group()


def test_run_timed_max_over_ranks_gloo_world2():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((x[0], x[1:]) for x in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dts = [got[r][0] for r in range(2)]
    assert dts[0] == dts[1]                      # one max, seen by every rank
    assert dts[0] >= 3 * 0.08                    # the slow rank's 3 timed steps (warmup excluded)
    assert dts[0] < 3 * 0.08 + 2 * 0.08 + 1.0   # ... and not its warmup
    assert all(got[r][1] == 5 for r in range(2))  # W + K steps on each rank
    assert all(got[r][2] == 3.0 for r in range(2))  # whole-job sum of per-rank rates


def test_legs_record_failures_and_keep_going():
    legs = bench.Legs()
    assert legs("a", lambda: 1) == 1

    def boom():
        raise RuntimeError("HIP error: device lost")
    assert legs("b", boom) is None
    assert legs("c", lambda: 3) == 3
    assert legs.errors == {"b": "RuntimeError: HIP error: device lost"}


def test_dist_info_single_process():
    assert bench.dist_info(False) == {"backend": None, "world_size_seen": 1, "rccl_version": None}


def test_bench_backend_switch_parses():
    import sys
    old = sys.argv
    try:
        sys.argv = ["bench.py", "--backend", "gloo", "--epoch-contrib", "4096"]
        a = bench.parse()
        assert a.backend == "gloo" and a.epoch_contrib == 4096
        sys.argv = ["bench.py", "--backend", "mpi"]
        with pytest.raises(SystemExit):
            bench.parse()
    finally:
        sys.argv = old


def test_checks_final_is_last_and_sets_exit_status():
    """The compact verdicts ride as the line's last key (the driver keeps the
    tail of a long line) and a false check or a failed leg makes bench.py exit
    non-zero; legs that did not run (None) do not count."""
    ok = bench.checks(None, None, None, None, {"all_decrypted_ok": True}, None, {"all_ok": True}, None)
    line = {"value": 1.0, "checks": ok, "leg_errors": None}
    line["checks_final"] = bench.checks_final(line)
    assert list(line)[-1] == "checks_final"
    assert line["checks_final"] == {"epoch_all_decrypted_ok": True, "coin_all_ok": True, "leg_errors": [],
                                    "all_ok": True}
    assert bench.exit_status(line) == 0
    bad = dict(line, checks=bench.checks({"oracle_match": False}, None, None, None, None, None, None, None))
    bad["checks_final"] = bench.checks_final(bad)
    assert bad["checks_final"]["decode_oracle_match"] is False and bench.exit_status(bad) == 1
    crashed = dict(line, leg_errors={"tdec": "RuntimeError: x"})
    crashed["checks_final"] = bench.checks_final(crashed)
    assert crashed["checks_final"]["leg_errors"] == ["tdec"] and bench.exit_status(crashed) == 1
    none_ran = {"checks": bench.checks(*[None] * 8), "leg_errors": None}
    none_ran["checks_final"] = bench.checks_final(none_ran)
    assert bench.exit_status(none_ran) == 0
