"""Probe: can two ranks of a torch.distributed "nccl" (RCCL) group share the
one GPU of a gpurun box?  Each rank all-gathers a small tensor and checks the
rank-major result.  Prints one JSON line per rank; exit status 0 iff both
ranks got the right answer.  Run under `timeout`."""
from __future__ import annotations

import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _rank(rank: int, world: int, port: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    out = {"rank": rank}
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        t = torch.full((4, 8), rank + 1, dtype=torch.int32, device=dev)
        g = torch.empty((world * 4, 8), dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(g, t)
        torch.cuda.synchronize()
        want = torch.cat([torch.full((4, 8), r + 1, dtype=torch.int32) for r in range(world)])
        out["ok"] = bool(torch.equal(g.cpu(), want))
        dist.destroy_process_group()
    except Exception as ex:  # reported, the parent decides
        out["ok"] = False
        out["error"] = f"{type(ex).__name__}: {ex}"[:400]
    q.put(out)


def main() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    for _ in procs:
        try:
            res.append(q.get(timeout=120))
        except Exception:
            res.append({"ok": False, "error": "timeout"})
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    for r in res:
        print(json.dumps(r), flush=True)
    return 0 if all(r.get("ok") for r in res) else 1


if __name__ == "__main__":
    sys.exit(main())
