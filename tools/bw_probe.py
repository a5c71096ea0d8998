"""HBM ceiling probe for the encoder's traffic shape (A/B context only):
write-only fill of the shard buffer and a read+write copy, bench launch shape."""
import json

import torch

B, N, L = 8192, 64, 47663
S = (L + 15) // 16 * 16
dev = torch.device("cuda", 0)
shards = torch.empty((B, N * S), dtype=torch.uint8, device=dev)
pay = torch.empty((B, 1 << 20), dtype=torch.uint8, device=dev)
pay.fill_(3)


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


wb = shards.numel()
ms_fill = t(lambda: shards.fill_(7))
ms_copy = t(lambda: shards[:, : 2 << 20].unflatten(1, (2, 1 << 20)).copy_(pay.unsqueeze(1).expand(B, 2, 1 << 20)))
print(json.dumps({"fill_GBps": wb / ms_fill / 1e6, "fill_ms": ms_fill,
                  "copy_1r2w_GBps": B * 3 * (1 << 20) / ms_copy / 1e6, "copy_ms": ms_copy}))
