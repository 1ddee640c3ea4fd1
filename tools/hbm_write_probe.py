"""Practical HBM write / mixed bandwidth on this GPU (torch kernels, HIP events): the ceiling a
store-heavy kernel like K2 (6.4 GB written + 1.7 GB read per C2 call) can reach.  Dev aid."""
import json

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


n_w = 6_370_000_000 // 4
out = torch.empty(n_w, dtype=torch.int32, device="cuda")
t = timed(lambda: out.fill_(7))
res = {"write_only_fill_GBps": round(out.numel() * 4 / t / 1e9, 1)}
src = torch.ones(1_700_000_000 // 4, dtype=torch.int32, device="cuda")
half = out[: src.numel()]
t = timed(lambda: torch.add(src, 1, out=half))
res["read1_write1_GBps"] = round(2 * src.numel() * 4 / t / 1e9, 1)
t = timed(lambda: out.copy_(out.flip(0)) if False else out.zero_())
res["zero_GBps"] = round(out.numel() * 4 / t / 1e9, 1)
print(json.dumps(res))
