"""Achievable HBM rate on this box for a read+write stream (the realistic ceiling of a kernel that
reads ~N bytes and writes ~N bytes): device-to-device copies of 0.65 GB buffers, HIP events."""
import json
import torch

torch.cuda.set_device(0)
res = {}
for n in (651_915_480 // 16 * 16, 1_299_408_096 // 16 * 16):
    a = torch.empty(n, dtype=torch.uint8, device="cuda").fill_(3)
    b = torch.empty_like(a)
    for name, fn in (("torch_copy_u8", lambda: b.copy_(a)),
                     ("torch_copy_i64", lambda: b.view(torch.int64).copy_(a.view(torch.int64)))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res[f"{name}_{n // 1_000_000}MB"] = {"ms": round(ms, 4),
                                             "rw_GBps": round(2 * n / ms / 1e6, 1)}
    del a, b
print(json.dumps(res))
