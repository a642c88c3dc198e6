"""Host->HBM copy rates on the box (pageable numpy vs pinned), for DESIGN.md §5."""
import time
import numpy as np
import torch

for mb in (16, 128, 512):
    n = mb << 20
    src = np.random.default_rng(1).integers(0, 255, n, dtype=np.uint8)
    dst = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    pin = torch.from_numpy(src.copy()).pin_memory()
    for name, s in (("pageable", torch.from_numpy(src)), ("pinned", pin)):
        dst.copy_(s, non_blocking=False)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            dst.copy_(s, non_blocking=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 5
        print(f"{mb:4d} MB {name:8s} {dt * 1e3:8.3f} ms  {n / dt / 1e9:6.1f} GB/s", flush=True)
