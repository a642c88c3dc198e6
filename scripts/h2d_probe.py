"""H2D upload rates on the box (tuning only): 16 MiB pageable vs pinned vs chunked pageable.

  python scripts/h2d_probe.py
"""
import time

import numpy as np
import torch


def rate(fn, nbytes, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return dt * 1e3, nbytes / dt / 1e9


def main():
    for mb in (16, 64, 256):
        nb = mb << 20
        host = np.random.randint(0, 2**63, size=nb // 8, dtype=np.int64)
        ht = torch.from_numpy(host)
        pin = ht.pin_memory()
        dev = torch.empty_like(ht, device="cuda")
        ms, gbs = rate(lambda: dev.copy_(ht, non_blocking=True), nb)
        print(f"{mb:4d} MiB pageable  {ms:8.3f} ms  {gbs:6.1f} GB/s", flush=True)
        ms, gbs = rate(lambda: dev.copy_(pin, non_blocking=True), nb)
        print(f"{mb:4d} MiB pinned    {ms:8.3f} ms  {gbs:6.1f} GB/s", flush=True)
        for ch in (4, 16):
            step = ht.numel() // ch

            def chunked():
                for i in range(ch):
                    dev[i * step:(i + 1) * step].copy_(ht[i * step:(i + 1) * step], non_blocking=True)
            ms, gbs = rate(chunked, nb)
            print(f"{mb:4d} MiB pageable/{ch:<2d} {ms:8.3f} ms  {gbs:6.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
