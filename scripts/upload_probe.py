"""zkp_prove from pageable vs pinned host traces vs device-resident (C2), tuning only."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from zk_stark_project_amd import AIR_MIMC, MimcProver, ProofOptions, _native  # noqa: E402

ctx = _native.Context(0)
opts = ProofOptions(40, 8, 21)
p = MimcProver(opts, ctx)
tr = p.build_trace(42 * 10**6, 1 << 20)
pub = p.get_pub_inputs(tr).to_elements()
host = tr.data
pinned_t = torch.empty(host.shape, dtype=torch.int64).pin_memory()
pinned = pinned_t.numpy().view(np.uint64)
pinned[...] = host
d = ctx.alloc(host.nbytes)
ctx.to_device(d, host)


def t(fn, k=60):
    for _ in range(5):
        fn()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return (time.perf_counter() - t0) / k * 1e3


for r in range(2):
    a = t(lambda: ctx.prove(AIR_MIMC, host, pub, opts))
    b = t(lambda: ctx.prove(AIR_MIMC, pinned, pub, opts))
    c = t(lambda: ctx.prove_device(AIR_MIMC, d, 1, 1 << 20, pub, opts))
    print(f"pageable {a:.3f} ms  pinned {b:.3f} ms  device-resident {c:.3f} ms", flush=True)
