"""Diagnostics (GPU box): per-launch device time of the Merkle tree kernels for
single-column row commitments of 2^k rows (zkp_merkle_commit_rows), so the
latency floor of the LDS-fused top (merkle_top9) can be read against its size."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zk_stark_project_amd import _native  # noqa: E402


def main():
    ctx = _native.Context(0)
    for k in (10, 11, 13, 15, 17, 19):
        cols = np.zeros((1, 1 << k, 2), dtype=np.uint64)
        cols[0, :, 0] = np.arange(1 << k, dtype=np.uint64)
        for _ in range(3):
            ctx.merkle_commit_rows(cols)
        ctx.reset_stats()
        ctx.set_profiling(True)
        reps = 20
        for _ in range(reps):
            ctx.merkle_commit_rows(cols)
        ctx.set_profiling(False)
        st = ctx.stats_table()
        line = " ".join(f"{n}={v['ms'] / reps * 1e3:.1f}us/{v['launches'] // reps}" for n, v in sorted(st.items())
                        if not n.startswith("host_"))
        print(f"rows=2^{k}: {line}", flush=True)


if __name__ == "__main__":
    main()
