"""Device work of ONE rank of an R-rank coset-sharded proof, measured alone on one GPU
(bench.emulate_rank: loopback caller transport, the rank's kernels at the shapes of an
R-GPU run; device time = union of its kernel intervals). The default bench line carries
the C4 case as `rank_emulation`; this script runs any AIR / world / rank.

  python scripts/rank_emulate.py [--air mimc|agg] [--world 8] [--rank 0] [--steps 2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--air", default="mimc")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    import bench
    from zk_stark_project_amd import _native

    ctx = _native.Context(0)
    wl = bench.make_workload(a.air, True, None, 8, 0, ctx)
    out = {"air": a.air, "workload": wl["workload"], **bench.emulate_rank(ctx, wl, a.world, a.rank, a.steps)}
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"rank_emulate_{a.air}_w{a.world}_r{a.rank}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
