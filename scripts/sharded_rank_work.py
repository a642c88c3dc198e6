"""Per-rank work of the coset-sharded proof, measured on ONE GPU.

An in-process group of R ranks (zkp_comm "local") shares the one device, so the
wall time of one sharded proof is the sum of every rank's device work, with the
exchanges done as device copies. wall_R / R is then the work each rank of an
R-GPU run does in parallel, and wall_R - wall_1 is the work sharding adds
(replicated stages, exchange copies, per-rank launch tails). The xGMI time of
the exchanges is not in it; DESIGN.md §6 adds it from the exchange volumes.

  python scripts/sharded_rank_work.py [--air mimc|agg|both] [--worlds 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--air", default="both")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--host", action="store_true", help="also time the host-trace entry point (row/column slices)")
    a = ap.parse_args()
    import bench
    from zk_stark_project_amd import _native
    from zk_stark_project_amd.sharded import prove_local_group

    worlds = [int(x) for x in a.worlds.split(",")]
    airs = ["mimc", "agg"] if a.air == "both" else [a.air]
    out = {}
    ctxs = [_native.Context(0) for _ in range(max(worlds))]
    for air in airs:
        wl = bench.make_workload(air, True, None, 8, 0, ctxs[0])
        width, n, opts, trace = wl["width"], wl["n"], wl["opts"], wl["trace"]
        pub = wl["prover"].get_pub_inputs(trace).to_elements()
        d = ctxs[0].alloc(trace.data.nbytes)
        ctxs[0].to_device(d, trace.data)
        ref = None
        rows = {}
        for R in worlds:
            for kind in (["dev", "host"] if a.host else ["dev"]):
                src, shape = (d, (width, n)) if kind == "dev" else (trace.data, None)

                def once():
                    return prove_local_group(R, wl["air_id"], src, pub, opts, contexts=ctxs[:R], shape=shape)
                res = once()  # warm: per-rank buffers, twiddles, coset tables
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    res = once()
                ms = (time.perf_counter() - t0) / a.steps * 1e3
                proof = res[0][0]
                ref = ref or proof
                same = proof == ref and all(p == proof for p, _ in res)
                rows[f"{kind}_w{R}"] = {"wall_ms": round(ms, 3), "per_rank_ms": round(ms / R, 3),
                                        "proof_identical": same}
                print(json.dumps({"air": air, "kind": kind, "world": R, **rows[f"{kind}_w{R}"]}), flush=True)
                if not same:
                    raise SystemExit(f"{air} {kind} world {R}: proof differs from world {worlds[0]}")
        w1 = rows.get("dev_w1")
        if w1:
            for k, v in rows.items():
                v["added_work_ms"] = round(v["wall_ms"] - w1["wall_ms"], 3)
        out[air] = {"workload": wl["workload"], **rows}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "sharded_rank_work.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("RANKWORKOK")


if __name__ == "__main__":
    main()
