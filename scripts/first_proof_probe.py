"""Where the first proof of a shape goes (verdict r04 #7): process-cold vs context-cold
vs warm, with the per-launch and host-stage table of a context-cold proof.
Run on the GPU box: python scripts/first_proof_probe.py [--air mimc|agg]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--air", default="mimc", choices=["mimc", "agg"])
    ap.add_argument("--after-mimc", action="store_true",
                    help="the bench's order: the context has proved C2 before the first proof of --air")
    args = ap.parse_args()
    import bench
    from zk_stark_project_amd import _native
    out = {}
    t0 = time.perf_counter()
    ctx = _native.Context(0)
    out["process_first_ctx_create_ms"] = (time.perf_counter() - t0) * 1e3
    wl = bench.make_workload(args.air, False, None, 8, 0, ctx)
    pub = wl["prover"].get_pub_inputs(wl["trace"]).to_elements()
    host = wl["trace"].data

    def once(c):
        t0 = time.perf_counter()
        c.prove(wl["air_id"], host, pub, wl["opts"])
        return (time.perf_counter() - t0) * 1e3
    if args.after_mimc:
        m = bench.make_workload("mimc", False, None, 8, 0, ctx)
        mp = m["prover"].get_pub_inputs(m["trace"]).to_elements()
        for _ in range(3):
            ctx.prove(m["air_id"], m["trace"].data, mp, m["opts"])
        ctx.reset_stats()
    ctx.set_profiling(True)
    out["process_cold_ms"] = once(ctx)
    ctx.set_profiling(False)
    tab = ctx.stats_table()
    out["process_cold_table"] = {k: {"n": v["launches"], "ms": round(v["ms"], 3)} for k, v in
                                 sorted(tab.items(), key=lambda kv: -kv[1]["ms"])}
    ctx.reset_stats()
    out["warm_ms"] = [once(ctx) for _ in range(3)]
    # the same trace in a fresh host buffer (a caller's next trace: pages never uploaded)
    import numpy as np
    fresh = []
    for _ in range(2):
        h2 = np.array(host, copy=True)
        t0 = time.perf_counter()
        ctx.prove(wl["air_id"], h2, pub, wl["opts"])
        fresh.append((time.perf_counter() - t0) * 1e3)
    out["warm_fresh_host_buffer_ms"] = fresh
    # the same warm context after the GPU sat idle (clock ramp / power state)
    idle = []
    for _ in range(3):
        time.sleep(0.5)
        idle.append(once(ctx))
    out["warm_after_idle_0.5s_ms"] = idle
    t0 = time.perf_counter()
    ctx2 = _native.Context(0)
    out["second_ctx_create_ms"] = (time.perf_counter() - t0) * 1e3
    ctx2.set_profiling(True)
    out["context_cold_ms"] = once(ctx2)
    ctx2.set_profiling(False)
    tab = ctx2.stats_table()
    out["context_cold_table"] = {k: {"n": v["launches"], "ms": round(v["ms"], 3)} for k, v in
                                 sorted(tab.items(), key=lambda kv: -kv[1]["ms"])}
    ctx2.reset_stats()
    ctx2.set_profiling(True)
    out["context_warm_ms"] = once(ctx2)
    ctx2.set_profiling(False)
    tab = ctx2.stats_table()
    out["context_warm_table"] = {k: {"n": v["launches"], "ms": round(v["ms"], 3)} for k, v in
                                 sorted(tab.items(), key=lambda kv: -kv[1]["ms"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
