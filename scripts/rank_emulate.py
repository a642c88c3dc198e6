"""Device work of ONE rank of an R-rank coset-sharded proof, measured alone on one GPU.

Rank r of R runs prove_sharded over a loopback caller transport (every
collective fills each receive block with this rank's own data, through host
memory), so its kernels see exactly the shapes and counts of an R-GPU run while
no other rank shares the device. The library's per-launch HIP-event stats give
the rank's kernel time per proof by kernel (the exchanges are host copies here
and are not in it; DESIGN.md §6 prices them on xGMI from their volumes). The
proof bytes are meaningless (the exchanged data is wrong) — a run that the host
replay rejects still has its kernel stats.

  python scripts/rank_emulate.py [--air mimc|agg] [--world 8] [--rank 0] [--steps 2]
"""
import argparse
import ctypes
import json
import os
import sys
import time

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
    width, n, opts, trace = wl["width"], wl["n"], wl["opts"], wl["trace"]
    pub = wl["prover"].get_pub_inputs(trace).to_elements()
    d = ctx.alloc(trace.data.nbytes)
    ctx.to_device(d, trace.data)
    R, r = a.world, a.rank
    moved = {"a2a": 0, "ag": 0, "calls": 0}

    def a2a(send, recv, block):
        moved["a2a"] += (R - 1) * block
        moved["calls"] += 1
        for s in range(R):
            ctypes.memmove(recv + s * block, send + r * block, block)

    def ag(send, recv, nbytes):
        moved["ag"] += (R - 1) * nbytes
        moved["calls"] += 1
        if nbytes == 16:
            # the shortcut checks' flags (LastCol, GlobalUpdate pairing): the loopback
            # data makes them fail, and a valid proof's flags are zero, so report zeros
            # and time the path a valid proof takes (not a second, unshortcut proof)
            ctypes.memset(recv, 0, R * nbytes)
            return
        for s in range(R):
            ctypes.memmove(recv + s * nbytes, send, nbytes)

    comm = _native.host_comm(r, R, a2a, ag) if R > 1 else _native.local_group(1)[0]

    def once():
        try:
            ctx.prove_sharded(comm, wl["air_id"], d, pub, opts, shape=(width, n))
            return "ok"
        except _native.ZkpError as e:  # the loopback data may fail the host replay
            return f"rejected ({e})"
    status = once()  # warm: tables, buffers
    ctx.set_profiling(True)
    ctx.reset_stats()
    for k in moved:
        moved[k] = 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        status = once()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    st = ctx.stats_table()
    ctx.set_profiling(False)
    per = {k: {"launches": v["launches"] / a.steps, "ms": round(v["ms"] / a.steps, 4)} for k, v in st.items()}
    total = sum(v["ms"] for k, v in per.items() if not k.startswith("host_"))  # host_*: stage wall timers
    out = {"air": a.air, "workload": wl["workload"], "world": R, "rank": r, "status": status.split(" (")[0],
           "kernel_ms_per_proof": round(total, 3),
           "launches_per_proof": sum(v["launches"] for k, v in per.items() if not k.startswith("host_")),
           "wall_ms_with_host_loopback": round(wall, 3),
           "exchange_MiB_in_per_proof": round((moved["a2a"] + moved["ag"]) / a.steps / 2**20, 1),
           "a2a_MiB": round(moved["a2a"] / a.steps / 2**20, 1), "ag_MiB": round(moved["ag"] / a.steps / 2**20, 1),
           "collectives_per_proof": moved["calls"] / a.steps,
           "kernels": dict(sorted(per.items(), key=lambda kv: -kv[1]["ms"]))}
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"rank_emulate_{a.air}_w{R}_r{r}.json"), "w") as f:
        json.dump(out, f, indent=1)
    comm.close()


if __name__ == "__main__":
    main()
