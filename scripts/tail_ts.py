"""Phase times inside k_fri_tail from an instrumented build (build_exp/ts, wall_clock64
stamps at the phase boundaries; tuning only). ZKP_LIB must point at that build."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zk_stark_project_amd import _native  # noqa: E402


def main():
    ctx = _native.Context(0)
    wl = bench.make_workload("mimc", False, None, 8, 0, ctx)
    pub = wl["prover"].get_pub_inputs(wl["trace"]).to_elements()
    host = wl["trace"].data
    d = ctx.alloc(host.nbytes)
    ctx.to_device(d, host)
    lib = ctx.lib
    buf = (ctypes.c_ulonglong * 64)()
    acc = {}
    N = 20
    for i in range(N + 3):
        ctx.prove_device(wl["air_id"], d, wl["width"], wl["n"], pub, wl["opts"])
        assert lib.zkp_debug_tail_ts(buf) == 0
        if i < 3:
            continue
        nl = buf[43]
        marks = [(0, "start")]
        for l in range(nl):
            marks += [(1 + 4 * l, f"L{l} leaves"), (2 + 4 * l, f"L{l} tree"), (3 + 4 * l, f"L{l} coin"),
                      (4 + 4 * l, f"L{l} fold")]
        marks += [(40, "rem coeffs"), (41, "rem hash"), (42, "rem reseed")]
        for (a, _), (b, name) in zip(marks, marks[1:]):
            acc[name] = acc.get(name, 0.0) + (buf[b] - buf[a]) * 10e-3  # 100 MHz ticks -> us
        acc["total"] = acc.get("total", 0.0) + (buf[42] - buf[0]) * 10e-3
    for k, v in acc.items():
        print(f"{k:14s} {v / N:7.2f} us")


if __name__ == "__main__":
    main()
