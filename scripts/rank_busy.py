#!/usr/bin/env python3
"""Device-busy time per proof of one emulated rank (tuning/measurement only): the union of
its kernels' execution intervals in a `rocprofv3 --kernel-trace` of scripts/rank_emulate.py,
over the last `steps` proofs. Unlike the library's per-launch event sum it counts time
once when kernels of two streams overlap (the sharded composition LDEs alternate streams).
  rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python scripts/rank_emulate.py ... --steps S
  python scripts/rank_busy.py OUT/run_kernel_trace.csv <launches per proof> <S>"""
import csv
import json
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "__amd_rocclr" not in r["Kernel_Name"]]
    lpp, steps = int(sys.argv[2]), int(sys.argv[3])
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    iv = iv[-lpp * steps:]
    busy, cur_s, cur_e, total = 0, None, None, 0
    for s, e in iv:
        total += e - s
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(json.dumps({"dispatches": len(iv), "busy_ms_per_proof": round(busy / steps / 1e6, 3),
                      "sum_ms_per_proof": round(total / steps / 1e6, 3)}))


if __name__ == "__main__":
    main()
