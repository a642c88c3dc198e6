#!/bin/bash
# A/B of two libzkp builds on one box (tuning only): scripts/ab_libs.sh <lib A> <lib B> [bench args]
# alternates A and B three times; prints ms_per_step (zkp_prove from the host trace), the
# trace-resident ms, the dominant kernel's live average launch and the per-kernel ms of the
# profiled proofs.
set -o pipefail
A=$1; B=$2; shift 2
for r in 1 2 3; do
  for L in "$A" "$B"; do
    out=$(ZKP_LIB=$L timeout -k 10 180 python bench.py --no-cpu-baseline --no-verify --sustain-s 0 --no-concurrent \
          --no-c3 --no-reference-flow --no-rank-emulation --steps 40 "$@") || exit 1
    echo "$L $(echo "$out" | python -c '
import json,sys
d=json.loads(sys.stdin.readline()); k=d["launches"]["by_kernel_ms"]
print(d["ms_per_step"], d["trace_resident"]["ms_per_proof"], d["roofline"]["kernel"], d["roofline"]["avg_launch_ms"],
      " ".join(f"{n}={k[n]}" for n in list(k)[:10]))')"
  done
done
