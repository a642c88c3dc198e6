#!/bin/bash
# C3 with the upload: geometric column-group growth 1.5 (default) vs 1.25 vs 2.0.
set -o pipefail
for r in 1 2; do
  for gr in 150 125 200; do
    out=$(ZKP_UPLOAD_GROWTH=$gr timeout -k 10 120 python bench.py --air agg --no-cpu-baseline --no-verify --sustain-s 0 --steps 30)
    echo "growth=$gr $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["pcie_inclusive"]["ms_per_proof"])')"
  done
done
