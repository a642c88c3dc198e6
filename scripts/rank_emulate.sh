#!/bin/bash
# One rank's device work at world 8 vs world 1 (scripts/rank_emulate.py), C4 and C5.
set -o pipefail
mkdir -p gpurun_out
for air in mimc agg; do
  for w in 1 8; do
    timeout -k 10 240 python -u scripts/rank_emulate.py --air $air --world $w --rank 0 > gpurun_out/emu_${air}_w$w.log 2>&1 \
      || { tail -20 gpurun_out/emu_${air}_w$w.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/rank_emulate_${air}_w${w}_r0.json')); print({k: d[k] for k in d if k != 'by_kernel_ms'})"
  done
done
echo EMUOK
