#!/bin/bash
# GPU check: session + stage tests, C3 and C2 bench lines with the session leg, the
# C2 per-kernel table (library events).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stages.py \
  > gpurun_out/check_stages.log 2>&1 || { tail -40 gpurun_out/check_stages.log; exit 1; }
tail -2 gpurun_out/check_stages.log
timeout -k 10 400 python bench.py --air agg --steps 10 --no-cpu-baseline > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err || { tail -20 gpurun_out/b_c3.err; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --no-cpu-baseline --stats > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || { tail -20 gpurun_out/b_c2.err; exit 1; }
python3 -c "
import json
for f in ('b_c2', 'b_c3'):
    d=json.loads(open('gpurun_out/%s.json' % f).read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'], d['roofline']['frac'], d['roofline']['valu_floor_frac'])
    print('  session', d['session']['session_ms'], d['session']['equals_zkp_prove_transcript'], d['session'].get('stage_ms'))
"
