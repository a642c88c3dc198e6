#!/bin/bash
# Round-4 GPU check: the non-slow GPU suite + the session C2/C3 channel test, a C2
# bench line with the session leg and the world-1 RCCL sharded-leg rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m "gpu and not slow" \
  > gpurun_out/check_tests.log 2>&1 || { tail -40 gpurun_out/check_tests.log; exit 1; }
tail -2 gpurun_out/check_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_stages.py \
  -k "c2_c3" > gpurun_out/check_slow.log 2>&1 || { tail -30 gpurun_out/check_slow.log; exit 1; }
tail -2 gpurun_out/check_slow.log
timeout -k 10 400 python bench.py --steps 20 --no-cpu-baseline --sharded-leg > gpurun_out/b_c2s.json 2> gpurun_out/b_c2s.err || { tail -20 gpurun_out/b_c2s.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/b_c2s.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'], d['roofline']['frac'], d['roofline']['valu_floor_frac'])
print('session', d['session'])
sh=d.get('sharded'); print('sharded', {k: sh[k] for k in sh if k not in ('fabric',)} if sh else None)
"
