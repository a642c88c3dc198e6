#!/bin/bash
# Round-6 closing run on the GPU box: the -m gpu suite, smoke(), then the default bench line
# (the driver's command). Each step time-limited, stopping at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q -v --timeout 120 --timeout-method thread > gpurun_out/t_final.log 2>&1 || { tail -30 gpurun_out/t_final.log; exit 1; }
tail -2 gpurun_out/t_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py > gpurun_out/b_final.json 2> gpurun_out/b_final.err || { tail -20 gpurun_out/b_final.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/b_final.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['step_ms'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['valu_floor_frac'])
print('c3', d['c3']['ms_per_step'], d['c3']['step_ms']['median'], d['c3']['first_proof_ms'])
print('rank', d['rank_emulation']['rank']['device_busy_ms_per_proof'])
"
