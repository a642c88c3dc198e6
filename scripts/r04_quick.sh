#!/bin/bash
# Round-4 quick GPU check: butterfly micro-benchmark (edge check + floor), the
# parity/stage tests that touch the changed paths, then a C2 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tests/native/ubench_bfly --check > gpurun_out/ubench_check.txt 2>&1 || { cat gpurun_out/ubench_check.txt; exit 1; }
cat gpurun_out/ubench_check.txt
timeout -k 10 120 tests/native/ubench_bfly > gpurun_out/ubench_bfly.txt 2>&1 || { cat gpurun_out/ubench_bfly.txt; exit 1; }
cat gpurun_out/ubench_bfly.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_sharded.py -k "not c5 and not c3 and not c4" > gpurun_out/quick_tests.log 2>&1 || { tail -30 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || { tail -20 gpurun_out/b_c2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/b_c2.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])
print(d['launches']['by_kernel_ms'])
"
