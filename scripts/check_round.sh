#!/bin/bash
# Parity/stage/sharded GPU tests, C3 A/B of the linear evaluation, one-rank emulation.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_stages.py tests/test_gpu_sharded.py tests/test_gpu_sharded_gloo.py tests/test_gpu_comm.py \
  -k "not oracle_bytes" > gpurun_out/round_tests.log 2>&1 || { tail -30 gpurun_out/round_tests.log; exit 1; }
tail -2 gpurun_out/round_tests.log
timeout -k 10 400 bash scripts/ab_env.sh ZKP_EVAL_POINTWISE=1 --air agg > gpurun_out/ab_lin.txt 2>&1 || { cat gpurun_out/ab_lin.txt; exit 1; }
cat gpurun_out/ab_lin.txt
bash scripts/rank_emulate.sh
