#!/bin/bash
# GPU: non-slow suite on the current library, then A/B against the saved previous build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m "gpu and not slow" \
  > gpurun_out/check_tests.log 2>&1 || { tail -40 gpurun_out/check_tests.log; exit 1; }
tail -1 gpurun_out/check_tests.log
ZKP_LIB=build_exp/two/libzkp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/two_tests.log 2>&1 || { tail -20 gpurun_out/two_tests.log; exit 1; }
tail -1 gpurun_out/two_tests.log
bash scripts/ab_libs.sh zk_stark_project_amd/libzkp.so build_exp/two/libzkp.so --stats > gpurun_out/ab_cur.txt 2>&1 || { tail -5 gpurun_out/ab_cur.txt; exit 1; }
cat gpurun_out/ab_cur.txt
