#!/bin/bash
# A/B: the 11-stage 256-thread NTT passes held to 5 waves/SIMD (launch bounds; the DIT lo = 0
# pass 97 -> 92 VGPRs, no spills) against the previous build (kbench_lbprev), tuning only.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in kbench_lbprev kbench_ntt; do
    echo "== $v round $r"
    timeout -k 10 90 ./tests/native/$v 20 || exit 1
    timeout -k 10 90 ./tests/native/$v 18 || exit 1
  done
done > gpurun_out/kbench_lb5.txt 2>&1
grep -E "==|DIT lde 6 cols|pass only|DIT lde 1 col|DIF" gpurun_out/kbench_lb5.txt
