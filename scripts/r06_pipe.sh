#!/bin/bash
# k_ntt8_pipe (the 9-stage direct-load pass software-pipelined by LDS-DMA) against the
# library's pass, interleaved on one box (tests/native/kbench_ntt 20 / 18), tuning only.
set -o pipefail
mkdir -p gpurun_out
for v in kbench_ntt kbench_ntt_pipe kbench_ntt kbench_ntt_pipe; do
  echo "== $v"
  timeout -k 10 90 ./tests/native/$v 20 || exit 1
done > gpurun_out/kbench_pipe.txt 2>&1
cat gpurun_out/kbench_pipe.txt
