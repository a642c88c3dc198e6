#!/bin/bash
# World-1 runs of the sharded configurations (the numbers DESIGN.md §6's per-rank
# model scales): C4 = MiMC 2^22 (BASELINE configs[3]) and C5 = GlobalUpdate
# 2^20 x 120, 256 updates, trace built on the device (configs[4]).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --mode sharded --steps 5 --warmup 1 --no-cpu-baseline --sustain-s 0 --stats \
  > gpurun_out/c4_w1.json 2> gpurun_out/c4_w1.err || { tail -20 gpurun_out/c4_w1.err; exit 1; }
timeout -k 10 300 python bench.py --mode sharded --air agg --steps 3 --warmup 1 --no-cpu-baseline --sustain-s 0 \
  --stats > gpurun_out/c5_w1.json 2> gpurun_out/c5_w1.err || { tail -20 gpurun_out/c5_w1.err; exit 1; }
echo SHARDOK
