#!/bin/bash
# Timing experiments on the NTT pass kernel (results are NOT proofs): builds
# libzkp variants with -DZKP_EXP_NOBFLY (data movement only) and
# -DZKP_EXP_NOGMEM (arithmetic + LDS only) into build_exp/. Run on the GPU box
# with: scripts/ntt_experiments.sh run  (swaps each variant in, runs bench.py --stats)
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/zk_stark_project_amd/csrc
if [ "${1:-build}" = build ]; then
  for v in NOBFLY NOGMEM; do
    mkdir -p $ROOT/build_exp/$v
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DZKP_EXP_$v -c $CS/kernels.hip -o $ROOT/build_exp/$v/kernels.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/build_exp/$v/libzkp.so $ROOT/build_exp/$v/kernels.o \
      $CS/build/prover.o $CS/build/verifier.o $CS/build/comm.o -Wl,--exclude-libs,ALL -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  done
else
  OUT=$ROOT/gpurun_out/ntt_exp
  mkdir -p $OUT
  cp $ROOT/zk_stark_project_amd/libzkp.so $OUT/libzkp.real.so
  for v in NOBFLY NOGMEM; do
    cp $ROOT/build_exp/$v/libzkp.so $ROOT/zk_stark_project_amd/libzkp.so
    timeout -k 10 200 python3 $ROOT/bench.py --stats --no-cpu-baseline --no-verify --steps 5 > $OUT/$v.log 2>&1
    timeout -k 10 200 python3 $ROOT/bench.py --air agg --stats --no-cpu-baseline --no-verify --steps 3 > $OUT/${v}_agg.log 2>&1
  done
  cp $OUT/libzkp.real.so $ROOT/zk_stark_project_amd/libzkp.so; rm -f $OUT/libzkp.real.so
fi
