#!/bin/bash
# PMC profile of the reference's TrainingUpdate proof shape (scripts/tu_probe.py: n = 8192,
# w = 240, blowup 16), the same passes as scripts/profile_round.sh.
set -u
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_r06_tu
mkdir -p $OUT
P="python3 $ROOT/scripts/tu_probe.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $P > $OUT/trace.log 2>&1 || { echo "kernel-trace pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $P > $OUT/fetch.log 2>&1 || { echo "FETCH_SIZE pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $P > $OUT/write.log 2>&1 || { echo "WRITE_SIZE pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU \
  --output-format csv -d $OUT/sq1 -o run -- $P > $OUT/sq1.log 2>&1 || { echo "SQ pass 1 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY \
  SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq2 -o run -- $P > $OUT/sq2.log 2>&1 || { echo "SQ pass 2 failed"; exit 1; }
python3 $ROOT/scripts/pmc_traffic.py $OUT > $OUT/traffic.txt || { echo "post-processing failed"; exit 1; }
mkdir -p $OUT/sq && cp -r $OUT/sq1 $OUT/sq2 $OUT/sq/ && python3 $ROOT/scripts/pmc_sq.py $OUT/sq > $OUT/sq.txt || { echo "SQ post-processing failed"; exit 1; }
head -16 $OUT/sq.txt
head -16 $OUT/traffic.txt
