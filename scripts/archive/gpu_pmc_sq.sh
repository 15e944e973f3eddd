#!/bin/bash
# SQ counter passes over the bench's step kernel (one rocprofv3 run per pass;
# counter sets stay within the per-block limits).
set -u
cd "$(dirname "$0")/../.."
OUT=gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--profile-only --steps 300 --warmup 20 ${BENCH_ARGS:-}"
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU" \
            "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTRS -d $OUT/sq$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/sq$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/sq$i.log; exit $rc;; esac
done
