#!/bin/bash
# PMC passes over the NN multi-agent step (bench --workload nn): HBM bytes
# (FETCH_SIZE, WRITE_SIZE in separate passes) and SQ occupancy/stall counters,
# one rocprofv3 run per pass.
set -u
cd "$(dirname "$0")/../.."
OUT=gpurun_out/pmc_nn
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--workload nn --envs ${NN_ENVS:-512} --profile-only --steps 6 --warmup 2"
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/p$i.log; exit $rc;; esac
done
python3 scripts/pmc_nn.py
