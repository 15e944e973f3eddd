#!/bin/bash
# PMC passes over the network workload (bench --workload mlp --hidden 256,256,
# 1024 envs): HBM bytes (FETCH_SIZE, WRITE_SIZE in separate passes), SQ
# occupancy / stall counters, L2 hit counters; one rocprofv3 run per pass,
# each under its own time limit.  Summaries per kernel: scripts/pmc_generic.py.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/pmc_net}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--workload mlp --hidden ${HIDDEN:-256,256} --envs ${ENVS:-1024} --batch-size 32 --profile-only --steps 4 --warmup 1"
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/p$i.log; exit $rc;; esac
done
for K in net_fwd_kernel net_grad_kernel net_update_kernel net_bwd_kernel; do
  python3 scripts/pmc_generic.py $OUT $K $OUT/$K.json > /dev/null
done
echo PMC_OK
