#!/bin/bash
# Round-4 checks, second form (OUT names the result directory): the config-3
# train phase alone (CE_MLP_PHASES=train) and the fused step, each with the
# LDS / instruction counter pass and the byte passes; then the NN step's PMC
# at 1024 envs.  Every GPU step has its own time limit; any failure stops.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/chk4b}
mkdir -p $OUT
export TMPDIR=/tmp MLP_ENVS=4096
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for PH in train fused; do
  if [ $PH = train ]; then export CE_MLP_PHASES=train; K=mlp_train_kernel; else unset CE_MLP_PHASES; K=mlp_step_kernel; fi
  i=0; mkdir -p $OUT/$PH
  for CTRS in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/$PH/p$i -o run --output-format csv -- python3 scripts/mlp_time.py > $OUT/$PH/p$i.log 2>&1; rc=$?
    echo "mlp $PH pmc pass $i rc=$rc"; fatal $rc
  done
  python3 scripts/pmc_generic.py $OUT/$PH $K $OUT/$PH/summary.json > $OUT/$PH/summary.txt 2>&1 || true
  head -30 $OUT/$PH/summary.txt
done
unset CE_MLP_PHASES
NN_ENVS=1024 bash scripts/gpu_pmc_nn.sh > $OUT/pmc_nn.txt 2>&1 || { tail -5 $OUT/pmc_nn.txt; exit 1; }
cp gpurun_out/pmc_nn/summary.json $OUT/pmc_nn_summary.json
echo ALL_OK
