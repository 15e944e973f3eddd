#!/bin/bash
# SQ / TCC counters of the MLP step kernel (CE_LIB build given as $1; KNAME
# selects another kernel, e.g. mlp_info_kernel with CE_MLP_PHASES=info), one
# pass per group.
set -u
cd "$(dirname "$0")/../.."
V=${1:-default}
OUT=${OUT:-gpurun_out/pmc_mlp_$V}
mkdir -p $OUT
export TMPDIR=/tmp
if [ $V != default ]; then export CE_LIB=$V; fi
export MLP_ENVS=4096
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python3 scripts/mlp_time.py > $OUT/p$i.log 2>&1; rc=$?
  echo "pmc pass $i rc=$rc"; fatal $rc
done
python3 scripts/pmc_generic.py $OUT ${KNAME:-mlp_step_kernel} $OUT/summary.json > $OUT/summary.txt 2>&1 || true
head -30 $OUT/summary.txt
echo ALL_OK
