#!/bin/bash
# Fused MLP step kernel: phase stamps (diag build) and SQ/TCC counters.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2g
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --workload mlp --steps 6 > $OUT/diag_mlp.json 2> $OUT/diag_mlp.err; rc=$?
echo "diag rc=$rc"; cat $OUT/diag_mlp.json; tail -3 $OUT/diag_mlp.err; fatal $rc
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/pmc_mlp/p$i -o run --output-format csv -- python3 bench.py --workload mlp --profile-only --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_mlp_p$i.log 2>&1; rc=$?
  echo "pmc pass $i rc=$rc"; fatal $rc
done
python3 scripts/pmc_generic.py $OUT/pmc_mlp mlp_step_kernel $OUT/pmc_mlp.json > $OUT/pmc_mlp_summary.txt 2>&1 || true
cat $OUT/pmc_mlp_summary.txt | head -40
echo ALL_OK
