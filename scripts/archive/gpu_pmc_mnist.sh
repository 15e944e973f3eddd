#!/bin/bash
# SQ counters of the mnist-shape MFMA kernel, one rocprofv3 pass per group.
set -u
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r2d
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/pmc_mnist/p$i -o run --output-format csv -- python3 bench.py --workload mnist --profile-only --steps 2 --warmup 1 > $OUT/pmc_mnist_p$i.log 2>&1; rc=$?
  echo "pmc pass $i rc=$rc"; fatal $rc
done
python3 scripts/pmc_generic.py $OUT/pmc_mnist optimize_mfma_kernel $OUT/pmc_mnist.json > $OUT/pmc_mnist_summary.txt 2>&1 || true
cat $OUT/pmc_mnist_summary.txt | head -40
