#!/bin/bash
# Round-4 checks (OUT names the result directory): the image-shape kernel
# tests and bench (single forward chain), the config-3 step kernel's PMC
# (LDS bank conflicts after the W2 stage stride change) and the NN step's PMC
# at 1024 envs.  Every GPU step has its own time limit; any failure stops.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/chk4}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest_mfma.log 2>&1; rc=$?
tail -1 $OUT/pytest_mfma.log; fatal $rc
timeout -k 10 300 python bench.py --workload mnist --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_mnist.log 2>&1; rc=$?
tail -1 $OUT/bench_mnist.log | cut -c1-300; fatal $rc
OUT=$OUT/pmc_mlp bash scripts/gpu_pmc_mlp.sh || exit $?
NN_ENVS=1024 bash scripts/gpu_pmc_nn.sh > $OUT/pmc_nn.txt 2>&1 || { tail -5 $OUT/pmc_nn.txt; exit 1; }
cp gpurun_out/pmc_nn/summary.json $OUT/pmc_nn_summary.json
echo ALL_OK
