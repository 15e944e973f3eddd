#!/bin/bash
# Per-variant kernel times of the NN multi-agent step (rocprofv3 kernel
# trace; CE_LIB selects experiment builds), 1024 envs.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/nnv
for V in ${VARIANTS:-main}; do
  if [ $V = main ]; then L=""; else L=$V; fi
  CE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/nnv/$V -o r --output-format csv -- python3 bench.py --workload nn --envs ${NN_ENVS:-1024} --steps 6 --warmup 2 --profile-only > gpurun_out/nnv/$V.log 2>&1; rc=$?
  echo "== $V rc=$rc"; grep -E "nn_(agent|update|grad|step)_kernel" gpurun_out/nnv/$V/r_kernel_stats.csv | cut -d, -f1,4; [ $rc = 0 ] || exit $rc
done
