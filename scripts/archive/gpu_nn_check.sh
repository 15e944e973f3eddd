#!/bin/bash
# NN problem session (OUT names the result directory): its GPU tests, the
# bench line, the kernel trace and the eval kernels' phase stamps (CE_DIAG
# build).  Every GPU step has its own time limit; any failure stops the script.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/nn}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_multinn.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; fatal $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload nn --steps 40 --warmup 4 --no-cpu-baseline > $OUT/bench_nn.log 2>&1; rc=$?
  echo "bench rep $rep: $(tail -1 $OUT/bench_nn.log | cut -c1-220)"; fatal $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload nn --profile-only --steps 10 --warmup 2 > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; fatal $rc
CE_LIB=diag timeout -k 10 200 python scripts/diag_nn.py --envs 1024 > $OUT/diag.json 2>&1; rc=$?
tail -1 $OUT/diag.json; fatal $rc
echo ALL_OK
