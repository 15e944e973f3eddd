#!/bin/bash
# MFMA runtime-shape kernel: its tests, the mnist-shape bench + kernel trace,
# and the graph-captured gather modes on one GPU.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2b
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_mfma.log 2>&1; rc=$?
echo "pytest mfma rc=$rc"; grep -E "PASS|FAIL|Error" $OUT/pytest_mfma.log | head -30; tail -3 $OUT/pytest_mfma.log; fatal $rc
timeout -k 10 300 python bench.py --workload mnist --steps 10 --warmup 2 --cpu-seconds 8 > $OUT/bench_mnist.log 2>&1; rc=$?
echo "bench mnist rc=$rc"; tail -1 $OUT/bench_mnist.log | cut -c1-600; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_mnist -o run --output-format csv -- python3 bench.py --workload mnist --profile-only --steps 8 --warmup 2 > $OUT/prof_mnist.log 2>&1; rc=$?
echo "rocprof mnist rc=$rc"; fatal $rc
timeout -k 10 300 python bench.py --force-gather --steps 300 --warmup 30 --no-cpu-baseline > $OUT/bench_gather.log 2>&1; rc=$?
echo "bench gather rc=$rc"; tail -1 $OUT/bench_gather.log | cut -c1-200; fatal $rc
echo ALL_OK
