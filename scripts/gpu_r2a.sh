#!/bin/bash
# Round-2 first GPU pass: f64 MFMA/VALU rates, the -m gpu suite, smoke, the
# bench at the driver's settings and at defaults, the gather modes on one GPU
# (a real 1-rank RCCL collective), and a rocprofv3 kernel trace.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2a
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 60 scripts/bin/mfma_f64 > $OUT/mfma_f64.jsonl 2>&1; rc=$?
echo "mfma rc=$rc"; cat $OUT/mfma_f64.jsonl; fatal $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; fatal $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1; rc=$?
echo "bench driver-settings rc=$rc"; tail -1 $OUT/bench_driver.log | cut -c1-400; fatal $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench_default.log 2>&1; rc=$?
echo "bench default rc=$rc"; tail -1 $OUT/bench_default.log | cut -c1-300; fatal $rc
timeout -k 10 300 python bench.py --force-gather --steps 300 --warmup 30 --no-cpu-baseline > $OUT/bench_gather.log 2>&1; rc=$?
echo "bench gather rc=$rc"; tail -1 $OUT/bench_gather.log | cut -c1-300; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 2000 --warmup 100 > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; fatal $rc
echo ALL_OK
