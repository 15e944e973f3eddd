#!/bin/bash
# One gpurun session: GPU tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "GPU step failed hard (rc=$1), stopping"; exit $1;; esac; }
ulimit -n > $OUT/ulimit.txt
nproc >> $OUT/ulimit.txt
lscpu | grep "Model name" >> $OUT/ulimit.txt
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -2 $OUT/bench.log; fatal $rc
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 300 python scripts/sweep.py > $OUT/sweep.log 2>&1; rc=$?
  echo "sweep rc=$rc"; cat $OUT/sweep.log | grep envs; fatal $rc
fi
if [ -n "${PROFILE:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 2000 --warmup 100 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -3 $OUT/prof.log; fatal $rc
fi
exit 0
