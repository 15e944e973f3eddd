#!/bin/bash
# MultiOptLRs over OptimizeNN: GPU tests, bench lines at two env counts, rocprof.
set -u
cd "$(dirname "$0")/../.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_multinn.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_nn.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest_nn.log; fatal $rc
for E in ${NN_ENVS:-512 1024}; do
  timeout -k 10 300 python -u bench.py --workload nn --envs $E --steps ${NN_STEPS:-20} --warmup 4 ${NN_BENCH_FLAGS:---no-cpu-baseline} > $OUT/bench_nn_$E.json 2> $OUT/bench_nn_$E.err; rc=$?
  echo "== E=$E"; tail -c 600 $OUT/bench_nn_$E.json; fatal $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_nn -o nn --output-format csv -- python3 bench.py --workload nn --envs ${NN_PROF_ENVS:-1024} --steps 10 --warmup 2 --profile-only > $OUT/prof_nn.log 2>&1; rc=$?
echo "rocprof rc=$rc"; find $OUT/prof_nn -name '*kernel_stats.csv' | head -1 | xargs -r head -6; fatal $rc
