#!/bin/bash
# MFMA kernel iteration: its tests, then the mnist-shape bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2c
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_mfma.log 2>&1; rc=$?
echo "pytest mfma rc=$rc"; tail -3 $OUT/pytest_mfma.log; fatal $rc
timeout -k 10 300 python bench.py --workload mnist --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_mnist.log 2>&1; rc=$?
echo "bench mnist rc=$rc"; tail -1 $OUT/bench_mnist.log | cut -c1-260; fatal $rc
python - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r2c/bench_mnist.log') if l.startswith('{')][-1])
print('mnist ms/step %.3f  kernel %.3f ms  frac %.3f' % (d['ms_per_step'], d['roofline']['kernel_ms_median'], d['roofline']['frac']))
PY
echo ALL_OK
