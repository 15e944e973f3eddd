#!/bin/bash
# Fused MLP step kernel: MLP tests, the config-3 bench (fused), its rocprof stats.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2f
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error" $OUT/pytest.log | head -20; tail -2 $OUT/pytest.log; fatal $rc
timeout -k 10 400 python bench.py --workload mlp --steps 20 --warmup 4 --no-cpu-baseline > $OUT/bench_mlp.log 2>&1; rc=$?
echo "bench mlp rc=$rc"; fatal $rc
python - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r2f/bench_mlp.log') if l.startswith('{')][-1])
print(json.dumps({k: d[k] for k in ('value', 'ms_per_step')}), json.dumps(d['roofline']))
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload mlp --steps 12 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; fatal $rc
head -5 $OUT/prof/run_kernel_stats.csv | cut -c1-160
echo ALL_OK
