#!/bin/bash
# Config 5 (MultiOptLRs, 1024 envs x 4 agents): one-wave workgroups (64
# CUs) vs four-wave (16 CUs, mw4 build); parity first.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2r
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -5; tail -2 $OUT/pytest.log; fatal $rc
run() {  # name, envs, env...
  local name=$1 envs=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --workload multi --envs $envs --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', '%.3g' % d['value'], round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3))"
}
for rep in 1 2; do
  run w1_1024_$rep 1024
  run w4_1024_$rep 1024 CE_LIB=mw4
  run w1_8192_$rep 8192
  run w4_8192_$rep 8192 CE_LIB=mw4
done
echo ALL_OK
