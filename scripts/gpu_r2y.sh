#!/bin/bash
# Two-class MFMA kernel: 8 waves x 2 tiles (default) vs 4 waves x 4 tiles
# per group (one wave per SIMD, software-pipelined group), parity for both.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2y
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; fatal $rc
CE_LIB=lrw4 timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_w4.log 2>&1; rc=$?
echo "pytest w4 rc=$rc"; grep -E "FAIL|Error" $OUT/pytest_w4.log | head -5; tail -1 $OUT/pytest_w4.log; fatal $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3))"
}
for rep in 1 2; do
  run w8_$rep
  run w4_$rep CE_LIB=lrw4
  run w4m2_$rep CE_LIB=lrw4 CE_LR_MODE=2
done
echo ALL_OK
