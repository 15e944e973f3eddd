#!/bin/bash
# LR kernel with the one-barrier meet + fused epilogue: parity, bench, phases.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2q
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -5; tail -2 $OUT/pytest.log; fatal $rc
run() {  # name, steps, warmup, env...
  local name=$1 st=$2 wu=$3; shift 3
  env "$@" timeout -k 10 120 python bench.py --steps $st --warmup $wu --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3), d['roofline']['kernel'])"
}
for rep in 1 2; do
  run lr20_$rep 20 5
  run lr_$rep 2000 200
done
run pair_1 2000 200 CE_LR_MFMA=0
CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --steps 30 > $OUT/diag_lr.json 2>&1; rc=$?; tail -1 $OUT/diag_lr.json; fatal $rc
echo ALL_OK
