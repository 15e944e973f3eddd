#!/bin/bash
# Two-class MFMA kernel: W' formed once per workgroup in LDS (default) vs
# per-wave W loads (wpw build), at 4 / 8 / 16 waves; parity first.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ad
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py tests/test_gpu_ref_pins.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -5; tail -1 $OUT/pytest.log; fatal $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_$name.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$name.log') if l.startswith('{')][-1]); print('$name', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3))"
}
for rep in 1 2; do
  for W in 4 8 16; do
    run lds_w${W}_$rep CE_LR_WAVES=$W
    run wpw_w${W}_$rep CE_LR_WAVES=$W CE_LIB=wpw
  done
done
CE_LR_WAVES=16 CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --steps 30 > $OUT/diag_w16.json 2>&1; rc=$?
tail -1 $OUT/diag_w16.json; fatal $rc
echo ALL_OK
