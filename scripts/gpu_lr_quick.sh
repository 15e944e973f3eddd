#!/bin/bash
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2h
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "lr_mfma or golden" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; fatal $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?; fatal $rc
python - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r2h/bench.log') if l.startswith('{')][-1])
r = d['roofline']
print('value %.4g  ms/step %.5f  kernel %.5f ms  frac %.4f  %s' % (d['value'], d['ms_per_step'], r['kernel_ms_median'], r['frac'], r['kernel']))
PY
CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --steps 30 > $OUT/diag_lr.json 2>&1; rc=$?
tail -1 $OUT/diag_lr.json; exit $rc
