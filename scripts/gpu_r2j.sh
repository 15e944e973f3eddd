#!/bin/bash
# Interleaved multi-row f64 step (rows_multi): parity, bench at U = 2 / 4,
# phase stamps.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2j
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; fatal $rc
for U in 2 4 2 4; do
  CE_PAIR_U=$U timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/b_$U.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_$U.log') if l.startswith('{')][-1]); print('U=$U', round(d['ms_per_step']*1e3,3), 'us/step; kernel', round(d['roofline']['kernel_ms_median']*1e3,3), d['roofline']['kernel'])"
done
CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --steps 30 > $OUT/diag_pair.json 2>&1; rc=$?; tail -1 $OUT/diag_pair.json; fatal $rc
echo ALL_OK
