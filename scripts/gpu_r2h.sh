#!/bin/bash
# Fused MLP step kernel after the pipelining: tests, bench, phase stamps.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2h
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -5; tail -2 $OUT/pytest.log; fatal $rc
timeout -k 10 400 python bench.py --workload mlp --steps 20 --warmup 4 --no-cpu-baseline > $OUT/bench_mlp.log 2>&1; rc=$?
echo "bench mlp rc=$rc"; fatal $rc
python - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r2h/bench_mlp.log') if l.startswith('{')][-1])
print(json.dumps({k: d[k] for k in ('value', 'ms_per_step')}), json.dumps(d['roofline']))
PY
CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --workload mlp --steps 6 > $OUT/diag_mlp.json 2> $OUT/diag_mlp.err; rc=$?
echo "diag rc=$rc"; cat $OUT/diag_mlp.json; fatal $rc
echo ALL_OK
