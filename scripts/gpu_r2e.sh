#!/bin/bash
# LR MFMA kernel: its tests + the tests that run the default kernel, then the bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2e
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py tests/test_gpu_ref_pins.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -5; tail -2 $OUT/pytest.log; fatal $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; fatal $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20.log 2>&1; rc=$?
echo "bench20 rc=$rc"; fatal $rc
python - <<'PY'
import json
for f in ('bench', 'bench20'):
    d = json.loads([l for l in open('gpurun_out/r2e/%s.log' % f) if l.startswith('{')][-1])
    r = d['roofline']
    print(f, 'value %.4g  ms/step %.5f  kernel %.5f ms  frac %.4f  %s' % (d['value'], d['ms_per_step'], r['kernel_ms_median'], r['frac'], r['kernel']))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 2000 --warmup 100 > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; fatal $rc
head -3 $OUT/prof/run_kernel_stats.csv | cut -c1-160
echo ALL_OK
