#!/bin/bash
# Image-shape kernel: last feature on the VALU (F % 16 == 1) vs all-MFMA;
# parity first, then the mnist-shape bench for both and a kernel trace.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2ag
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error" $OUT/pytest.log | head -5; tail -1 $OUT/pytest.log; fatal $rc
for V in 1 0; do
  CE_GEN_TAIL=$V timeout -k 10 300 python bench.py --workload mnist --no-cpu-baseline > $OUT/b_tail$V.log 2>&1; rc=$?; fatal $rc
  python3 -c "import json; d=json.loads([l for l in open('$OUT/b_tail$V.log') if l.startswith('{')][-1]); print('tail$V', '%.4g' % d['value'], round(d['ms_per_step'],3), 'ms/step', d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_mnist -o run --output-format csv -- python3 bench.py --workload mnist --profile-only --steps 10 --warmup 2 > $OUT/prof_mnist.log 2>&1; rc=$?
echo "rocprof mnist rc=$rc"; fatal $rc
echo ALL_OK
