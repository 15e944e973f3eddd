#!/bin/bash
# Config 5 A/B: the multi GPU tests on the current library, then interleaved
# config-5 bench runs (long run and driver form) of the K-step kernel forms
# (FORMS: CE_MULTI_FORM values, "four" = the default) and experiment
# libraries (LIBS, CE_LIB names).  Every GPU step has its own time limit;
# any failure stops the script.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/abm}
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
if [ "${TESTS:-multi}" != none ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; fatal $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${FORMS:-four three} ${LIBS:-}; do
    case $v in four|five|six|three|one) F=$v; L="";; *) F=${LIB_FORM:-}; L=$v;; esac
    CE_MULTI_FORM=$F CE_LIB=$L timeout -k 10 300 python -u bench.py --workload multi --no-cpu-baseline \
        --no-measure-traffic > $OUT/bench_${v}_$rep.json 2>> $OUT/bench.err; rc=$?; fatal $rc
    CE_MULTI_FORM=$F CE_LIB=$L timeout -k 10 300 python -u bench.py --workload multi --steps 20 --warmup 5 \
        --no-cpu-baseline --no-measure-traffic > $OUT/bench20_${v}_$rep.json 2>> $OUT/bench.err; rc=$?; fatal $rc
  done
done
for f in $OUT/bench*_*.json; do
  python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$(basename $f)', '%.4g' % d['value'], 'us/step %.4f' % (d['ms_per_step']*1e3), 'kernel %.4f' % (r.get('kernel_ms_median',0)*1e3), r.get('kernel'))"
done
echo ALL_OK
