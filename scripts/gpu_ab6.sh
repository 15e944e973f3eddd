#!/bin/bash
# Round 6 A/B runner: the GPU tests (TESTS; default the whole -m gpu suite)
# and smoke on the current library, optional probes, then interleaved
# headline bench runs of the current library against experiment libraries
# (LIBS, CE_LIB names; "default" = the product build), long run and driver
# form, REPS repeats.  Every GPU step has its own time limit; any failure
# stops the script.
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab6}
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
if [ "${TESTS:-all}" != none ]; then
  if [ "${TESTS:-all}" = all ]; then T="tests -m gpu"; else T="$TESTS"; fi
  timeout -k 10 900 python -u -m pytest $T -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; fatal $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -5 $OUT/smoke.log; fatal $rc
fi
if [ "${PROBE:-0}" = 1 ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -w scripts/mfma4x4_layout.hip -o /tmp/mfma4x4_layout || exit 1
  timeout -k 10 60 /tmp/mfma4x4_layout > $OUT/mfma4x4_layout.json 2>&1; rc=$?
  echo "probe rc=$rc"; fatal $rc
fi
if [ "${DIAG:-0}" = 1 ]; then
  # phase stamps of the K-step kernel (CE_LIB=diag builds the stamp library
  # on the box from the pushed sources: it never travels)
  CE_LIB=diag timeout -k 10 600 python -u scripts/diag_persist.py --k 20 250 > $OUT/diag_persist.jsonl 2> $OUT/diag.err; rc=$?
  echo "diag rc=$rc"; cat $OUT/diag_persist.jsonl | cut -c1-600; fatal $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-default prev}; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic ${BENCH_ARGS:-} \
        > $OUT/bench_${lib}_$rep.json 2>> $OUT/bench.err; rc=$?; fatal $rc
    CE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        --no-measure-traffic ${BENCH_ARGS:-} > $OUT/bench20_${lib}_$rep.json 2>> $OUT/bench.err; rc=$?; fatal $rc
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); r=d['roofline']
    print(f.split('/')[-1], '%.4g'%d['value'], 'us/step %.4f'%(d['ms_per_step']*1e3), 'kernel %.4f'%(r.get('kernel_ms_median',0)*1e3), 'frac %.3f'%r['frac'], d.get('value_per_step_launch'))" $OUT/bench_*.json $OUT/bench20_*.json
echo ALL_OK
