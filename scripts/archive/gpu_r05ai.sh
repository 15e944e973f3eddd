#!/bin/bash
# Round 5 A/B: the per-step two-class kernel's exp table as one copy per wave
# at 4 waves, no barrier before the first lookup (CE_LIB=tabwave, built with
# -DCE_LR_TAB_WAVE=1), against one workgroup copy behind a barrier (default);
# the parity tests on the variant first, then value_per_step_launch and the
# headline, interleaved.  The switch was removed after this run: the
# per-wave copies were slower (profiles/r05ai_*).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05ai
mkdir -p $OUT
CE_LIB=tabwave timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_persist.py tests/test_gpu_parity.py tests/test_gpu_mfma.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in default tabwave; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_${lib}_$rep.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); print(f, '%.4g'%d['value'], round(d['ms_per_step']*1e3,4), '%.4g'%d.get('value_per_step_launch'))" $OUT/bench_*.json
