#!/bin/bash
# Round 5 timing-only diagnostics of the K-step kernel (outputs wrong, not
# checked): CE_LIB=noconf reads conflict-free table entries (lane + 64 r
# instead of the random index: what the table's LDS bank conflicts cost),
# CE_LIB=noepi skips the epilogue waves' parameter roles (what the
# epilogue's f64 work costs the row waves).  Long run, interleaved.  The
# CE_X_NOCONF / CE_X_NOEPI switches were removed after this run
# (profiles/r05al_*).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05al
mkdir -p $OUT
for rep in 1 2 3; do
  for lib in default noconf noepi; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_${lib}_$rep.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); print(f, '%.4g'%d['value'], round(d['ms_per_step']*1e3,4))" $OUT/bench_*.json
