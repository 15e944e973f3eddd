#!/bin/bash
# Round 5 timing A/B (timing-only builds, results not checked): the table
# exponential with a degree-3 polynomial (CE_LIB=texp1, one f64 FMA fewer per
# value, as a 2048-entry table would need) and additionally the 2^n scaling
# as an integer add on the table entry's exponent (CE_LIB=texp3, no
# v_ldexp_f64), against the shipped build; long run and driver form,
# interleaved.  The builds came from a CE_TEXP_X switch in exp_neg_tab
# (bit 0: drop the r^4/24 term; bit 1: the integer exponent add), removed
# once the 2048-entry table shipped (profiles/r05af_*).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05af
mkdir -p $OUT
for rep in 1 2 3; do
  for lib in default texp1 texp3; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    CE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_${lib}_$rep.json 2>> $OUT/bench.err || exit $?
    CE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        --no-measure-traffic > $OUT/bench20_${lib}_$rep.json 2>> $OUT/bench.err || exit $?
  done
done
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); print(f, '%.4g'%d['value'], round(d['ms_per_step']*1e3,4), d['roofline'].get('kernel_ms'))" $OUT/bench_*.json $OUT/bench20_*.json
