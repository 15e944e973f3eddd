#!/bin/bash
# (CE_LP_ROW_WAVES was an experiment build's switch: the 8-row-wave variant measured
# slower and was withdrawn; the switch is gone from the tree.)
# Round 5 A/B: the wave-specialised K-step kernel with 8 row waves (two per
# SIMD, CE_LP_ROW_WAVES=8) against 4, interleaved; phase stamps of both.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05q
mkdir -p $OUT
for i in 1 2; do
  for rw in 4 8; do
    CE_LP_ROW_WAVES=$rw timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic \
        > $OUT/bench_rw${rw}_$i.json 2> $OUT/bench.err || exit $?
    CE_LP_ROW_WAVES=$rw timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        --no-measure-traffic --repeat-timed 5 > $OUT/bench20_rw${rw}_$i.json 2>> $OUT/bench.err || exit $?
  done
done
CE_LP_ROW_WAVES=8 CE_LIB=diag timeout -k 10 240 python -u scripts/diag_persist.py --k 20 250 > $OUT/diag_rw8.jsonl 2> $OUT/diag.err || exit $?
cat $OUT/diag_rw8.jsonl
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['roofline']['kernel'], d['value'], d['ms_per_step']*1e3, d.get('timed_repeats_ms'))" $OUT/bench*_rw*.json
