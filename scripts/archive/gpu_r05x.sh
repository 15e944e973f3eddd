#!/bin/bash
# Round 5: the headline kernel's time per step three ways -- HIP events in a
# separate loop after the timed region (roofline.kernel_ms_median), HIP
# events around every launch inside the timed region (--timed-events), and
# rocprofv3's kernel trace of the same workload.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05x
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic > $OUT/bench_$i.json 2>> $OUT/bench.err || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-measure-traffic --timed-events > $OUT/bench_ev_$i.json 2>> $OUT/bench.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-measure-traffic > $OUT/prof_bench.json 2> $OUT/prof.log || exit $?
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads([l for l in open(f).read().splitlines() if l.startswith('{')][-1]); r=d['roofline']; print(f, round(d['ms_per_step']*1e3,4), round(r['kernel_ms_median']*1e3,4), r.get('kernel_ms_timed_region'))" $OUT/bench*.json $OUT/prof_bench.json
grep persist $OUT/prof/run_kernel_stats.csv | cut -c1-200
