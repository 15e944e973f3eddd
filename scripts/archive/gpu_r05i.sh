#!/bin/bash
# Round 5: the chunk schedule's fixed cost per collective at world 1 (RCCL,
# in place: nothing moves), kernel traces of the persistent kernels, and the
# bench lines with their in-run traffic passes.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05i
mkdir -p $OUT
for c in 1 5 10 20; do
  timeout -k 10 200 python -u bench.py --force-gather --chunk-steps $c --steps 400 --warmup 40 --no-cpu-baseline --no-measure-traffic > $OUT/fg_c$c.json 2>> $OUT/bench.err || exit $?
done
timeout -k 10 200 python -u bench.py --force-gather --chunk-steps 10 --steps 20 --warmup 5 --no-cpu-baseline --no-measure-traffic > $OUT/fg20_c10.json 2>> $OUT/bench.err || exit $?
python - $OUT/fg*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f, 'value %.4g' % d['value'], {k: round(v * 1e3, 3) for k, v in d.get('ms_per_step_modes', {}).items()},
          d.get('gather_graph'), d.get('gather_chunk_steps'))
PY
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_opt -o run --output-format csv -- \
    python -u bench.py --profile-only --steps 20 --warmup 5 > $OUT/prof_opt.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_multi -o run --output-format csv -- \
    python -u bench.py --workload multi --profile-only --steps 20 --warmup 5 > $OUT/prof_multi.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || exit $?
timeout -k 10 400 python -u bench.py --workload multi --steps 20 --warmup 5 > $OUT/bench20_multi.json 2> $OUT/bench20_multi.err || exit $?
python - $OUT/bench20.json $OUT/bench20_multi.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    r = d['roofline']
    print(f, 'value %.4g' % d['value'], 'us/step %.3f' % (d['ms_per_step'] * 1e3), 'traffic', r.get('traffic'),
          r.get('traffic_source'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))
PY
find $OUT/prof_opt $OUT/prof_multi -name '*kernel_stats.csv' -exec head -3 {} \;
