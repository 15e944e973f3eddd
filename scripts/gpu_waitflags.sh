#!/bin/bash
# The HIP runtime's host-wait settings against the driver form's fixed cost:
# the launch floor and the driver-form bench under each setting (ENVS: a
# list of VAR=VALUE[,VAR=VALUE] settings, "none" = the runtime defaults).
# (ROC_SYSTEM_SCOPE_SIGNAL=0 hung the launch floor in r06o: do not list it.)
set -u
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/waitflags}
mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for rep in 1 2; do
  for setting in ${ENVS:-none}; do
    tag=$(echo $setting | tr ',=' '__')
    if [ "$setting" = none ]; then vars=""; else vars=$(echo $setting | tr ',' ' '); fi
    env $vars timeout -k 10 200 python -u scripts/launch_floor.py --k 1 5 20 40 --repeat 20 > $OUT/floor_${tag}_$rep.json 2>> $OUT/err.log; rc=$?; fatal $rc
    env $vars timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --repeat-timed 10 --no-cpu-baseline --no-measure-traffic > $OUT/bench20_${tag}_$rep.json 2>> $OUT/err.log; rc=$?; fatal $rc
    python3 -c "
import json
f=json.loads(open('$OUT/floor_${tag}_$rep.json').read().strip().splitlines()[-1])
b=json.loads([l for l in open('$OUT/bench20_${tag}_$rep.json') if l.startswith('{')][-1])
print('$tag', $rep, 'empty %.2f' % f['empty_torch_kernel_us'], 'fixed %.2f' % f['after_warmup5']['fixed_us'], 't20 %.2f' % f['after_warmup5']['t_us']['20'], 'bench20 %.4g' % b['value'], 'us/step %.3f' % (b['ms_per_step']*1e3), 'repeats', [round(x*1e3,1) for x in b.get('timed_repeats_ms', [])])"
  done
done
echo ALL_OK
