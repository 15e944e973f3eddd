#!/bin/bash
# The driver's 20-step form under four launch schedules, interleaved reps:
# 20 plain launches (default), LEAD plain launches + a 20 - LEAD step hipGraph
# (CE_MANY_LEAD), and one 20-step hipGraph (CE_MANY_DIRECT=0).  One bench
# process per run (the switches are read at ce_create).  CE_MANY_LEAD was an
# experiment patch of engine.hip, withdrawn after this A/B
# (profiles/r04_ab_lead.txt); without it the lead runs repeat `plain`.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/lead_ab}
mkdir -p $OUT
for rep in 1 2 3; do
  for V in plain lead2 lead4 lead8 graph; do
    case $V in
      plain) ENVS="" ;;
      lead*) ENVS="CE_MANY_LEAD=${V#lead}" ;;
      graph) ENVS="CE_MANY_DIRECT=0" ;;
    esac
    env $ENVS timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/$V.$rep.log 2>&1; rc=$?
    if [ $rc != 0 ]; then echo "$V rc=$rc"; tail -5 $OUT/$V.$rep.log; exit $rc; fi
    python3 -c "import json; d=json.loads([l for l in open('$OUT/$V.$rep.log') if l.startswith('{')][-1]); print('$V', $rep, '%.4f us/step' % (d['ms_per_step']*1e3), '%.4g' % d['value'])"
  done
done
echo ALL_OK
