#!/bin/bash
# Issue counters of the headline K-step kernel (optimize_lr_persist_ws_kernel)
# over 250-step dispatches: two --pmc passes (8 SQ counters + GRBM_GUI_ACTIVE,
# then 8 SQ counters), each its own run under a time limit.
# Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's duration;
# MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (128 SIMDs per XCD x GRBM_GUI_ACTIVE).
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc_persist}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
ARGS="--profile-only --steps 2000 --warmup 250"
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY"
i=0
for CTRS in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"; fatal $rc
done
python3 scripts/pmc_generic.py $OUT optimize_lr_persist_ws_kernel $OUT/counters.json > /dev/null || exit 1
python3 - $OUT <<'PY'
import csv, glob, json, sys
d = sys.argv[1]
c = json.load(open(d + '/counters.json'))
durs = []
for p in glob.glob(d + '/p1/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        if 'optimize_lr_persist_ws_kernel' in r['Kernel_Name']:
            durs.append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
durs.sort()
med = durs[len(durs) // 2]
K, E = 250, 4096
row_waves = c['SQ_WAVES'] / 2
out = {
    'kernel': 'optimize_lr_persist_ws_kernel<3,4,false>, 4096 envs, 250-step dispatches',
    'dispatch_median_us': med / 1e3,
    'us_per_step': med / 1e3 / K,
    'clock_ghz': c['GRBM_GUI_ACTIVE'] / 8 / med,
    'mfma_busy_frac': c['SQ_VALU_MFMA_BUSY_CYCLES'] / (128 * c['GRBM_GUI_ACTIVE']),
    'valu_insts_per_wave_step': c['SQ_INSTS_VALU'] / c['SQ_WAVES'] / K,
    'mfma_insts_per_row_wave_step': c['SQ_INSTS_MFMA'] / row_waves / K,
    'lds_insts_per_wave_step': c['SQ_INSTS_LDS'] / c['SQ_WAVES'] / K,
    'salu_insts_per_wave_step': c['SQ_INSTS_SALU'] / c['SQ_WAVES'] / K,
    'lds_bank_conflict_cycles_per_step': c['SQ_LDS_BANK_CONFLICT'] / K,
    'counters_per_dispatch': c,
}
json.dump(out, open(d + '/summary.json', 'w'), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != 'counters_per_dispatch'}, indent=1))
PY
echo ALL_OK
