#!/bin/bash
# Effective clock and issue counters of the class-concatenated (mnist image
# shape) kernel, per build in VARIANTS ("main" = the product library): one
# --pmc pass each over 200 back-to-back steps (> 2 s of load).
# Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / the kernel's duration.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/pmc_cat}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for V in ${VARIANTS:-main}; do
  if [ $V = main ]; then L=""; else L=$V; fi
  CE_LIB=$L timeout -s KILL 180 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $OUT/$V/p1 -o run --output-format csv -- python3 bench.py --workload mnist --steps 200 --warmup 5 --no-cpu-baseline > $OUT/$V.log 2>&1; rc=$?
  echo "pmc $V rc=$rc"; fatal $rc
  python3 scripts/pmc_generic.py $OUT/$V optimize_cat_kernel $OUT/$V.json > /dev/null 2>&1 || true
  python3 - $OUT/$V <<'PY'
import csv, glob, json, sys
d = sys.argv[1]
c = json.load(open(d + '.json'))
durs = []
for p in glob.glob(d + '/p1/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        if 'optimize_cat_kernel' in r['Kernel_Name']:
            durs.append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
durs.sort()
med = durs[len(durs) // 2] if durs else float('nan')
print('%s: median kernel %.3f ms, clock %.3f GHz, MFMA busy %.3f of GRBM cycles, VALU insts %.4g, MFMA insts %.4g' % (
    d, med / 1e6, c['GRBM_GUI_ACTIVE'] / 8 / med, c['SQ_VALU_MFMA_BUSY_CYCLES'] / c['GRBM_GUI_ACTIVE'],
    c['SQ_INSTS_VALU'], c['SQ_INSTS_MFMA']))
PY
done
echo ALL_OK
