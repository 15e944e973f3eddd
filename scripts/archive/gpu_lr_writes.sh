#!/bin/bash
# Headline kernel (optimize_lr_mfma_kernel, 4096 envs): WRITE_SIZE / FETCH_SIZE
# per variant (CE_LIB; "main" = the product library), one counter pass each,
# then the interleaved step-time A/B.  OUT names the result directory.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/lrw}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
for V in ${VARIANTS:-main}; do
  if [ $V = main ]; then L=""; else L=$V; fi
  for C in WRITE_SIZE FETCH_SIZE; do
    CE_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/${V}_$C -o run --output-format csv -- python3 bench.py --profile-only --steps 50 --warmup 5 > $OUT/${V}_$C.log 2>&1; rc=$?
    fatal $rc
  done
  python3 - "$OUT" "$V" <<'PY'
import csv, glob, sys
out, v = sys.argv[1], sys.argv[2]
for c in ('WRITE_SIZE', 'FETCH_SIZE'):
    vals = [float(r['Counter_Value']) for f in glob.glob('%s/%s_%s/**/*counter_collection.csv' % (out, v, c), recursive=True)
            for r in csv.DictReader(open(f)) if 'optimize_lr_mfma' in r['Kernel_Name'] and r['Counter_Name'] == c]
    m = sum(vals) / len(vals) * 1024 * (2 if c == 'FETCH_SIZE' else 1)
    print('%s %s %.0f bytes per dispatch (%d dispatches)' % (v, c, m, len(vals)))
PY
done
VARIANTS="${VARIANTS:-main}" OUT=$OUT bash scripts/gpu_ab.sh
