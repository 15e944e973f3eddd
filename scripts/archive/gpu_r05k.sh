#!/bin/bash
# Round 5: where the driver form's time goes -- one launch's fixed cost vs
# its per-step slope (launch_floor.py), and the ws kernel's step-1 split
# into row work, barrier wait and epilogue work (diag build).
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05k
mkdir -p $OUT
timeout -k 10 240 python -u scripts/launch_floor.py > $OUT/floor.json 2> $OUT/floor.err || exit $?
cat $OUT/floor.json
CE_LIB=diag timeout -k 10 240 python -u scripts/diag_persist.py --k 20 250 > $OUT/diag_ws.jsonl 2> $OUT/diag_ws.err || exit $?
cat $OUT/diag_ws.jsonl
