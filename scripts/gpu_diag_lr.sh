#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2g
export TMPDIR=/tmp
CE_LIB=diag timeout -k 10 200 python scripts/diag_phases.py --steps 30 > gpurun_out/r2g/diag_lr.json 2>&1; rc=$?
cat gpurun_out/r2g/diag_lr.json; exit $rc
