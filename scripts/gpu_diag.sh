#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for E in 1024 4096 16384; do
  for P in f64 f32; do
    CE_LIB=diag timeout -k 10 120 python scripts/diag_phases.py --envs $E --precision $P >> gpurun_out/diag.log 2>&1; rc=$?
    case $rc in 0) ;; *) echo "diag failed rc=$rc"; tail -5 gpurun_out/diag.log; exit $rc;; esac
  done
done
grep envs gpurun_out/diag.log
