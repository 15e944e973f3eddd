#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/r2d/avail.txt 2>&1; echo "list rc=$?"
grep -o "SQ_[A-Z0-9_]*" gpurun_out/r2d/avail.txt | sort -u | tr '\n' ' ' | head -c 6000
