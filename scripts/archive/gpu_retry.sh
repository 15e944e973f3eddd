#!/bin/bash
# usage: scripts/gpu_retry.sh OUTFILE TIMEOUT CMD  -- retries only when no box/slot was available
# (exit 3 / transient infrastructure states only; a command that ran and failed is never retried)
out=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" $out && ! grep -q "status=ok" $out; then
    echo "[retry $i rc=$rc]" >> $out.tries; sleep 150; continue
  fi
  break
done
