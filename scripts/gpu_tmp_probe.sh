set -u
OUT=gpurun_out/probe; mkdir -p $OUT /tmp/xb
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/boundary_probe.hip -o /tmp/xb/bp 2>/dev/null || exit 1
timeout -k 10 60 /tmp/xb/bp > $OUT/boundary_probe.jsonl 2>&1; rc=$?; cat $OUT/boundary_probe.jsonl; [ $rc = 0 ] || exit $rc
CE_LIB=diag timeout -k 10 120 python scripts/diag_phases.py --envs 4096 > $OUT/diag_lr.json 2>&1; rc=$?; cat $OUT/diag_lr.json; [ $rc = 0 ] || exit $rc
