#!/bin/bash
# r06a: the MFMA/VALU overlap micro-benchmark, this round's new and changed
# GPU tests, smoke, and a driver-form bench line as the round's baseline.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/r06a}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "GPU step failed (rc=$1), stopping"; exit $1;; esac; }
if [ "${OVERLAP:-0}" = 1 ]; then
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -w scripts/mfma_overlap.hip -o /tmp/mfma_overlap || exit 1
timeout -k 10 120 /tmp/mfma_overlap > $OUT/overlap.jsonl 2>&1; rc=$?
echo "overlap rc=$rc"; fatal $rc
fi
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  tests/test_gpu_persist.py::test_strided_argument_checks tests/test_gpu_persist.py::test_misaligned_obs_is_refused_not_rerouted \
  tests/test_gpu_multi.py::test_config5_global_size_on_one_engine \
  tests/test_gpu_multi.py::test_multi_rollout_argument_checks \
  tests/test_gpu_multinn.py > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; fatal $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-measure-traffic > $OUT/bench20.log 2>&1; rc=$?
echo "bench20 rc=$rc"; tail -1 $OUT/bench20.log | cut -c1-400; fatal $rc
echo ALL_OK
