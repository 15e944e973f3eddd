#!/bin/bash
# NN update kernel: envs per block (CE_NN_UPD_ENVS, one row-table read for
# all of them) A/B: the NN tests on the u4 build, then scripts/gpu_nn_ab.sh
# twice, interleaved.  CE_NN_UPD_ENVS was an experiment patch of
# multinn_kernels.h, withdrawn after this A/B (profiles/r04_ab_nn_upd_envs.txt).
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/nnupd
CE_LIB=u4 timeout -k 10 400 python -u -m pytest tests/test_gpu_multinn.py -x -q --timeout 150 --timeout-method thread > gpurun_out/nnupd/pytest.log 2>&1; rc=$?
tail -1 gpurun_out/nnupd/pytest.log; [ $rc = 0 ] || exit $rc
VARIANTS="main u2 u4" bash scripts/gpu_nn_ab.sh && VARIANTS="u4 u2 main" OUT=gpurun_out/nn_ab2 bash scripts/gpu_nn_ab.sh
