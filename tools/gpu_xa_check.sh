#!/bin/bash
# The direct all-reduces (single process and IPC) and the kernels they use, on virtual ranks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_xgmi_comm.py tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_xa.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_xa.log
exit $rc
