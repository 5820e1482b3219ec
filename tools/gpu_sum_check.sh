#!/bin/bash
# After a change to the sum kernel: its numerics and every path that uses it, then its rate.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py tests/test_xgmi_comm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sum.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sum.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/sum_rate_box.py --wg-per-cu 0,4 > gpurun_out/sum_rate.json 2> gpurun_out/sum_rate.err || { tail -20 gpurun_out/sum_rate.err; exit 1; }
cat gpurun_out/sum_rate.json
