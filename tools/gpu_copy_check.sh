#!/bin/bash
# After a change to the copy kernels: the whole GPU suite, then the probe's loopback copy rate.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 network_operator_amd/_lib/netop-xgmi-probe --bytes=1073741824 --iters=20 > gpurun_out/xgmi_probe_1g.json 2>&1 || { cat gpurun_out/xgmi_probe_1g.json; exit 1; }
cat gpurun_out/xgmi_probe_1g.json
