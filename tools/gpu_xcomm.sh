#!/bin/bash
# Multi-process xGMI all-reduce on the 1-GPU box: GPU tests, then 8 virtual ranks on one GPU.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_xgmi_comm.py tests/test_gpu_ops.py -k "multi_copy or multiprocess" -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/xcomm_pytest.log 2>&1; rc=$?
tail -8 gpurun_out/xcomm_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -m network_operator_amd.parallel.xgmi_comm --world 8 --devices 0,0,0,0,0,0,0,0 \
  --bytes 268435456 --min-bytes 65536 --iters 5 --warmup 2 --timeout 200 > gpurun_out/xcomm_virtual8.json 2> gpurun_out/xcomm_virtual8.err; rc=$?
cat gpurun_out/xcomm_virtual8.json
[ $rc -eq 0 ] || { tail -30 gpurun_out/xcomm_virtual8.err; exit $rc; }
