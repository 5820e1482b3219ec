#!/bin/bash
# HIP validation kernels: numerics vs the fp32 PyTorch reference, then their time under rocprofv3
# (the bench's verification at 64 MiB, and an 8-rank expected-sum fill/verify at 1 GiB).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py tests/test_xgmi_comm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_kernels.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_kernels.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_k -o kern --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kernel_timing.py > $GRAFT_REPO_ROOT/gpurun_out/prof_k.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_k.log; exit 1; }
tail -12 $GRAFT_REPO_ROOT/gpurun_out/prof_k.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_k -name '*kernel_stats*'
