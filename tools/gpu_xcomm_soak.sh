#!/bin/bash
# Soak of the direct xGMI all-reduces on the 1-GPU box: the two GPU soak tests, then 8 virtual
# ranks x 20000 calls (random sizes up to 64 MiB, the three algorithms), every call checked exactly.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_xgmi_comm.py -k soak -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/xcomm_soak_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/xcomm_soak_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -m network_operator_amd.parallel.xgmi_comm --world 8 --devices 0,0,0,0,0,0,0,0 \
  --bytes 67108864 --soak 20000 --timeout 380 > gpurun_out/xcomm_soak_virtual8.json 2> gpurun_out/xcomm_soak_virtual8.err; rc=$?
cat gpurun_out/xcomm_soak_virtual8.json
[ $rc -eq 0 ] || { tail -30 gpurun_out/xcomm_soak_virtual8.err; exit $rc; }
# The single-process all-reduce (netop-xgmi-allreduce, what bench.py runs on a whole node): 8 ranks
# on the one GPU, 5000 calls up to 64 MiB, pull and push in turn.
timeout -k 10 400 network_operator_amd/_lib/netop-xgmi-allreduce --ranks 8 -e 64M --mode both --soak 5000 > gpurun_out/xa_soak_virtual8.json 2> gpurun_out/xa_soak_virtual8.err; rc=$?
cat gpurun_out/xa_soak_virtual8.json
[ $rc -eq 0 ] || { tail -30 gpurun_out/xa_soak_virtual8.err; exit $rc; }
