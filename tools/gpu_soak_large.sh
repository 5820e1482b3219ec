#!/bin/bash
# Large-message soaks of both direct all-reduces on the 1-GPU box (the bench's 1 GiB message size):
# 8 virtual ranks, random sizes up to 1 GiB, every call checked exactly.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -m network_operator_amd.parallel.xgmi_comm --world 8 --devices 0,0,0,0,0,0,0,0 \
  --bytes 1073741824 --soak 2000 --timeout 380 > gpurun_out/xcomm_soak_1g.json 2> gpurun_out/xcomm_soak_1g.err; rc=$?
cat gpurun_out/xcomm_soak_1g.json
[ $rc -eq 0 ] || { tail -30 gpurun_out/xcomm_soak_1g.err; exit $rc; }
timeout -k 10 400 network_operator_amd/_lib/netop-xgmi-allreduce --ranks 8 -e 1G --mode both --soak 1000 > gpurun_out/xa_soak_1g.json 2> gpurun_out/xa_soak_1g.err; rc=$?
cat gpurun_out/xa_soak_1g.json
[ $rc -eq 0 ] || { tail -30 gpurun_out/xa_soak_1g.err; exit $rc; }
