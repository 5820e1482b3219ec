#!/bin/bash
# Bench at n=1 + rocprofv3 kernel stats of the direct xGMI all-reduce (8 virtual ranks on one GPU).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python3 -c 'import __graft_entry__ as g; g.build()' > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -c 600 gpurun_out/bench.log; echo
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_xa -o xa --output-format csv -- $R/network_operator_amd/_lib/netop-xgmi-allreduce --ranks 8 -b 256M -e 256M -n 5 -w 1 > $R/gpurun_out/prof_xa.log 2>&1 || { tail -20 $R/gpurun_out/prof_xa.log; exit 1; }
cat $R/gpurun_out/prof_xa.log | tail -5
find $R/gpurun_out/prof_xa -name '*kernel_stats*' -exec cat {} \; | cut -c1-220
