#!/bin/bash
# Smoke (GDR/xGMI facts of the box), native RCCL harness in one-process-per-GPU mode (id file),
# and rocprofv3 kernel stats of the harness.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python3 -c 'import __graft_entry__ as g; g.build()' > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
rm -f /tmp/netop-id
timeout -k 10 120 network_operator_amd/_lib/netop-rccl-bench --nranks 1 --rank 0 --device 0 --id-file /tmp/netop-id -b 1M -e 64M -f 8 -n 5 -w 1 > gpurun_out/rccl_mp.jsonl 2> gpurun_out/rccl_mp.txt || { cat gpurun_out/rccl_mp.txt; exit 1; }
cat gpurun_out/rccl_mp.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rccl -o rccl --output-format csv -- $R/network_operator_amd/_lib/netop-rccl-bench -g 1 -b 1G -e 1G -n 10 -w 2 > $R/gpurun_out/prof_rccl.log 2>&1 || { tail -20 $R/gpurun_out/prof_rccl.log; exit 1; }
cut -c1-200 $R/gpurun_out/prof_rccl/rccl_kernel_stats.csv | head -8
